#!/usr/bin/env python3
"""Run only the beam-search decode-step benchmark of bench.py (for rocprofv3 runs)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--beam", default="c1,c3,c5")
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
for name in a.beam.split(","):
    r = bench.run_beam(name, 1, 0, dev, a.steps, 20)
    print(json.dumps({name: r}), flush=True)
