#!/usr/bin/env python3
"""cs_segmented_topk latency (HIP events, GPU kept busy) on the shapes the methods use:
python tools/topk_time.py  ->  one JSON line per (n_seg, seg_len, k)."""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")
from beam_ab import timed  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
for n_seg, seg_len, k in ((1, 64, 1), (1, 256, 1), (1, 800, 16), (1, 1024, 256), (8, 4096, 64),
                          (1, 16384, 32), (1, 800, 800)):
    W = torch.randn(n_seg, seg_len, device=dev)
    us = timed(lambda: ops.topk(W, k), n=40)
    print(json.dumps({"n_seg": n_seg, "seg_len": seg_len, "k": k, "us": round(us, 2),
                      "path": "select" if k <= 256 and seg_len > 64 else "bitonic"}), flush=True)
