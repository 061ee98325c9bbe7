#!/usr/bin/env python3
"""Fixed cost vs bandwidth of the vocab stream: lse-only cs_logsoftmax_gather over
256..4096 rows of 256,000 bf16 (HIP events, GPU kept busy), fitted t = t0 + bytes / bw."""
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")
from beam_ab import timed  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
V = 256000
caps = (0.0, 30.0)
pts = {c: [] for c in caps}
big = (torch.randn(4096, V, device=dev) * 3).to(torch.bfloat16)
ws = ops.Workspace()
for rows in (64, 128, 256, 512, 1024, 2048, 4096):
    x = big[:rows]
    for cap in caps:
        us = timed(lambda: ops.logsoftmax_gather(x, None, softcap=cap, workspace=ws, want_lse=True))
        pts[cap].append((rows * V * 2, us))
        print(json.dumps({"rows": rows, "cap": cap, "MB": rows * V * 2 / 1e6, "us": us,
                          "TBps": rows * V * 2 / us / 1e6}), flush=True)
for cap in caps:
    b = np.array([p[0] for p in pts[cap][2:]], dtype=np.float64)
    t = np.array([p[1] for p in pts[cap][2:]])
    slope, t0 = np.polyfit(b, t, 1)
    print(json.dumps({"fit_cap": cap, "t0_us": t0, "bw_TBps": 1 / slope / 1e6}), flush=True)
