#!/usr/bin/env python3
"""A/B two builds of the library on the C2 stream (HIP events): python tools/ab_lib.py LIB.so"""
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
_lib = importlib.import_module(PKG + "._lib")
_lib.LIB_NAME = os.path.relpath(os.path.abspath(sys.argv[1]), os.path.join(REPO, PKG))
ops = importlib.import_module(PKG + ".ops")
dev = torch.device("cuda:0")
rows, V = int(sys.argv[2]) if len(sys.argv) > 2 else 76800, 128256
x = torch.empty(rows, V, dtype=torch.bfloat16, device=dev)
g = torch.Generator(device=dev).manual_seed(1)
for r0 in range(0, rows, 4096):
    x[r0:r0 + 4096] = torch.randn(min(4096, rows - r0), V, generator=g, device=dev) * 3
t = torch.randint(0, V, (rows, 1), generator=g, device=dev, dtype=torch.int32)
st = torch.cuda.current_stream()
for _ in range(3):
    ops.logsoftmax_gather(x, t)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
for a, b in ev:
    a.record(st)
    ops.logsoftmax_gather(x, t)
    b.record(st)
torch.cuda.synchronize()
ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
print(json.dumps({"lib": os.path.basename(sys.argv[1]), "rows": rows, "ms": ms,
                  "GBps": rows * V * 2 / (ms * 1e-3) / 1e9}), flush=True)
