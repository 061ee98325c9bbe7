#!/usr/bin/env python3
"""cs_gated_act alone at the C2 pass's shape (76,800 x 14,336 of a 28,672-wide gate|up
product), HIP events: python tools/act_ab.py [LIB.so] (another build of the library)."""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
_lib = importlib.import_module(PKG + "._lib")
if len(sys.argv) > 1:
    _lib.LIB_NAME = os.path.relpath(os.path.abspath(sys.argv[1]), os.path.join(REPO, PKG))
ops = importlib.import_module(PKG + ".ops")
dev = torch.device("cuda:0")
M, F = 76800, 14336
gu = torch.randn(M, 2 * F, device=dev, dtype=torch.bfloat16)
out = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
ts = []
for r in range(8):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.gated_act(gu[:, :F], gu[:, F:], "silu", out=out)
    e1.record()
    torch.cuda.synchronize()
    if r:
        ts.append(e0.elapsed_time(e1) / 5)
ts.sort()
med = ts[len(ts) // 2]
print(json.dumps({"lib": sys.argv[1] if len(sys.argv) > 1 else "tree", "ms": round(med, 4),
                  "TBps": round(M * F * 6 / (med * 1e-3) / 1e12, 3)}), flush=True)
