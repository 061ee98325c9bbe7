#!/usr/bin/env python3
"""Phase timestamps of cs_beam_step's last workgroup (diagnostics): builds a -DCS_TRACE_BEAM
copy of the library under tools/ (build it here: python tools/beam_trace.py --build), then on
the GPU runs a few beam steps per config; the kernel printf()s wall-clock deltas (10 ns)."""
import importlib
import os
import subprocess
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
OUT = os.path.join(REPO, "tools", "libcs_trace.so")

if "--build" in sys.argv:
    bld = importlib.import_module(PKG + ".build")
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + bld._flags() +
                          ["-DCS_TRACE_DECODE", "-DCS_TRACE_TOPK", "-shared", "-o", OUT] + bld.SOURCES)
    sys.exit(0)

_lib = importlib.import_module(PKG + "._lib")
_lib.LIB_NAME = os.path.relpath(OUT, os.path.join(REPO, PKG))
ops = importlib.import_module(PKG + ".ops")
dev = torch.device("cuda:0")
for name, (A, B, K, V, cap, dt) in {"c1": (4, 4, 10, 128256, 0.0, torch.float32),
                                     "c3": (16, 16, 50, 256000, 30.0, torch.bfloat16),
                                     "c5": (64, 8, 32, 128256, 0.0, torch.bfloat16)}.items():
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(A * B, V, generator=g, device=dev) * 3).to(dt)
    t = torch.randint(0, V, (B, K), generator=g, device=dev, dtype=torch.int32)
    R = torch.zeros(A, B, device=dev)
    wb = ops.Workspace(zeroed=True)
    for i in range(4):
        ops.beam_step(x, t, R, "min", softcap=cap, workspace=wb)
        torch.cuda.synchronize()
    ref = (torch.randn(B, V, generator=g, device=dev) * 3).to(dt)
    for i in range(3):
        ops.beam_decode_step(ref, x, R, K, "min", n_order=B, softcap=cap)
        torch.cuda.synchronize()
    print(name, "done", flush=True)
