#!/usr/bin/env python3
"""Phase timestamps of one cs_beam_decode_step launch (diagnostics).

Build here:  python tools/beam_trace.py --build   (a -DCS_TRACE_DECODE copy under tools/)
Run on GPU:  python tools/beam_trace.py           (C1 / C3 / C5 shapes; µs from launch start)"""
import ctypes
import importlib
import json
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
                          ["-DCS_TRACE_DECODE", "-shared", "-o", OUT] + bld.SOURCES)
    sys.exit(0)

_lib = importlib.import_module(PKG + "._lib")
_lib.LIB_NAME = os.path.relpath(OUT, os.path.join(REPO, PKG))
ops = importlib.import_module(PKG + ".ops")
L = _lib.load()
L.cs_trace_read.argtypes = [ctypes.c_void_p]
NAMES = ["start", "last_prop_chunk_start", "last_prop_chunk_published", "last_prop_merge_done",
         "last_row_start", "first_row_lse", "last_row_lse", "last_gather_done", "tail_start",
         "tail_end", "last_prop_keys_ready", "last_prop_cut_done", "first_prop_chunk_published"]
dev = torch.device("cuda:0")
buf = (ctypes.c_ulonglong * 16)()
for name, (A, B, K, V, cap, dt) in {"c1": (4, 4, 10, 128256, 0.0, torch.float32),
                                     "c3": (16, 16, 50, 256000, 30.0, torch.bfloat16),
                                     "c5": (64, 8, 32, 128256, 0.0, torch.bfloat16)}.items():
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(A * B, V, generator=g, device=dev) * 3).to(dt)
    ref = (torch.randn(B, V, generator=g, device=dev) * 3).to(dt)
    R = torch.zeros(A, B, device=dev)
    wd = ops.Workspace(zeroed=True)
    rows = []
    for i in range(6):
        L.cs_trace_read(ctypes.addressof(buf))
        ops.beam_decode_step(ref, x, R, K, "min", n_order=B, softcap=cap, workspace=wd)
        torch.cuda.synchronize()
        L.cs_trace_read(ctypes.addressof(buf))
        t0 = buf[0]
        rows.append({n: round((buf[i] - t0) / 100.0, 2) for i, n in enumerate(NAMES)})  # 100 MHz
    print(json.dumps({"config": name, "us": rows[-1]}), flush=True)
