#!/usr/bin/env python3
"""Stream rate vs launch size at V = 128,256 bf16 (the C2 / C4 vocabulary): per-launch
time of cs_logsoftmax_gather (k = 1) next to the pure-read kernel (tools/read_floor.hip,
one workgroup per row-sized slice) over the same bytes, HIP events, GPU kept busy.
python tools/read_floor.py --build here, then on the GPU box: python tools/size_sweep.py"""
import ctypes
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
if os.environ.get("SWEEP_LIB"):   # time another build of the library
    _lib = importlib.import_module(
        "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd._lib")
    _lib.LIB_NAME = os.path.relpath(os.path.abspath(os.environ["SWEEP_LIB"]), os.path.join(
        REPO, "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"))
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")
from beam_ab import timed  # noqa: E402

lib = ctypes.CDLL(os.path.join(REPO, "tools", "libread_floor.so"))
lib.rf_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                        ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
V = 128256
ROWS = [int(r) for r in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
    [2048, 4096, 8192, 10880, 16384, 32768, 65536, 76800, 131072]
x = torch.empty(max(ROWS), V, dtype=torch.bfloat16, device=dev)
g = torch.Generator(device=dev).manual_seed(1)
for r0 in range(0, x.shape[0], 4096):
    x[r0:r0 + 4096] = torch.randn(min(4096, x.shape[0] - r0), V, generator=g, device=dev) * 3
t = torch.randint(0, V, (x.shape[0], 1), generator=g, device=dev, dtype=torch.int32)
out = torch.zeros(4, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
REP = int(os.environ.get("SWEEP_REP", "1"))
for rows in ROWS:
    nbytes = rows * V * 2
    lsg, lsg0, rd = [], [], {"1024x2": [], "1024x4": []}
    for _ in range(REP):   # interleaved repeats: box drift hits both kernels alike
        lsg.append(timed(lambda: ops.logsoftmax_gather(x[:rows], t[:rows]), n=10))
        lsg0.append(timed(lambda: ops.logsoftmax_gather(x[:rows], None, want_lse=True), n=10))
        for block, unroll in ((1024, 2), (1024, 4)):
            rd[f"{block}x{unroll}"].append(timed(lambda: lib.rf_read(
                x.data_ptr(), nbytes, rows, block, unroll, out.data_ptr(), st), n=10))
    us = min(lsg)
    rd = {k: min(v) for k, v in rd.items()}
    print(json.dumps({"rows": rows, "GB": nbytes / 1e9, "lsg_us": round(us, 1),
                      "lsg_TBps": round(nbytes / us / 1e6, 3),
                      "lse_only_us": round(min(lsg0), 1),
                      "read_us": {k: round(v, 1) for k, v in rd.items()},
                      "read_TBps": {k: round(nbytes / v / 1e6, 3) for k, v in rd.items()}}),
          flush=True)
