#!/usr/bin/env python3
"""Pure-read floor of the MI355X for the beam-shape stream sizes (python tools/read_floor.py
--build here, then on the GPU box without --build): grid x block x unroll sweep per size."""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libread_floor.so")
if "--build" in sys.argv:
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared",
                           os.path.join(HERE, "read_floor.hip"), "-o", SO])
    sys.exit(0)
sys.path.insert(0, HERE)
from beam_ab import timed  # noqa: E402

lib = ctypes.CDLL(SO)
lib.rf_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                        ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
buf = torch.randint(0, 2**31 - 1, (2 * 2**30 // 4,), dtype=torch.int32, device=dev)
out = torch.zeros(4, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
for mb in (32.768, 65.536, 131.072, 262.144, 1048.576):
    nbytes = int(mb * 1e6)
    best = None
    for wgs in (256, 512, 1024, 2048, 4096, 8192):
        for block in (256, 512, 1024):
            for unroll in (2, 4, 8):
                us = timed(lambda: lib.rf_read(buf.data_ptr(), nbytes, wgs, block, unroll,
                                               out.data_ptr(), st), n=20)
                r = {"MB": mb, "wgs": wgs, "block": block, "unroll": unroll, "us": round(us, 2),
                     "TBps": round(nbytes / us / 1e6, 3)}
                if best is None or us < best["us"]:
                    best = r
                if "-v" in sys.argv:
                    print(json.dumps(r), flush=True)
    print(json.dumps({"best": best}), flush=True)
