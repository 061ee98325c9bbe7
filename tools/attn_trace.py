"""Phase timestamps of one decode-step cs_prefix_attention launch (diagnostics build).

    python tools/build_alt.py /tmp/libattn_trace.so -DCS_TRACE_ATTN=1
    python tools/attn_trace.py /tmp/libattn_trace.so c3r8=2,210,1700,16,1,16,8,256,25,50 ...

Shapes as tools/attn_bench.py.  Prints, per shape and phase, [min, median, max] over the
workgroups of wall_clock64 stamps in microseconds from the first attention workgroup's start
(csrc/attn.hip CS_TRACE_ATTN): start, prologue loads in, prefix loop done, history loop done,
partial stored; merge workgroups' start and end.
"""
import ctypes
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
LIB = os.path.abspath(sys.argv[1])
_lib = importlib.import_module(PKG + "._lib")
_lib.LIB_NAME = os.path.relpath(LIB, os.path.join(REPO, PKG))
import attn_bench  # noqa: E402

NAMES = ["start", "prologue", "prefix_done", "hist_done", "stored", "merge_start", "merge_done"]
NWG = 4096


def main():
    ops = importlib.import_module(PKG + ".ops")
    L = _lib.load()
    L.cs_attn_trace_read.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * (NWG * 8))()
    captured = {}

    orig = ops.prefix_attention

    def once(*a, **k):
        captured["call"] = (a, k)
        return orig(*a, **k)

    for spec in sys.argv[2:]:
        ops.prefix_attention = once
        attn_bench.run(spec, reps=5)
        ops.prefix_attention = orig
        a, k = captured["call"]
        for _ in range(3):
            orig(*a, **k)
        torch.cuda.synchronize()
        L.cs_attn_trace_read(buf)
        orig(*a, **k)
        torch.cuda.synchronize()
        L.cs_attn_trace_read(buf)
        import numpy as np
        ts = np.frombuffer(buf, dtype=np.uint64).reshape(NWG, 8).astype(np.int64)
        att = ts[:, 0] > 0
        t0 = ts[att, 0].min()
        rec = {"shape": spec.split("=")[0], "attn_wgs": int(att.sum())}
        for i, n in enumerate(NAMES):
            col = ts[:, i]
            v = col[col > 0]
            if v.size:
                q = (v - t0) * 0.01
                rec[n] = [round(float(q.min()), 2), round(float(np.median(q)), 2),
                          round(float(q.max()), 2)]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
