#!/usr/bin/env python3
"""In-process A/B of the compiled cs_logsoftmax_gather variants (CS_LSG_VARIANT) on the
bench's own data (torch randn*3 -> bf16), interleaved round by round.

    python tools/lsg_variants.py [rows] [vocab] [rounds]
"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")

NAMES = {0: "auto", 5: "b256_u4", 1: "b512_u4", 2: "b1024_u1", 3: "b1024_u2", 4: "b256_u8",
         6: "b1024_u4", 7: "b512_u8"}


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 76800
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 128256
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.empty(rows, V, dtype=torch.bfloat16, device=dev)
    for r0 in range(0, rows, 4096):
        r1 = min(rows, r0 + 4096)
        x[r0:r1] = torch.randn(r1 - r0, V, generator=g, device=dev) * 3.0
    t = torch.randint(0, V, (rows, 1), generator=g, device=dev, dtype=torch.int32)
    ws = ops.Workspace()
    times = {v: [] for v in NAMES}
    ref = None
    outs = {}
    for r in range(rounds + 1):
        for v in NAMES:
            os.environ["CS_LSG_VARIANT"] = str(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                tok, _ = ops.logsoftmax_gather(x, t, workspace=ws)
            e1.record()
            torch.cuda.synchronize()
            if r > 0:
                times[v].append(e0.elapsed_time(e1) / 5)
            outs[v] = tok
    os.environ.pop("CS_LSG_VARIANT")
    nbytes = rows * V * 2 + rows * 8
    for v, ts in times.items():
        ts.sort()
        med = ts[len(ts) // 2]
        print(json.dumps({"variant": NAMES[v], "rows": rows, "vocab": V, "median_ms": med,
                          "min_ms": ts[0], "GBps": nbytes / (med * 1e-3) / 1e9,
                          "frac_8TBs": nbytes / (med * 1e-3) / 8e12,
                          "max_abs_diff_vs_auto": float((outs[v] - outs[0]).abs().max())}))


if __name__ == "__main__":
    main()
