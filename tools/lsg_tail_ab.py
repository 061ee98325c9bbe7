#!/usr/bin/env python3
"""What the per-row target gather costs the C2 logits stream: cs_logsoftmax_gather on the
bench's 76,800 x 128,256 bf16 rows with one target per row (the product) against the
same launch with no targets (lse only), alternated in one process, HIP events.

    python tools/lsg_tail_ab.py [rows] [vocab] [rounds]
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


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 76800
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 128256
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.empty(rows, V, dtype=torch.bfloat16, device=dev)
    for r0 in range(0, rows, 4096):
        r1 = min(rows, r0 + 4096)
        x[r0:r1] = torch.randn(r1 - r0, V, generator=g, device=dev) * 3.0
    t = torch.randint(0, V, (rows, 1), generator=g, device=dev, dtype=torch.int32)
    lse = torch.empty(rows, dtype=torch.float32, device=dev)
    out = torch.empty(rows, 1, dtype=torch.float32, device=dev)
    ws = ops.Workspace()
    forms = {"k1": lambda: ops.logsoftmax_gather(x, t, out=out, workspace=ws),
             "k1_lse": lambda: ops.logsoftmax_gather(x, t, out=out, lse_out=lse, workspace=ws),
             "lse_only": lambda: ops.logsoftmax_gather(x, None, lse_out=lse, workspace=ws)}
    ts = {k: [] for k in forms}
    for r in range(rounds + 1):
        for k, fn in forms.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            torch.cuda.synchronize()
            if r > 0:
                ts[k].append(e0.elapsed_time(e1) / 5)
    nbytes = rows * V * 2
    for k, v in ts.items():
        v.sort()
        med = v[len(v) // 2]
        print(json.dumps({"form": k, "rows": rows, "vocab": V, "median_ms": round(med, 4),
                          "min_ms": round(v[0], 4), "frac_8TBs": round(nbytes / (med * 1e-3) / 8e12, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
