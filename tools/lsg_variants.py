#!/usr/bin/env python3
"""A/B of the compiled cs_logsoftmax_gather variants (CS_LSG_VARIANT, read once per
process by the library) on the bench's own data (torch randn*3 -> bf16): one child process
per variant, each printing its timing and a checksum of its output.

    python tools/lsg_variants.py [rows] [vocab] [rounds]
"""
import importlib
import json
import os
import subprocess
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")

NAMES = {0: "auto", 5: "b256_u4", 1: "b512_u4", 2: "b1024_u1", 3: "b1024_u2", 4: "b256_u8",
         6: "b1024_u4", 7: "b512_u8"}


def child(v):
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
    ts = []
    for r in range(rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            tok, _ = ops.logsoftmax_gather(x, t, workspace=ws)
        e1.record()
        torch.cuda.synchronize()
        if r > 0:
            ts.append(e0.elapsed_time(e1) / 5)
    nbytes = rows * V * 2 + rows * 8
    ts.sort()
    med = ts[len(ts) // 2]
    print(json.dumps({"variant": NAMES[v], "rows": rows, "vocab": V, "median_ms": med,
                      "min_ms": ts[0], "GBps": nbytes / (med * 1e-3) / 1e9,
                      "frac_8TBs": nbytes / (med * 1e-3) / 8e12,
                      "checksum": float(tok.double().sum())}), flush=True)


def main():
    if "CS_LSG_VARIANT" in os.environ:
        child(int(os.environ["CS_LSG_VARIANT"]))
        return
    for v in NAMES:
        env = dict(os.environ, CS_LSG_VARIANT=str(v))
        subprocess.run([sys.executable, os.path.abspath(__file__)] + sys.argv[1:4], env=env,
                       check=True)


if __name__ == "__main__":
    main()
