#!/usr/bin/env python3
"""cs_rope_place at the C2 scoring-chunk shape (8 agents x 64 candidate streams x 150
tokens, Llama-3.1-8B heads) and a decode step (C5: 520 streams x 1 token): HIP-event us per
launch and the bytes it must move (qkv read + q / k / v written).

    CS_ROPE_VTILE=0|1 python tools/rope_bench.py
"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"

SHAPES = {  # name: (groups, streams per group, T, H, Hkv, D)
    "c2": (8, 64, 150, 32, 8, 128),
    "c5": (65, 8, 1, 64, 8, 128),
}


def run(name, reps=50):
    ops = importlib.import_module(PKG + ".ops")
    G, n_str, T, H, Hkv, D = SHAPES[name]
    dev = torch.device("cuda:0")
    S = G * n_str
    n = S * T
    ldh = max(32, (T + 31) // 32 * 32)
    bf = torch.bfloat16
    qkv = torch.randn(n, (H + 2 * Hkv) * D, device=dev).to(bf)
    inv_freq = 1.0 / (500000.0 ** (torch.arange(0, D, 2, device=dev).float() / D))
    plen = torch.full((G,), 200, dtype=torch.int32, device=dev)
    hb = torch.zeros(1, dtype=torch.int32, device=dev)
    q_out = torch.empty(n, H, D, device=dev, dtype=bf)
    kh = torch.zeros(S, Hkv, ldh, D, device=dev, dtype=bf)
    vh = torch.zeros(S, Hkv, ldh // 32, D, 32, device=dev, dtype=bf)

    def go():
        ops.rope_place(qkv, inv_freq, plen, hb, n_str, T, H, Hkv, D, q_out, kh, vh)

    for _ in range(5):
        go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nbytes = 2 * n * (H + 2 * Hkv) * D * 2
    print(json.dumps({"shape": name, "vtile_env": os.environ.get("CS_ROPE_VTILE", "default"),
                      "us": us, "bytes": nbytes, "gb_per_s": nbytes / us / 1e3}), flush=True)


if __name__ == "__main__":
    for s in (sys.argv[1:] or SHAPES):
        run(s)
