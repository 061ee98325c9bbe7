"""cs_prefix_attention at the method shapes (HIP-event timing, no model): decode steps of
BASELINE C1 / C3 / C5 (history G slots, BPE-length agent prompts, the long reference
prompt) and the C2 scoring chunk.  Prints one JSON line per shape: us per launch (kernel +
merge) and the K/V bytes the launch must read (prefix once per (agent, head) + every
stream's history).

    python tools/attn_bench.py
"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
LIB = None
if "--lib" in sys.argv:   # A/B another build of the library: --lib path/to/lib.so
    i = sys.argv.index("--lib")
    LIB = sys.argv[i + 1]
    del sys.argv[i:i + 2]
    _lib = importlib.import_module(PKG + "._lib")
    _lib.LIB_NAME = os.path.relpath(os.path.abspath(LIB), os.path.join(REPO, PKG))

SHAPES = {
    # name: (n agent prefixes, agent len, ref len, n_str, T, H, Hkv, D, hist G, softcap)
    "c1": (4, 210, 600, 4, 1, 32, 8, 64, 25, 0.0),
    "c3": (16, 210, 1700, 16, 1, 16, 8, 256, 25, 50.0),
    "c5": (64, 210, 5500, 8, 1, 64, 8, 128, 25, 0.0),
    "c2": (8, 200, None, 64, 149, 32, 8, 128, 0, 0.0),
    # one rank of eight (agents sharded): the per-rank decode shapes
    "c3r8": (2, 210, 1700, 16, 1, 16, 8, 256, 25, 50.0),
    "c5r8": (8, 210, 5500, 8, 1, 64, 8, 128, 25, 0.0),
}


def ceil32(n):
    return max(32, (n + 31) // 32 * 32)


def run(name, reps=50):
    ops = importlib.import_module(PKG + ".ops")
    if "=" in name:     # ad-hoc shape: name=nA,La,Lr,n_str,T,H,Hkv,D,G,cap (Lr 0: none)
        name, spec = name.split("=", 1)
        v = [float(x) for x in spec.split(",")]
        SHAPES[name] = tuple(int(x) for x in v[:9]) + (v[9],)
        if not SHAPES[name][2]:
            SHAPES[name] = SHAPES[name][:2] + (None,) + SHAPES[name][3:]
    nA, La, Lr, n_str, T, H, Hkv, D, G, cap = SHAPES[name]
    dev = torch.device("cuda:0")
    lens = [La] * nA + ([Lr] if Lr else [])
    n_grp = len(lens)
    off, o = [], 0
    for n in lens:
        off.append(o)
        o += ceil32(n)
    bf = torch.bfloat16
    kp = torch.randn(Hkv, o, D, device=dev).to(bf)
    vt = torch.randn(Hkv, o // 32, D, 32, device=dev).to(bf)
    S = n_grp * n_str
    ldh = ceil32(G + T)
    kh = torch.randn(S, Hkv, ldh, D, device=dev).to(bf)
    vh = torch.randn(S, Hkv, ldh // 32, D, 32, device=dev).to(bf)
    q = torch.randn(S * T, H, D, device=dev).to(bf)
    plen = torch.tensor(lens, dtype=torch.int32, device=dev)
    offt = torch.tensor(off, dtype=torch.int64, device=dev)
    hb = torch.tensor([G], dtype=torch.int32, device=dev)
    out = torch.empty_like(q)

    def go():
        ops.prefix_attention(q, kp, vt, offt, plen, max(lens), kh, vh, hb, n_str, T,
                             scale=D ** -0.5, softcap=cap, out=out, prefix_len_host=lens)

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
    kv_bytes = 2 * Hkv * sum(lens) * D * 2 + 2 * S * Hkv * (G + T) * D * 2
    flops = 4 * S * T * H * D * (sum(lens) / n_grp + G + T / 2)
    print(json.dumps({"shape": name, "lib": LIB or "tree", "us": us, "kv_bytes": kv_bytes,
                      "gb_per_s": kv_bytes / us / 1e3, "tflops": flops / us / 1e6}), flush=True)


if __name__ == "__main__":
    for n in (sys.argv[1:] or SHAPES):
        run(n)
