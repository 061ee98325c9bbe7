"""A/B of cs_hist_gather builds on the beam-reorder shapes of a C3 / C5 decode step:
python tools/hist_gather_ab.py --lib ablibs/X.so.  One JSON line per (config, filled slots):
us per launch (HIP events, mean of 20) and the copy's HBM rate (bytes read + written)."""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else ""
if lib:
    _l = importlib.import_module(PKG + "._lib")
    _l.LIB_NAME = os.path.relpath(os.path.abspath(lib), os.path.join(REPO, PKG))
ops = importlib.import_module(PKG + ".ops")
dev = torch.device("cuda:0")
# (config, layers, streams, kv heads, slots, head dim)
for name, L, S, Hkv, ldh, D in [("c3", 42, 272, 8, 64, 256), ("c5", 80, 520, 8, 64, 128)]:
    sk = torch.randn(L, S, Hkv, ldh, D, device=dev).to(torch.bfloat16)
    sv = torch.randn(L, S, Hkv, ldh // 32, D, 32, device=dev).to(torch.bfloat16)
    dk, dv = torch.zeros_like(sk), torch.zeros_like(sv)
    parent = torch.randint(0, S, (S,), device=dev)
    for hb in (9, 25, 49):
        base = torch.tensor([hb], dtype=torch.int32, device=dev)
        for _ in range(3):
            ops.hist_gather(sk, dk, sv, dv, parent, base)
        torch.cuda.synchronize()
        e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in e:
            a.record()
            ops.hist_gather(sk, dk, sv, dv, parent, base)
            b.record()
        torch.cuda.synchronize()
        us = sum(a.elapsed_time(b) for a, b in e) / len(e) * 1e3
        vslots = (hb // 32) * 32 + ((hb % 32) + 7) // 8 * 8
        nbytes = 2 * L * S * Hkv * D * (hb + vslots) * 2          # read + write, K and V
        sig = int(dk.view(torch.int16).sum().item()) ^ int(dv.view(torch.int16).sum().item())
        print(json.dumps({"lib": os.path.basename(lib) or "tree", "config": name, "hb": hb,
                          "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 3), "sig": sig}),
              flush=True)
    del sk, sv, dk, dv
