#!/usr/bin/env python3
"""cs_beam_decode_step: round-1 grid (CS_DECODE_V2=0) vs v2 (rows first, proposer on the
free slots, rows gathered by the later side of the lse / ids hand-off).  Checks the two
launches give bit-identical outputs on the same inputs, then times both (HIP events, GPU
kept busy) and the v2 grid knobs.  python tools/decode_v2_ab.py [--only c3,c5] [--sweep]"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
if "--lib" in sys.argv:   # A/B another build of the library: --lib path/to/lib.so
    _lib = importlib.import_module(PKG + "._lib")
    _lib.LIB_NAME = os.path.relpath(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]),
                                    os.path.join(REPO, PKG))
ops = importlib.import_module(PKG + ".ops")
from beam_ab import timed  # noqa: E402

CASES = {"c1": (4, 4, 10, 128256, 0.0, torch.float32),
         "c3": (16, 16, 50, 256000, 30.0, torch.bfloat16),
         "c3nocap": (16, 16, 50, 256000, 0.0, torch.bfloat16),
         "c5": (64, 8, 32, 128256, 0.0, torch.bfloat16),
         "odd": (5, 3, 7, 5003, 0.0, torch.float16),
         "wide": (3, 64, 16, 32000, 0.0, torch.bfloat16)}


def run(ref, x, R, K, B, cap, ws):
    kept = torch.empty(R.shape[0], B, device=x.device)
    ids, U, W, order, oval = ops.beam_decode_step(ref, x, R, K, "min", n_order=B, softcap=cap,
                                                  workspace=ws, kept_out=kept)
    return [ids, U, W, order, oval, kept]


def same(a, b):
    return all(torch.equal(torch.nan_to_num(p.float(), nan=7.0), torch.nan_to_num(q.float(), nan=7.0))
               for p, q in zip(a, b))


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    for name, (A, B, K, V, cap, dt) in CASES.items():
        if only and name not in only:
            continue
        g = torch.Generator(device=dev).manual_seed(7)
        x = (torch.randn(A * B, V, generator=g, device=dev) * 3).to(dt)
        ref = (torch.randn(B, V, generator=g, device=dev) * 3).to(dt)
        R = -torch.rand(A, B, generator=g, device=dev) * 5
        ws = ops.Workspace(zeroed=True)
        r = {"config": name, "lib": sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else "tree"}
        os.environ["CS_DECODE_V2"] = "0"
        o1 = run(ref, x, R, K, B, cap, ws)
        os.environ["CS_DECODE_V2"] = "1"
        o2 = run(ref, x, R, K, B, cap, ws)
        o3 = run(ref, x, R, K, B, cap, ws)
        torch.cuda.synchronize()
        r["v2_equals_v1"] = same(o1, o2)
        r["v2_repeatable"] = same(o2, o3)
        os.environ["CS_DECODE_V2"] = "0"
        r["v1_us"] = timed(lambda: run(ref, x, R, K, B, cap, ws))
        os.environ["CS_DECODE_V2"] = "1"
        r["v2_us"] = timed(lambda: run(ref, x, R, K, B, cap, ws))
        if "--sweep" in sys.argv:
            for p0, pw in (("0", None), (None, "64"), (None, "128"), ("0", "64"), ("0", "128")):
                for k, v in (("CS_DECODE_P0", p0), ("CS_DECODE_PW", pw)):
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
                o4 = run(ref, x, R, K, B, cap, ws)
                r[f"v2_p0{p0}_pw{pw}_us"] = timed(lambda: run(ref, x, R, K, B, cap, ws))
                r[f"v2_p0{p0}_pw{pw}_same"] = same(o1, o4)
            os.environ.pop("CS_DECODE_P0", None)
            os.environ.pop("CS_DECODE_PW", None)
        r["bytes"] = (A * B + B) * V * x.element_size()
        r["v2_frac_8tbs"] = r["bytes"] / (r["v2_us"] * 1e-6) / 8e12
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
