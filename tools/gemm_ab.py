"""A/B of the decode-step projection GEMMs: cs_gemm_bf16 (csrc/gemm.hip) against torch
(hipBLASLt / rocBLAS with the committed TunableOp selection) on the C1 / C3 / C5 step shapes,
weights STREAMED from HBM as in a step (distinct matrices rotated past the 256 MB Infinity
Cache), both captured in one hipGraph of 20 calls; plus a max-error check against an fp32
product.  One JSON line per (shape, variant).

    python tools/gemm_ab.py [--shapes c3] [--splits 0,1,2,4]
"""
import argparse
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
if "--lib" in sys.argv:         # an A/B build (tools/build_alt.py) instead of the tree's library
    _l = importlib.import_module(PKG + "._lib")
    _l.LIB_NAME = os.path.relpath(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]),
                                  os.path.join(REPO, PKG))
R = importlib.import_module(PKG + ".runtime")
ops = importlib.import_module(PKG + ".ops")

SHAPES = {
    # name: (M, N, K, gated)
    "c1_qkv": (20, 3072, 2048, 0), "c1_o": (20, 2048, 2048, 0), "c1_gu": (20, 16384, 2048, 0),
    "c1_gu_gated": (20, 16384, 2048, 1), "c1_down": (20, 2048, 8192, 0),
    "c1_lmhead": (20, 128256, 2048, 0), "c3_lmhead": (272, 256000, 3584, 0),
    "c5_lmhead": (520, 128256, 8192, 0),
    "c3_qkv": (272, 8192, 3584, 0), "c3_o": (272, 3584, 4096, 0), "c3_gu": (272, 28672, 3584, 0),
    "c3_gu_gated": (272, 28672, 3584, 1), "c3_down": (272, 3584, 14336, 0),
    "c5_qkv": (520, 10240, 8192, 0), "c5_o": (520, 8192, 8192, 0), "c5_gu": (520, 57344, 8192, 0),
    "c5_gu_gated": (520, 57344, 8192, 1), "c5_down": (520, 8192, 28672, 0),
    # agent-sharded step shapes (8 ranks: C3 3 x 16 rows, C5 9 x 8 rows)
    "r8c3_qkv": (48, 8192, 3584, 0), "r8c3_gu_gated": (48, 28672, 3584, 1),
    "r8c3_down": (48, 3584, 14336, 0), "r8c5_qkv": (72, 10240, 8192, 0),
    "r8c5_gu_gated": (72, 57344, 8192, 1), "r8c5_down": (72, 8192, 28672, 0),
    "r8c3_o": (48, 3584, 4096, 0), "r8c5_o": (72, 8192, 8192, 0),
    "r8c3_lmhead": (48, 256000, 3584, 0), "r8c5_lmhead": (72, 128256, 8192, 0),
}


def timed(fn, reps=5):
    fn()                      # eager warm-up: library handles / tuned solutions outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="c1,c3,c5")
    ap.add_argument("--splits", default="0")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--msweep", default="", help="torch only: comma list of M for the C3 shapes")
    ap.add_argument("--lib", default="", help="time this build of the library (read before import)")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--packed", action="store_true",
                    help="also time cs_gemm_bf16_packed on cs_gemm_pack'ed copies of the weights")
    ap.add_argument("--warm", action="store_true",
                    help="one weight matrix for every call (L2 / Infinity-Cache resident when it "
                         "fits): the rate the kernel reaches when HBM is not what bounds it")
    args = ap.parse_args()
    print("tuning:", R.use_gemm_tuning(), file=sys.stderr)
    dev = torch.device("cuda:0")
    pre = tuple(args.shapes.split(","))
    if args.msweep:
        for M in [int(v) for v in args.msweep.split(",")]:
            for name, (N, K) in {"gu": (28672, 3584), "down": (3584, 14336), "qkv": (8192, 3584),
                                 "o": (3584, 4096)}.items():
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                nw = max(2, min(20, (700 << 20) // (N * K * 2) + 1))
                ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nw)]
                t = timed(lambda: [x @ ws[i % nw].t() for i in range(20)]) / 20 * 1e3
                print(json.dumps({"shape": "c3_" + name, "M": M, "impl": "torch", "us": round(t, 2),
                                  "weight_GBps": round(N * K * 2 / t / 1e3, 1)}), flush=True)
                del ws
        return
    for name, (M, N, K, gated) in SHAPES.items():
        if not name.startswith(pre):
            continue
        torch.manual_seed(0)
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        nw = 1 if args.warm else max(2, min(20, (700 << 20) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05 for _ in range(nw)]
        calls = 20
        # correctness on ws[0]
        ref = x.float() @ ws[0].float().t()
        if gated:
            F = N // 2
            g = ref[:, :F].to(torch.bfloat16)
            u = ref[:, F:].to(torch.bfloat16)
            ref = ops.gated_act(g, u, "silu").float()
        for var, sp in [(int(v), int(s)) for v in args.variants.split(",")
                        for s in args.splits.split(",")]:
            if gated and sp > 1:
                continue
            y = ops.gemm(x, ws[0], gated=bool(gated), splits=sp, variant=var)
            torch.cuda.synchronize()
            err = (y.float() - ref).abs().max().item()
            scale = ref.abs().max().item()
            t = timed(lambda: [ops.gemm(x, ws[i % nw], gated=bool(gated), splits=sp, variant=var)
                               for i in range(calls)]) / calls * 1e3
            eff = ("sk" if sp < 0 else
                   int(ops._lib.load().cs_gemm_splits(M, N, K, gated, var)) if sp == 0 else sp)
            yb = y.contiguous().view(torch.int16).to(torch.int64)
            ysig = int(((yb * torch.arange(1, yb.numel() + 1, device=dev).view_as(yb)) % 1000003).sum().item())
            rec = {"lib": os.path.basename(args.lib) or "tree", "ysig": ysig, "warm": args.warm,
                   "shape": name, "M": M, "N": N, "K": K, "impl": f"cs_gemm_v{var}", "splits": eff,
                   "us": round(t, 2), "weight_GBps": round(N * K * 2 / t / 1e3, 1),
                   "TFLOPs": round(2 * M * N * K / t / 1e6, 1), "max_err": err, "ref_max": scale}
            print(json.dumps(rec), flush=True)
        if args.packed:
            pws = [ops.gemm_pack(wi) for wi in ws]
            for var in [int(v) for v in args.variants.split(",") if int(v) in (0, 2, 3, 4)]:
                y = ops.gemm_packed(x, pws[0], gated=bool(gated), variant=var)
                same = bool(torch.equal(y, ops.gemm(x, ws[0], gated=bool(gated), variant=var)))
                t = timed(lambda: [ops.gemm_packed(x, pws[i % nw], gated=bool(gated), variant=var)
                                   for i in range(calls)]) / calls * 1e3
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "warm": args.warm,
                                  "impl": f"cs_gemm_v{var}_packed", "us": round(t, 2),
                                  "weight_GBps": round(N * K * 2 / t / 1e3, 1),
                                  "bitwise_equal_unpacked": same}), flush=True)
            del pws
        if args.no_torch:
            del ws
            continue
        if gated:
            F = N // 2

            def tfn():
                for i in range(calls):
                    gu = x @ ws[i % nw].t()
                    ops.gated_act(gu[:, :F], gu[:, F:], "silu")
        else:
            def tfn():
                for i in range(calls):
                    x @ ws[i % nw].t()
        t = timed(tfn) / calls * 1e3
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "impl": "torch", "warm": args.warm,
                          "us": round(t, 2), "weight_GBps": round(N * K * 2 / t / 1e3, 1),
                          "TFLOPs": round(2 * M * N * K / t / 1e6, 1)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
