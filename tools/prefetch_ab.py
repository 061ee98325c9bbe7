"""Does reading the next GEMM's weight into the Infinity Cache beside an HBM-idle phase
(cs_prefetch on a side stream) make that GEMM faster?  Per call: an idle phase (a spin
kernel of about --idle-us, standing in for the step's attention / norm launches), then
the GEMM on one of several rotated weights (HBM-cold), with or without a side-stream
prefetch of that weight launched at the start of the idle phase; 20 calls per hipGraph.

    python tools/prefetch_ab.py [--shapes r8c3,r8c5] [--idle-us 30]
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
ops = importlib.import_module(PKG + ".ops")

SHAPES = {"r8c3_qkv": (48, 8192, 3584, 0), "r8c3_o": (48, 3584, 4096, 0),
          "r8c3_gu_gated": (48, 28672, 3584, 1), "r8c3_down": (48, 3584, 14336, 0),
          "r8c5_qkv": (72, 10240, 8192, 0), "r8c5_o": (72, 8192, 8192, 0),
          "r8c5_gu_gated": (72, 57344, 8192, 1), "r8c5_down": (72, 8192, 28672, 0)}


def graph_time(fn, calls, reps=5):
    fn()
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
        t = e0.elapsed_time(e1) / reps / calls * 1e3
        best = t if best is None else min(best, t)
    return best


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="r8c3,r8c5")
    ap.add_argument("--idle-us", type=float, default=30.0)
    ap.add_argument("--blocks", default="128,256")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    calls = 20
    # calibrate the spin kernel
    cyc = 100000
    t = graph_time(lambda: [torch.cuda._sleep(cyc) for _ in range(calls)], calls)
    cyc = max(1000, int(cyc * a.idle_us / t))
    t_idle = graph_time(lambda: [torch.cuda._sleep(cyc) for _ in range(calls)], calls)
    side = torch.cuda.Stream(device=dev)
    for name, (M, N, K, gated) in SHAPES.items():
        if not name.startswith(tuple(a.shapes.split(","))):
            continue
        nw = max(2, min(20, (1400 << 20) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05 for _ in range(nw)]
        pws = [ops.gemm_pack(w) for w in ws]
        del ws
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        ch = ops.gemm_choice(M, N, K, bool(gated), packed=True) or {"variant": 2, "splits": 1}
        var, sp = ch["variant"], ch["splits"]

        def gemm(i):
            ops.gemm_packed(x, pws[i % nw], gated=bool(gated), splits=sp, variant=var)

        def plain():
            for i in range(calls):
                torch.cuda._sleep(cyc)
                gemm(i)

        def with_prefetch(blocks):
            def run():
                main_s = torch.cuda.current_stream()
                for i in range(calls):
                    side.wait_stream(main_s)
                    with torch.cuda.stream(side):
                        ops.prefetch(pws[i % nw], blocks)
                    torch.cuda._sleep(cyc)
                    gemm(i)
                    main_s.wait_stream(side)
            return run

        def warm():
            for i in range(calls):
                torch.cuda._sleep(cyc)
                ops.gemm_packed(x, pws[0], gated=bool(gated), splits=sp, variant=var)

        rec = {"shape": name, "M": M, "N": N, "K": K, "variant": var, "splits": sp,
               "idle_us": round(t_idle, 2)}
        rec["gemm_cold_us"] = round(graph_time(plain, calls) - t_idle, 2)
        rec["gemm_warm_us"] = round(graph_time(warm, calls) - t_idle, 2)
        for b in map(int, a.blocks.split(",")):
            rec[f"gemm_prefetched_b{b}_us"] = round(graph_time(with_prefetch(b), calls) - t_idle, 2)
        print(json.dumps(rec), flush=True)
        del pws
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
