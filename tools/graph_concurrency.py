"""Do two streams' kernels overlap inside a captured hipGraph on this MI355X / ROCm?  And does a
weight read on a side stream warm the Infinity Cache for the next GEMM?

    python tools/graph_concurrency.py
Prints JSON lines: sleep-kernel overlap eager vs graph, and the r8c3 gate|up GEMM cold / after
a concurrent side-stream read of its weight (eager and graph).
"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"


def t_of(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def graphed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g.replay


def main():
    ops = importlib.import_module(PKG + ".ops")
    dev = torch.device("cuda:0")
    side = torch.cuda.Stream(device=dev)
    cyc = 60000

    def one():
        torch.cuda._sleep(cyc)

    def two_serial():
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)

    def two_forked():
        m = torch.cuda.current_stream()
        side.wait_stream(m)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
        m.wait_stream(side)

    rec = {"one_eager": t_of(one), "serial_eager": t_of(two_serial), "forked_eager": t_of(two_forked),
           "one_graph": t_of(graphed(one)), "serial_graph": t_of(graphed(two_serial)),
           "forked_graph": t_of(graphed(two_forked))}
    print(json.dumps({k: round(v, 2) for k, v in rec.items()}), flush=True)

    # gate|up of per-rank C3 on packed weights, rotated over weights that do not fit the cache
    M, N, K = 48, 28672, 3584
    nw = 8
    pws = [ops.gemm_pack(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05) for _ in range(nw)]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ch = ops.gemm_choice(M, N, K, True, packed=True) or {"variant": 3, "splits": 1}
    st = {"i": 0}

    def gemm(w):
        ops.gemm_packed(x, w, gated=True, splits=ch["splits"], variant=ch["variant"])

    def read(w):      # a plain full read of the weight (torch reduction: every byte once)
        w.data.view(torch.int32).sum(dtype=torch.int64)

    def cold():
        for i in range(nw):
            torch.cuda._sleep(cyc)
            gemm(pws[i])

    def warm():
        for i in range(nw):
            torch.cuda._sleep(cyc)
            gemm(pws[0])

    def prefetched():
        m = torch.cuda.current_stream()
        for i in range(nw):
            side.wait_stream(m)
            with torch.cuda.stream(side):
                read(pws[i])
            torch.cuda._sleep(cyc)
            m.wait_stream(side)
            gemm(pws[i])

    def idle():
        for i in range(nw):
            torch.cuda._sleep(cyc)

    r2 = {}
    for mode, wrap in (("eager", lambda f: f), ("graph", graphed)):
        t_idle = t_of(wrap(idle))
        for name, fn in (("cold", cold), ("warm", warm), ("prefetched", prefetched)):
            r2[f"{name}_{mode}_us"] = round((t_of(wrap(fn)) - t_idle) / nw, 2)
        r2[f"idle_{mode}_us"] = round(t_idle / nw, 2)
    print(json.dumps({"shape": "r8c3 gate|up packed", **r2}), flush=True)


if __name__ == "__main__":
    main()
