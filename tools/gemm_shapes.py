"""Decode-step GEMM shapes (C1 / C3 / C5) through torch (hipBLASLt / rocBLAS, with the
committed TunableOp selection unless TUNE=0), eager and captured, with the weights
STREAMED from HBM as in a step (20 distinct matrices rotated; one reused matrix would sit in
the 256 MB Infinity Cache and overstate the rate).

    python tools/gemm_shapes.py
"""
import os, sys, time, torch
sys.path.insert(0, os.getcwd())
import importlib
R = importlib.import_module("generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.runtime")
if os.environ.get("TUNE", "1") == "1":
    print("tuning:", R.use_gemm_tuning())
dev = torch.device("cuda:0")
shapes = [(20, 128256, 2048), (16, 3072, 2048), (64, 3072, 2048), (272, 8192, 3584), (272, 3584, 4096), (272, 28672, 3584), (272, 3584, 14336), (20, 3072, 2048), (20, 2048, 2048), (20, 16384, 2048), (20, 2048, 8192), (520, 10240, 8192), (520, 57344, 8192), (520, 8192, 28672)]
for M, N, K in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    # 20 distinct weight matrices (>= 600 MB): each call streams its weights from HBM, as a
    # decode step's layers do (one matrix reused would sit in the 256 MB Infinity Cache)
    nw = max(2, min(20, (700 << 20) // (N * K * 2) + 1))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nw)]
    w = ws[0]
    for _ in range(3): y = x @ w.t()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(20): y = x @ ws[i % nw].t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        for i in range(20): y = x @ ws[i % nw].t()
    e1.record(); torch.cuda.synchronize()
    eager = e0.elapsed_time(e1) / 100 * 1e3
    e0.record()
    for _ in range(5): g.replay()
    e1.record(); torch.cuda.synchronize()
    gr = e0.elapsed_time(e1) / 100 * 1e3
    wb = N * K * 2
    sk = ""
    del ws
    print(f"M={M} N={N} K={K}: eager {eager:.1f} us graph {gr:.1f} us  weights {wb/1e6:.1f} MB -> {wb/gr/1e3:.0f} GB/s, {2*M*N*K/gr/1e6:.0f} TF/s{sk}", flush=True)
