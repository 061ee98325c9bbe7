"""A/B of the 8B MLP / attention-projection GEMM layouts on the e2e token counts: separate
q, k, v and gate, up GEMMs vs one fused GEMM each (+ the SiLU·up elementwise on
contiguous vs split halves)."""
import json
import torch
import torch.nn.functional as F

dev = "cuda"
d, F_, Hq, Hkv = 4096, 14336, 4096, 1024


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for rows in (1600, 16346):
    x = torch.randn(rows, d, device=dev, dtype=torch.bfloat16)
    wg = torch.randn(F_, d, device=dev, dtype=torch.bfloat16) * 0.02
    wu = torch.randn(F_, d, device=dev, dtype=torch.bfloat16) * 0.02
    wgu = torch.cat([wg, wu])
    wq = torch.randn(Hq, d, device=dev, dtype=torch.bfloat16) * 0.02
    wk = torch.randn(Hkv, d, device=dev, dtype=torch.bfloat16) * 0.02
    wv = torch.randn(Hkv, d, device=dev, dtype=torch.bfloat16) * 0.02
    wqkv = torch.cat([wq, wk, wv])
    r = {"rows": rows}
    r["mlp_sep_us"] = timed(lambda: F.silu(x @ wg.t()) * (x @ wu.t()))
    r["mlp_fused_us"] = timed(lambda: (lambda g, u: F.silu(g) * u)(*(x @ wgu.t()).split(F_, -1)))
    r["gemm_gate_us"] = timed(lambda: x @ wg.t())
    r["gemm_gate_up_us"] = timed(lambda: x @ wgu.t())
    r["qkv_sep_us"] = timed(lambda: (x @ wq.t(), x @ wk.t(), x @ wv.t()))
    r["qkv_fused_us"] = timed(lambda: (x @ wqkv.t()).split([Hq, Hkv, Hkv], -1))
    print(json.dumps(r), flush=True)
