"""A/B: the model's RMSNorm chain (fp32 cast, pow, mean, rsqrt, casts, weight multiply)
vs torch.nn.functional.rms_norm on the e2e shapes (bf16 [rows, 4096])."""
import json
import torch
import torch.nn.functional as F

dev = "cuda"
for rows in (16384, 65536):
    x = torch.randn(rows, 4096, device=dev, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(4096, device=dev)).to(torch.bfloat16)

    def chain():
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
        return w * y.to(x.dtype)

    def fused():
        return F.rms_norm(x, (4096,), w, 1e-5)

    out = {}
    for name, fn in (("chain", chain), ("rms_norm", fused)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        out[name + "_us"] = s.elapsed_time(e) / 20 * 1e3
    d = (chain().float() - fused().float()).abs().max().item()
    out.update(rows=rows, max_abs_diff=d, read_write_floor_us=rows * 4096 * 4 / 8e12 * 1e6)
    print(json.dumps(out), flush=True)
