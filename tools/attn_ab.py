#!/usr/bin/env python3
"""A/B of the extend attention on the C2 chunk shape (8B model: H 32, Hkv 8, D 128, bf16):
GQA by repeat_interleave + masked SDPA (model.py today) vs SDPA(enable_gqa=True), and the
cost of building K = cat(prefix K gathered per stream, new K).  HIP events."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from beam_ab import timed  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
R, H, Hkv, T, P, D = 109, 32, 8, 149, 200, 128
A = 8
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(R, H, T, D, generator=g, device=dev, dtype=torch.bfloat16)
kp = torch.randn(A, Hkv, P, D, generator=g, device=dev, dtype=torch.bfloat16)
vp = torch.randn(A, Hkv, P, D, generator=g, device=dev, dtype=torch.bfloat16)
kn = torch.randn(R, Hkv, T, D, generator=g, device=dev, dtype=torch.bfloat16)
vn = torch.randn(R, Hkv, T, D, generator=g, device=dev, dtype=torch.bfloat16)
own = torch.arange(R, device=dev) % A
valid = torch.ones(A, P, dtype=torch.bool, device=dev)
causal = torch.ones(T, T, dtype=torch.bool, device=dev).tril()
m = torch.cat([valid[own][:, None, :].expand(R, T, P), causal[None].expand(R, T, T)], -1)[:, None]


def build():
    K = torch.cat([kp[own], kn], 2)
    V = torch.cat([vp[own], vn], 2)
    return K, V


K, V = build()


def today():
    k = K.repeat_interleave(H // Hkv, dim=1)
    v = V.repeat_interleave(H // Hkv, dim=1)
    return F.scaled_dot_product_attention(q, k, v, attn_mask=m)


def gqa():
    return F.scaled_dot_product_attention(q, K, V, attn_mask=m, enable_gqa=True)


o1, o2 = today(), gqa()
r = {"build_kv_us": timed(build, n=20), "repeat_sdpa_us": timed(today, n=20),
     "gqa_sdpa_us": timed(gqa, n=20),
     "max_abs_diff": float((o1.float() - o2.float()).abs().max())}
print(json.dumps({k: (round(v, 1) if k.endswith("us") else v) for k, v in r.items()}), flush=True)
