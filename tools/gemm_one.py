"""Run one decode-step GEMM shape through cs_gemm_bf16 (or torch) a few times, for
rocprofv3 kernel-trace / PMC passes:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES ... -- python3 tools/gemm_one.py c3_gu [splits] [torch | variant]
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
ops = importlib.import_module(PKG + ".ops")
from gemm_ab import SHAPES  # noqa: E402

name = sys.argv[1]
splits = int(sys.argv[2]) if len(sys.argv) > 2 else 0
use_torch = len(sys.argv) > 3 and sys.argv[3] == "torch"
variant = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "torch" else 0
M, N, K, gated = SHAPES[name]
dev = torch.device("cuda:0")
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
nw = max(2, min(8, (700 << 20) // (N * K * 2) + 1))
ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nw)]
for i in range(10):
    if use_torch:
        x @ ws[i % nw].t()
    else:
        ops.gemm(x, ws[i % nw], gated=bool(gated), splits=splits, variant=variant)
torch.cuda.synchronize()
print("done", name, splits, "torch" if use_torch else "cs_gemm")
