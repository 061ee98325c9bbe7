"""A/B of cs_add_rms_norm's block shape on the decode-step shapes: run once as is and once
under CS_NORM_VPT=1 (the round-4 form: 256 threads, up to 4 vectors each).  One JSON line per
(shape, form): mean launch time over 500 launches replayed from a captured graph (HIP events).

    python tools/norm_block_ab.py > a.jsonl; CS_NORM_VPT=1 python tools/norm_block_ab.py > b.jsonl
"""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")

# (label, rows, d, splits of the folded branch (0: a bf16 branch), post-norm weight)
SHAPES = [
    ("c1", 20, 2048, 0, False),
    ("c3_r8", 48, 3584, 0, True), ("c3_r8_fold", 48, 3584, 8, True),
    ("c3", 272, 3584, 0, True), ("c3_fold", 272, 3584, 8, True),
    ("c5_r8", 72, 8192, 0, False), ("c5_r8_fold", 72, 8192, 8, False),
    ("c5", 520, 8192, 0, False), ("c5_fold", 520, 8192, 4, False),
    ("c4", 528, 4096, 0, False), ("c4_2112", 2112, 4096, 0, False),
]


def main() -> None:
    dev = "cuda"
    form = "vpt" if os.environ.get("CS_NORM_VPT") == "1" else "block"
    g = torch.Generator(device=dev).manual_seed(0)
    for label, rows, d, splits, post in SHAPES:
        a = torch.randn(rows, d, device=dev, generator=g).to(torch.bfloat16)
        w = (1 + 0.1 * torch.randn(d, device=dev, generator=g)).to(torch.bfloat16)
        wb = (1 + 0.1 * torch.randn(d, device=dev, generator=g)).to(torch.bfloat16) if post else None
        if splits:
            b = ops.SplitPartials(torch.randn(splits, rows, d, device=dev, generator=g))
        else:
            b = torch.randn(rows, d, device=dev, generator=g).to(torch.bfloat16)
        s = torch.empty_like(a)
        out = torch.empty_like(a)

        def run():
            ops.add_rms_norm(a, w, 1e-6, b=b, b_weight=wb, s_out=s, out=out)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        # 50 launches captured in one graph: the device time per launch, not the host's
        # ctypes launch rate (~11 us per call)
        graph = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st), torch.cuda.graph(graph, stream=st):
            for _ in range(50):
                run()
        torch.cuda.current_stream().wait_stream(st)
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 10
        e0.record()
        for _ in range(n):
            graph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / (50 * n) * 1e3
        moved = rows * d * 2 * 3 + (splits * rows * d * 4 if splits else rows * d * 2)
        print(json.dumps({"shape": label, "form": form, "rows": rows, "d": d, "splits": splits,
                          "us": round(us, 2), "GBps": round(moved / us / 1e3, 1),
                          "checksum": float(out.float().sum().item())}), flush=True)


if __name__ == "__main__":
    main()
