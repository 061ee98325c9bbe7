#!/usr/bin/env python3
"""A/B timing of the beam-step pieces on resident logits (HIP events, GPU kept busy so the
host never gaps the queue).  python tools/beam_ab.py [--only c3,c5] [--lib alt.so]

The library reads its planning knobs (CS_DECODE_BLOCK, CS_DECODE_KP, CS_DECODE_ROWS_FIRST,
CS_TARGET_WGS) once per process: sweep them by running this tool once per setting, e.g.
CS_DECODE_KP=4 python tools/beam_ab.py --only c5."""
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
if "--lib" in sys.argv:   # A/B another build of the library: --lib path/to/lib.so
    _lib = importlib.import_module(PKG + "._lib")
    _lib.LIB_NAME = os.path.relpath(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]),
                                    os.path.join(REPO, PKG))
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")
import bench  # noqa: E402


def timed(fn, n=40):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    bench.gpu_busy(st, 10.0)
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1000.0


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    for name, (A, B, K, V, cap, dt) in {"c1": (4, 4, 10, 128256, 0.0, torch.float32),
                                         "c3": (16, 16, 50, 256000, 30.0, torch.bfloat16),
                                         "c3nocap": (16, 16, 50, 256000, 0.0, torch.bfloat16),
                                         "c5": (64, 8, 32, 128256, 0.0, torch.bfloat16),
                                         # per-rank shapes at 8 ranks (agents sharded)
                                         "r8c3": (2, 16, 50, 256000, 30.0, torch.bfloat16),
                                         "r8c5": (8, 8, 32, 128256, 0.0, torch.bfloat16)}.items():
        g = torch.Generator(device=dev).manual_seed(1)
        x = (torch.randn(A * B, V, generator=g, device=dev) * 3).to(dt)
        ref = (torch.randn(B, V, generator=g, device=dev) * 3).to(dt)
        t = torch.randint(0, V, (B, K), generator=g, device=dev, dtype=torch.int32)
        R = torch.zeros(A, B, device=dev)
        ws, wb = ops.Workspace(), ops.Workspace(zeroed=True)
        if "--only" in sys.argv and name not in sys.argv[sys.argv.index("--only") + 1].split(","):
            continue
        r = {"config": name, "lib": "alt" if "--lib" in sys.argv else "tree"}
        r["lsg_k0_us"] = timed(lambda: ops.logsoftmax_gather(x, None, softcap=cap, workspace=ws, want_lse=True))
        r["lsg_kK_us"] = timed(lambda: ops.logsoftmax_gather(x, t.repeat(A, 1), softcap=cap, workspace=ws))
        r["beam_sort_us"] = timed(lambda: ops.beam_step(x, t, R, "min", softcap=cap, workspace=wb))
        r["beam_topB_us"] = timed(lambda: ops.beam_step(x, t, R, "min", n_order=B, softcap=cap, workspace=wb))
        r["beam_nosort_us"] = timed(lambda: ops.beam_step(x, t, R, "min", n_order=0, softcap=cap, workspace=wb))
        r["vocab_topk_us"] = timed(lambda: ops.vocab_topk(ref, K, softcap=cap, workspace=ws))
        wp = ops.Workspace()

        def serial():
            ids, _ = ops.vocab_topk(ref, K, softcap=cap, workspace=wp)
            return ops.beam_step(x, ids, R, "min", n_order=B, softcap=cap, workspace=wb)

        r["step_us"] = timed(serial)   # proposer + fused scoring step, top-B kept
        wd = ops.Workspace(zeroed=True)
        r["decode_us"] = timed(lambda: ops.beam_decode_step(ref, x, R, K, "min", n_order=B,
                                                            softcap=cap, workspace=wd))
        r["bytes"] = A * B * V * x.element_size()
        r["ideal_us"] = r["bytes"] / 8e12 * 1e6
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
