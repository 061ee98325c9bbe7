"""One method-level beam-search statement of a BASELINE config (bench.py METHOD_CONFIGS),
for rocprofv3 kernel traces of the decode step:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o c3 -- python tools/profile_decode.py c3
"""
import importlib
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

PKG = bench.PKG_DIR


def main(name="c3", steps=20):
    R = importlib.import_module(PKG + ".runtime")
    methods = importlib.import_module(PKG + ".methods")
    mc = bench.METHOD_CONFIGS[name]
    dev = torch.device("cuda:0")
    eng, tok = R.random_engine(mc["preset"], dev, reuse_caches=0, tokenizer_dir=bench.BPE_FIXTURE)
    R.register_engine("p", eng, tok)
    ops_ = bench.synthetic_opinions(mc["agents"])
    cfg = {"beam_width": mc["beam_width"], "max_tokens": steps, "proposer": "topk",
           "top_k": mc["top_k"], "seed": 1}
    methods.get_method_generator("beam_search", dict(cfg, max_tokens=4), "p").generate_statement(
        bench.SCENARIO_ISSUE, ops_)
    torch.cuda.synchronize()
    gen = methods.get_method_generator("beam_search", dict(cfg), "p")
    t0 = time.perf_counter()
    gen.generate_statement(bench.SCENARIO_ISSUE, ops_)
    torch.cuda.synchronize()
    import numpy as np
    d = np.diff(gen.step_times)
    print(f"{name}: {gen.steps_run} steps in {time.perf_counter() - t0:.3f} s, median step "
          f"{1e3 * float(np.median(d[2:])):.3f} ms, prefill (host) {gen.prefill_s:.3f} s, "
          f"path {gen.decode_path}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c3", int(sys.argv[2]) if len(sys.argv) > 2 else 20)
