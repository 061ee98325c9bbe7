"""BASELINE C4 finite-lookahead statement on the stream path, for rocprofv3 kernel traces:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o c4 -f csv -- \
        python tools/profile_fl.py 8

prints the median host step time; the kernel stats divided by the steps give the GPU
time per step (the difference is host time between launches)."""
import importlib
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main(tokens=8):
    R = importlib.import_module(bench.PKG_DIR + ".runtime")
    methods = importlib.import_module(bench.PKG_DIR + ".methods")
    R.use_gemm_tuning()
    mc = bench.METHOD_CONFIGS["c4"]
    dev = torch.device("cuda:0")
    eng, tok = R.random_engine(mc["preset"], dev, reuse_caches=0, tokenizer_dir=bench.BPE_FIXTURE)
    R.register_engine("random:c4", eng, tok)
    cfg = {"branching_factor": mc["branching_factor"], "max_depth": mc["max_depth"],
           "max_tokens": tokens, "seed": 1, "welfare": mc["welfare"], "retokenize": "ids"}
    ops_ = bench.synthetic_opinions(mc["agents"])
    methods.get_method_generator("finite_lookahead", dict(cfg, max_tokens=2),
                                 "random:c4").generate_statement(bench.SCENARIO_ISSUE, ops_)
    torch.cuda.synchronize()
    g = methods.get_method_generator("finite_lookahead", cfg, "random:c4")
    t0 = time.perf_counter()
    g.generate_statement(bench.SCENARIO_ISSUE, ops_)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    d = np.diff(np.asarray(g.step_times + [t0 + el]))
    print(f"c4: {len(g.trace)} steps, median step {np.median(d[1:]) * 1e3:.2f} ms, "
          f"statement {el:.2f} s, stats {g.stream_stats}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
