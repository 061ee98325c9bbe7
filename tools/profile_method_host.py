#!/usr/bin/env python3
"""Host time of one method-level beam decode (bench method leg c1 / c3): cProfile of the
generator's loop after warm-up, top functions by own time, plus the median step and the
graph step alone.  python tools/profile_method_host.py c3 [c3:text]  (":text": the product
default retokenize "text" over 5 steps, with the text path's counters)"""
import cProfile
import importlib
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

PKG = bench.PKG_DIR


def main(name):
    name, _, mode = name.partition(":")
    text = mode == "text"
    dev = torch.device("cuda:0")
    R = importlib.import_module(PKG + ".runtime")
    methods = importlib.import_module(PKG + ".methods")
    R.use_gemm_tuning()
    mc = bench.METHOD_CONFIGS[name]
    eng, tok = R.random_engine(mc["preset"], dev, reuse_caches=0, tokenizer_dir=bench.BPE_FIXTURE)
    R.register_engine("random:" + mc["preset"], eng, tok)
    ops_ = bench.synthetic_opinions(mc["agents"])
    cfg = {"beam_width": mc["beam_width"], "max_tokens": 20, "proposer": "topk",
           "top_k": mc["top_k"], "seed": 1, "retokenize": "ids"}
    methods.get_method_generator("beam_search", dict(cfg, max_tokens=4),
                                 "random:" + mc["preset"]).generate_statement(bench.SCENARIO_ISSUE, ops_)
    if text:
        cfg = dict(cfg, retokenize="text", max_tokens=5)
    gen = methods.get_method_generator("beam_search", dict(cfg), "random:" + mc["preset"])
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    gen.generate_statement(bench.SCENARIO_ISSUE, ops_)
    pr.disable()
    el = time.perf_counter() - t0
    d = np.diff(np.asarray(gen.step_times))
    print(f"{name}: statement {el:.3f} s, {gen.steps_run} steps, median step {np.median(d[2:] if d.size > 3 else d) * 1e3:.3f} ms, path {gen.decode_path}")
    if text:
        print(f"text path: re-scored {gen.text_compat_candidates}, from decode rows "
              f"{gen.text_rows_candidates}, prefix reuse {eng.reuse_stats}")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())
    if text:
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
        print(s.getvalue())


if __name__ == "__main__":
    for n in sys.argv[1:] or ["c3"]:
        main(n)
