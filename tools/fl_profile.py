"""torch.profiler over one C4 lookahead statement (2 tokens) on a random-init Llama-3.1-8B:
the host stacks of the launches the C2 / kernel tables cannot attribute (torch indexing,
copies).  python tools/fl_profile.py"""
import importlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
R = importlib.import_module(PKG + ".runtime")
methods = importlib.import_module(PKG + ".methods")


def main():
    dev = torch.device("cuda:0")
    mc = bench.METHOD_CONFIGS["c4"]
    eng, tok = R.random_engine(mc["preset"], dev, reuse_caches=0, tokenizer_dir=bench.BPE_FIXTURE)
    R.register_engine("random:c4", eng, tok)
    ops_ = bench.synthetic_opinions(mc["agents"])
    cfg = {"branching_factor": mc["branching_factor"], "max_depth": mc["max_depth"],
           "max_tokens": 2, "seed": 1, "welfare": mc["welfare"], "retokenize": "ids"}
    methods.get_method_generator("finite_lookahead", dict(cfg), "random:c4").generate_statement(
        bench.SCENARIO_ISSUE, ops_)
    torch.cuda.synchronize()
    gen = methods.get_method_generator("finite_lookahead", dict(cfg, max_tokens=3), "random:c4")
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 with_modules=False) as prof:
        gen.generate_statement(bench.SCENARIO_ISSUE, ops_)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=25,
                                    max_name_column_width=60))
    # where the small torch launches come from: the package's Python frames enclosing each
    # copy / index / fill op in the trace (python_function events nest by time per thread)
    import collections
    import json
    path = os.path.join(REPO, "gpurun_out", "fl_trace.json")
    prof.export_chrome_trace(path)
    with open(path) as f:
        ev = json.load(f)["traceEvents"]
    os.remove(path)
    py = [e for e in ev if e.get("cat") == "python_function" and "dur" in e]
    py.sort(key=lambda e: e["ts"])
    for op in ("aten::copy_", "aten::index", "aten::index_put_", "aten::fill_", "aten::cat",
               "aten::contiguous", "aten::to"):
        c = collections.Counter()
        ops_ev = [e for e in ev if e.get("name") == op and e.get("cat") == "cpu_op"]
        for e in ops_ev:
            t = e["ts"]
            enc = [p for p in py if p["tid"] == e["tid"] and p["ts"] <= t <= p["ts"] + p["dur"]
                   and ("mdps_amd" in p["name"] or "bench" in p["name"])]
            enc.sort(key=lambda p: -p["ts"])
            c[" <- ".join(p["name"][-90:] for p in enc[:3])] += 1
        print(f"== {op}: {len(ops_ev)} calls")
        for k, v in c.most_common(5):
            print(f"  {v:5d}  {k}")


if __name__ == "__main__":
    main()
