"""A/B of ScoringEngine prefix reuse on the methods that re-prefill per call (MCTS, finite
lookahead): wall time per generate_statement with reuse on / off, the engine's reuse
counters, the statements, and the largest per-agent log-prob difference reuse causes on
the same scoring prompts.  Random-init bf16 Llama-3.2-1B architecture, char tokenizer.

python tools/prefix_reuse_ab.py > gpurun_out/prefix_reuse_ab.jsonl
"""
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
methods = importlib.import_module(PKG + ".methods")
runtime = importlib.import_module(PKG + ".runtime")
utils = importlib.import_module(PKG + ".utils")

MODEL = "meta-llama/Llama-3.2-1B-Instruct"
ISSUE = "Should the city expand its network of protected bike lanes?"
OPINIONS = {f"Agent {i + 1}": t for i, t in enumerate([
    "Bike lanes make commuting safer and cut traffic; the city should build many more of them.",
    "Lanes take parking away from small shops. Expansion must come with support for businesses.",
    "I drive to work and worry about congestion; any expansion should be planned carefully.",
    "Cycling is healthy and cheap. Protected lanes are the only way families will ride.",
])}
RUNS = [
    ("mcts", {"num_simulations": 8, "max_tokens": 6, "rollout_depth": 6, "seed": 11,
              "expansion_sample_width": 3}),
    ("finite_lookahead", {"branching_factor": 2, "max_depth": 2, "max_tokens": 8, "seed": 5}),
]


def run(reuse: int):
    runtime.clear_engines()
    eng, _ = runtime.get_engine(MODEL)
    eng.reuse_caches = reuse
    eng.reset_prefix_store()
    out = []
    for name, cfg in RUNS:
        gen = methods.get_method_generator(name, dict(cfg), MODEL)
        gen.generate_statement(ISSUE, dict(OPINIONS))          # warm (allocator, kernels)
        eng.reset_prefix_store()
        eng.reuse_stats = {k: 0 for k in eng.reuse_stats}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stmt = gen.generate_statement(ISSUE, dict(OPINIONS))
        torch.cuda.synchronize()
        out.append({"method": name, "config": cfg, "reuse_caches": reuse,
                    "seconds": time.perf_counter() - t0, "statement": stmt,
                    "reuse_stats": dict(eng.reuse_stats)})
    return out


def lp_delta():
    """max |Δ| of summed user-span log-probs: prompts scored after their one-token-shorter
    versions (reuse) vs scored cold."""
    eng, _ = runtime.get_engine(MODEL)
    systems = [f"Issue: {ISSUE}\nOpinion: {op}\nStatement: Cities should" for op in OPINIONS.values()]
    users = [" build safe lanes"] * len(systems)
    eng.reuse_caches = 0
    cold = utils.user_span_sums(MODEL, systems, users)
    eng.reuse_caches = 4
    eng.reset_prefix_store()
    utils.user_span_sums(MODEL, [s[:-1] for s in systems], users)
    warm = utils.user_span_sums(MODEL, systems, users)
    return float((cold - warm).abs().max())


def profile_mcts(path: str) -> None:
    """cProfile of one MCTS generate_statement (reuse on), top functions by own time."""
    import cProfile
    import pstats
    runtime.clear_engines()
    eng, _ = runtime.get_engine(MODEL)
    name, cfg = RUNS[0]
    gen = methods.get_method_generator(name, dict(cfg), MODEL)
    gen.generate_statement(ISSUE, dict(OPINIONS))
    pr = cProfile.Profile()
    pr.enable()
    gen.generate_statement(ISSUE, dict(OPINIONS))
    torch.cuda.synchronize()
    pr.disable()
    with open(path, "w") as f:
        st = pstats.Stats(pr, stream=f)
        st.sort_stats("tottime").print_stats(30)
        st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--profile":
        profile_mcts(sys.argv[2])
        sys.exit(0)
    res = run(0) + run(4)
    for r in res:
        print(json.dumps(r), flush=True)
    for name, _ in RUNS:
        off = next(r for r in res if r["method"] == name and r["reuse_caches"] == 0)
        on = next(r for r in res if r["method"] == name and r["reuse_caches"] == 4)
        print(json.dumps({"method": name, "speedup": off["seconds"] / on["seconds"],
                          "same_statement": off["statement"] == on["statement"]}), flush=True)
    print(json.dumps({"max_abs_span_logprob_delta_bf16": lp_delta()}), flush=True)
