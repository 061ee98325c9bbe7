"""Shared method-level parity harness (used by the GPU tests and by the CPU tests that
emulate the C-ABI ops with the oracle to check the methods' HOST logic).

Replays every run recorded in tests/golden/method_traces.json (produced by the
reference's own generators, see make_method_traces.py) through the product's
generators on the same seeded fixture model, and compares:
  * final statements (exact), BoN candidates (exact), BoN agent rewards and welfare
    (1e-3 abs, north_star tolerance), MCTS root-child visit counts and chosen token of
    every step (exact);
  * StatementEvaluator log-prob metrics (1e-3 abs on log-probs, 1e-3 rel on welfare);
  * get_prompt_logprobs tokens (exact) and log-probs (1e-3 abs).
"""
from __future__ import annotations

import importlib
import json
import math
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
TOL = 1e-3


# + 16 agents on the Gemma-2 fixture with beam width 8, BoN N = 8, FL bf 3 (wider than the
# appendix scenario; ~1 min of the CPU suite)
TRACE_FILES = ["method_traces.json", "method_traces_gemma.json", "method_traces_bpe.json",
               "method_traces_wide.json",
               # Gemma-2's real head shape (head_dim 256, query_pre_attn_scalar 256, both
               # soft-caps, the 8-token sliding window) with 16 agents; its lookahead run
               # records the reference's tree and draws (make_method_traces.py gemma256)
               "method_traces_gemma256.json"]
# BASELINE C1 shape (Llama-3.2-1B widths and vocabulary, 2 layers; beam 4, BoN N = 8, FL
# bf 3 / depth 2): replayed on the GPU (the CPU emulation of its 128,256-wide LM head
# over ~700 reference scoring calls is too slow for the CPU suite)
GPU_TRACE_FILES = TRACE_FILES + ["method_traces_c1.json",
                                  # BASELINE C1 at its full 50-token horizon (beam 4 x 8
                                  # attempts; histories span two 32-slot V^T tiles)
                                  "method_traces_c1_long.json",
                                  # finite lookahead at the reference's main-body setting
                                  # (branching 2, depth 4) on the C1-shaped fixture
                                  "method_traces_fl4.json",
                                  # the reference's main-body experiment on a Llama-3.1-8B
                                  # shape (head_dim 128, 32 / 8 heads, Llama-3.1 RoPE
                                  # scaling, vocabulary 128,256; 2 layers): 5 agents, BoN
                                  # 4 x 200 tokens, lookahead bf 2 / d 4, beam 4 x 100 tokens
                                  "method_traces_main128.json.gz"]


def trace_exists(name: str) -> bool:
    return os.path.exists(os.path.join(HERE, "golden", name))


def load_traces(name: str = "method_traces.json"):
    path = os.path.join(HERE, "golden", name)
    if name.endswith(".gz"):
        import gzip
        with gzip.open(path, "rt") as f:
            return json.load(f)
    with open(path) as f:
        return json.load(f)


def register_fixture_engine(traces, device, dtype=torch.float32, model_id=None):
    Mm = importlib.import_module(PKG + ".model")
    T = importlib.import_module(PKG + ".tokenizer")
    E = importlib.import_module(PKG + ".engine")
    R = importlib.import_module(PKG + ".runtime")
    if traces.get("tokenizer") == "bpe_fixture":
        tok = T.BPETokenizer(os.path.join(HERE, "golden", "bpe_fixture"),
                             family=traces.get("family", "llama3"))
    else:
        tok = T.CharTokenizer(traces.get("family", "llama3"),
                              vocab_size=traces.get("tokenizer_vocab", 0))
    cfg = Mm.preset(traces["preset"], vocab=traces["vocab"], **traces.get("preset_overrides", {}))
    cpu = Mm.Model(cfg, "cpu", torch.float32, seed=traces["weight_seed"])
    if "embed_scale" in traces:          # the C1-shaped fixture (make_method_traces.py)
        cpu.w["embed"].mul_(traces["embed_scale"])
    if traces.get("weights_bf16"):
        # the reference ran on the seeded weights rounded to bf16 (make_method_traces.py
        # --bf16-weights): the fp32 replay holds the same values, and the bf16 replay's
        # rounding below is exact -- both sides of every comparison hold IDENTICAL weights
        with torch.no_grad():
            for v in cpu.w.values():
                v.copy_(v.bfloat16().float())
    # dtype=bfloat16: the same seeded fp32 weights rounded once to bf16 (the shipped path
    # for bf16 checkpoints: stream kernels, DecodeState, _score_fused)
    w = {k: v.to(device=device, dtype=dtype) for k, v in cpu.w.items()}
    model = Mm.Model(cfg, device, dtype, weights=w)
    eng = E.ScoringEngine(model)
    R.register_engine(model_id or traces["model_id"], eng, tok)
    return eng, tok


def beam_reference_steps(traces, run, tok):
    """The reference's beam search, step by step, rebuilt from its recorded scoring calls
    (beam_search.py:462-538 calls get_prompt_logprobs for beam, then token, then agent):
    [step][(candidate text, {agent: last log-prob})] in the reference's insertion order.
    A candidate of step s is a beam text of s tokens plus one token."""
    prompts = importlib.import_module(PKG + ".methods.prompts")
    users = [prompts.BEAM["agent_user"].format(issue=traces["issue"], opinion=op)
             for op in traces["agent_opinions"].values()]
    steps = {}
    for c in run["calls"]:
        if c["system"] != prompts.BEAM["agent_system"]:
            continue
        a = next(i for i, u in enumerate(users) if c["user"].startswith(u))
        cand = c["user"][len(users[a]):]
        s = len(tok.encode(cand)) - 1
        lp = c["tail"][-1] if c["tail"] else -10.0     # beam_search.py:384 fallback
        step = steps.setdefault(s, {})
        step.setdefault(cand, {})[a] = lp
    return [list(steps[s].items()) for s in sorted(steps)], users


def run_methods(traces):
    methods = importlib.import_module(PKG + ".methods")
    results = []
    for run in traces["runs"]:
        gen = methods.get_method_generator(run["method"], dict(run["config"]), traces["model_id"])
        stmt = gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        results.append((run, gen, stmt))
    return results


def check_methods(traces):
    failures = []
    for run, gen, stmt in run_methods(traces):
        tag = f"{run['method']} {run['config']}"
        if run["method"] == "best_of_n":
            if gen.last_candidates != run["candidates"]:
                failures.append(f"{tag}: candidates differ {gen.last_candidates} vs {run['candidates']}")
                continue
            for aid, ref in run["agent_rewards"].items():
                got = gen.last_agent_rewards[aid]
                d = max(abs(a - b) for a, b in zip(got, ref))
                if d > TOL:
                    failures.append(f"{tag}: agent {aid} rewards differ by {d}")
            d = max(abs(a - b) for a, b in zip(gen.last_welfare, run["welfare"]))
            if d > TOL:
                failures.append(f"{tag}: welfare differs by {d}")
        if run["method"] == "mcts" and gen.trace != run["steps"]:
            failures.append(f"{tag}: search steps {gen.trace} != reference {run['steps']}")
        if stmt != run["statement"]:
            failures.append(f"{tag}: statement {stmt!r} != reference {run['statement']!r}")
    return failures


def check_beam_increments(traces):
    """Every beam candidate's per-agent log-prob increment (the product's U - R) against the
    reference's own get_prompt_logprobs call for (agent prompt + statement + token): its
    last log-prob (beam_search.py:386-395).  With a BPE tokenizer this pins the text path
    for candidates whose re-tokenization differs from the id-level append."""
    methods = importlib.import_module(PKG + ".methods")
    prompts = importlib.import_module(PKG + ".methods.prompts")
    failures, n_checked = [], 0
    users = [prompts.BEAM["agent_user"].format(issue=traces["issue"], opinion=op)
             for op in traces["agent_opinions"].values()]
    for run in traces["runs"]:
        if run["method"] != "beam_search":
            continue
        ref = {(c["system"], c["user"]): c["tail"][-1] for c in run["calls"] if c["tail"]}
        gen = methods.get_method_generator("beam_search", dict(run["config"]), traces["model_id"])
        gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        for si, step in enumerate(gen.step_log):
            inc = step.get("increments")
            if inc is None:
                continue
            for i, cand in enumerate(step["candidates"]):
                for a, u in enumerate(users):
                    r = ref.get((prompts.BEAM["agent_system"], u + cand))
                    if r is None:
                        continue
                    n_checked += 1
                    if abs(inc[a][i] - r) > TOL:
                        failures.append(f"beam step {si} candidate {cand[-16:]!r} agent {a}: "
                                        f"{inc[a][i]:.5f} vs reference {r:.5f}")
    return failures, n_checked


def check_evaluations(traces):
    ev_mod = importlib.import_module(PKG + ".evaluation")
    ev = ev_mod.StatementEvaluator(traces["model_id"], include_comparative_ranking=False,
                                   verbose=False)
    failures = []
    for rec in traces.get("evaluations", []):     # (absent from the beam-only c1long trace)
        got = ev.evaluate_statement(rec["statement"], traces["issue"], dict(traces["agent_opinions"]))
        for k, ref in rec["result"].items():
            g = got.get(k, "MISSING")
            if g == "MISSING":
                failures.append(f"eval {rec['statement'][:20]!r}: key {k} missing")
                continue
            if ref is None or (isinstance(ref, float) and math.isnan(ref)):
                if not (g is None or (isinstance(g, float) and math.isnan(g))):
                    failures.append(f"eval key {k}: {g} vs reference {ref}")
                continue
            tol = TOL if (k.startswith("avg_logprob") or k.startswith("utility_avg")) else \
                TOL * max(1.0, abs(ref))
            if g is None or abs(float(g) - ref) > tol:
                failures.append(f"eval key {k}: {g} vs reference {ref}")
    return failures


def check_prompt_logprobs(traces):
    utils = importlib.import_module(PKG + ".utils")
    failures = []
    for rec in traces.get("prompt_logprobs", []):
        toks, lps = utils.get_prompt_logprobs(traces["model_id"], rec["system"], rec["user"])
        if toks != rec["tokens"]:
            failures.append(f"prompt_logprobs {rec['user']!r}: tokens {toks} vs {rec['tokens']}")
            continue
        for a, b in zip(lps, rec["logprobs"]):
            if (a is None) != (b is None) or (a is not None and abs(a - b) > TOL):
                failures.append(f"prompt_logprobs {rec['user']!r}: {a} vs {b}")
                break
    return failures
