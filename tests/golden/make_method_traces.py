"""Golden METHOD TRACES from the reference's own generators (build container only).

Imports the reference's src/ from /root/reference with `together` replaced by
fake_together (an offline client over an independent CPU transformers forward) and
`dotenv` stubbed, runs BeamSearchGenerator / BestOfNGenerator /
FiniteLookaheadGenerator / StatementEvaluator / get_prompt_logprobs on a small
seeded model, and writes inputs + outputs + every scoring call's log-probs to
tests/golden/method_traces.json.  Nothing from the reference is copied: only the
data its code produced.  The GPU tests replay the same configs through the
product and compare.

Usage:  python tests/golden/make_method_traces.py [--reference /root/reference]
        [--family llama3|gemma2|c1|bpe|wide]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import tempfile
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"

MODEL_ID = "tiny-llama-fixture"
WEIGHT_SEED = 3
FAMILIES = {"llama3": ("tiny-llama-fixture", "method_traces.json"),
            "gemma2": ("tiny-gemma-fixture", "method_traces_gemma.json"),
            # BASELINE C1 shape: Llama-3.2-1B widths (d 2048, 32/8 heads of 64, vocab
            # 128,256 -- the kernels' shapes) with 2 of its 16 layers, so that the
            # reference's ~1,300 serial CPU calls finish in minutes
            "c1": ("llama-3.2-1b-shaped-fixture", "method_traces_c1.json"),
            # the byte-level BPE fixture tokenizer (tests/golden/bpe_fixture): the hosted
            # API re-tokenizes every appended string, so beam candidates whose text merges
            # with the statement differently than the id-level append are scored on the
            # re-tokenized text by the reference
            "bpe": ("tiny-llama-bpe-fixture", "method_traces_bpe.json"),
            # wider than the appendix scenario: 16 agents (BASELINE C3's agent count; the
            # scenario's 4 opinions cycled and tagged per participant, as bench.py's
            # synthetic_opinions), beam width 8 (the top of the main-body sweep
            # configs/main_body/scenario_1.yaml beam_width [2, 4, 6, 8]), BoN N = 8, FL bf 3
            "wide": ("tiny-gemma-wide-fixture", "method_traces_wide.json"),
            # C1 at its full horizon: the same Llama-3.2-1B-shaped fixture, beam 4 x 8
            # attempts over 50 tokens (configs/appendix/llama/scenario_1/beam_search.yaml:33-38
            # max_tokens 50): beams whose histories span two 32-slot tiles
            "c1long": ("llama-3.2-1b-shaped-fixture", "method_traces_c1_long.json"),
            # finite lookahead at the reference's main-body setting (configs/main_body/
            # scenario_1.yaml:47-49: branching_factor 2, max_depth 4) on the C1-shaped
            # fixture: 16 paths of 4 tokens per step, the depth-dependent seed schedule
            # path_seed + i * (max_depth + 1) (finite_lookahead.py:298-301, 376-377)
            "fl4": ("llama-3.2-1b-shaped-fixture", "method_traces_fl4.json"),
            # Gemma-2's real head shape (C3: head_dim 256, query_pre_attn_scalar 256) with
            # both soft-caps and the fixture's 8-token sliding window, 16 agents
            "gemma256": ("tiny-gemma-d256-fixture", "method_traces_gemma256.json"),
            # the reference's main-body experiment (configs/main_body/scenario_1.yaml: 5
            # agents, Best-of-N n 4 x 200 tokens, lookahead bf 2 / depth 4, beam 4) on a
            # Llama-3.1-8B-shaped fixture: widths 4096 / 14336, 32 / 8 heads of 128, the
            # Llama-3.1 RoPE frequency scaling, vocabulary 128,256; 2 of its 32 layers
            "main128": ("llama-3.1-8b-shaped-fixture", "method_traces_main128.json.gz")}
BPE_DIR = os.path.join(HERE, "bpe_fixture")
# untied LM head: with the random tied embedding a shallow model's residual stream makes
# the last token's own logit ~45 sigma above the rest (every draw repeats it); an
# independent head (std 0.02) gives logits of std ~1 and diverse samples
C1_OVERRIDES = {"n_layers": 2, "tie_embeddings": False}
# the 16-agent Gemma-2 fixture with 64-wide heads (the stream attention kernels serve head
# dims 64 / 128 / 256), so the same trace also pins the bf16 stream-decode path
WIDE_OVERRIDES = {"head_dim": 64, "query_pre_attn_scalar": 64.0}
GEMMA256_OVERRIDES = {"head_dim": 256, "query_pre_attn_scalar": 256.0}
MAIN128_OVERRIDES = {"n_layers": 2}


def fixture_model(family: str = "llama3"):
    """The seeded fixture model (CPU fp32) and tokenizer shared by both sides."""
    Mm = importlib.import_module(PKG + ".model")
    T = importlib.import_module(PKG + ".tokenizer")
    if family in ("c1", "c1long", "fl4"):
        cfg = Mm.preset("llama-3.2-1b", **C1_OVERRIDES)
        tok = T.CharTokenizer("llama3", vocab_size=cfg.vocab)
    elif family == "main128":
        cfg = Mm.preset("llama-3.1-8b", **MAIN128_OVERRIDES)
        tok = T.CharTokenizer("llama3", vocab_size=cfg.vocab)
    elif family == "bpe":
        tok = T.BPETokenizer(BPE_DIR, family="llama3")
        cfg = Mm.preset("tiny-llama", vocab=tok.vocab_size)
    else:
        tok = T.CharTokenizer("llama3" if family == "llama3" else "gemma2")
        name = "tiny-llama" if family == "llama3" else "tiny-gemma"
        cfg = Mm.preset(name, vocab=tok.vocab_size,
                        **(WIDE_OVERRIDES if family == "wide" else
                           GEMMA256_OVERRIDES if family == "gemma256" else {}))
    model = Mm.Model(cfg, "cpu", torch.float32, seed=WEIGHT_SEED)
    return cfg, model, tok


# BASELINE C1 (configs/appendix/llama/scenario_1/beam_search.yaml:18-40: beam_width 4,
# max_sampling_attempts 8), Best-of-N with N = 8, finite lookahead bf 3 / depth 2
C1_RUNS = [
    ("beam_search", {"beam_width": 4, "max_tokens": 10, "max_sampling_attempts": 8, "seed": 1,
                     "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
    ("best_of_n", {"n": 8, "max_tokens": 16, "seed": 7, "temperature": 1.0, "api_delay": 0,
                   "log_level": "WARNING"}),
    ("finite_lookahead", {"branching_factor": 3, "max_depth": 2, "max_tokens": 3, "seed": 11,
                          "api_delay": 0, "log_level": "WARNING"}),
]


C1_LONG_RUNS = [
    ("beam_search", {"beam_width": 4, "max_tokens": 50, "max_sampling_attempts": 8, "seed": 1,
                     "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
]


FL4_RUNS = [
    ("finite_lookahead", {"branching_factor": 2, "max_depth": 4, "max_tokens": 3, "seed": 11,
                          "api_delay": 0, "log_level": "WARNING"}),
]


GEMMA256_RUNS = [
    ("beam_search", {"beam_width": 4, "max_tokens": 4, "max_sampling_attempts": 8, "seed": 31,
                     "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
    ("best_of_n", {"n": 8, "max_tokens": 8, "seed": 27, "temperature": 1.0, "api_delay": 0,
                   "log_level": "WARNING"}),
    ("finite_lookahead", {"branching_factor": 2, "max_depth": 3, "max_tokens": 2, "seed": 29,
                          "api_delay": 0, "log_level": "WARNING"}),
]


# configs/main_body/scenario_1.yaml:36-59 (api_delay 0, brushup off, seeds the fixture's):
# Best-of-N at its full 200 tokens, lookahead at bf 2 / depth 4 over 8 committed tokens,
# beam 4 (10 sampling attempts) over its full 200 tokens
MAIN128_RUNS = [
    ("best_of_n", {"n": 4, "max_tokens": 200, "seed": 42, "temperature": 1.0, "api_delay": 0,
                   "log_level": "WARNING"}),
    ("finite_lookahead", {"branching_factor": 2, "max_depth": 4, "max_tokens": 8, "seed": 42,
                          "api_delay": 0, "log_level": "WARNING"}),
    ("beam_search", {"beam_width": 4, "max_tokens": 200, "max_sampling_attempts": 10, "seed": 42,
                     "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
]
# echo log-probs of the prompt tail only (the LM head over these rows): beam search keeps
# the last one (beam_search.py:389-390), the lookahead the path's last <= 4
# (finite_lookahead.py:508-520), and a recorded call keeps its span's last 6 -- all of them
# within the last ~20 positions (the chat frame after the user text is 14 tokens of the
# fixture's tokenizer, tokenizer.render_chat; every recorded tail is checked finite as it is
# recorded); Best-of-N needs the user span (a <= 200-token candidate + that frame); the
# evaluator every position (the reference's find() of a short statement can land in the
# system prompt, src/utils.py:321-363)
MAIN128_TAIL = {"beam_search": 32, "best_of_n": 320, "finite_lookahead": 32, "eval": None}
# the same for the short-candidate traces regenerated on bf16-representable weights (C1:
# Best-of-N candidates <= 16 tokens, gemma256: <= 8)
SHORT_TAIL = {"beam_search": 32, "best_of_n": 96, "finite_lookahead": 32, "eval": None}
TAILS = {"main128": MAIN128_TAIL, "c1": SHORT_TAIL, "gemma256": SHORT_TAIL, "c1long": SHORT_TAIL,
         "fl4": SHORT_TAIL, "wide": SHORT_TAIL}


WIDE_AGENTS = 16
WIDE_RUNS = [
    ("beam_search", {"beam_width": 8, "max_tokens": 3, "max_sampling_attempts": 8, "seed": 21,
                     "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
    ("best_of_n", {"n": 8, "max_tokens": 8, "seed": 17, "temperature": 1.0, "api_delay": 0,
                   "log_level": "WARNING"}),
    ("finite_lookahead", {"branching_factor": 3, "max_depth": 2, "max_tokens": 2, "seed": 19,
                          "api_delay": 0, "log_level": "WARNING"}),
]


BPE_RUNS = [
    ("beam_search", {"beam_width": 3, "max_tokens": 8, "max_sampling_attempts": 6, "seed": 3,
                     "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
    ("beam_search", {"beam_width": 2, "max_tokens": 10, "max_sampling_attempts": 4, "seed": 8,
                     "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
    ("best_of_n", {"n": 4, "max_tokens": 12, "seed": 7, "temperature": 1.0, "api_delay": 0,
                   "log_level": "WARNING"}),
    ("finite_lookahead", {"branching_factor": 2, "max_depth": 2, "max_tokens": 4, "seed": 11,
                          "api_delay": 0, "log_level": "WARNING"}),
]


def round_weights_bf16(model) -> None:
    """Every weight rounded to the nearest bf16 in place (stored fp32): the same rounding
    the product applies when it loads these weights as bf16, so that rounding is exact."""
    with torch.no_grad():
        for v in model.w.values():
            v.copy_(v.bfloat16().float())


def write_traces(name: str, out) -> None:
    """JSON (gzip-compressed for *.gz: the thousands of recorded calls of the wide traces
    repeat the same prompts)."""
    path = os.path.join(HERE, name)
    if name.endswith(".gz"):
        import gzip
        with gzip.open(path, "wt") as f:
            json.dump(out, f)
    else:
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    print("wrote", name)


def load_existing(name: str):
    path = os.path.join(HERE, name)
    if name.endswith(".gz"):
        import gzip
        with gzip.open(path, "rt") as f:
            return json.load(f)
    with open(path) as f:
        return json.load(f)


def install(reference: str, backend) -> None:
    import fake_together

    fake_together.set_backend(backend)
    mod = types.ModuleType("together")
    mod.Together = fake_together.Together
    sys.modules["together"] = mod
    dot = types.ModuleType("dotenv")
    dot.load_dotenv = lambda *a, **k: False
    sys.modules["dotenv"] = dot
    sys.dont_write_bytecode = True
    if reference not in sys.path:
        sys.path.insert(0, reference)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--family", default="llama3", choices=sorted(FAMILIES))
    ap.add_argument("--bf16-weights", action="store_true",
                    help="round the seeded fixture weights to bf16 once (kept as fp32), so the "
                         "reference's fp32 run and the product's bf16 path hold IDENTICAL "
                         "weights; recorded as weights_bf16 in the trace")
    ap.add_argument("--only", default="",
                    help="run only this method's runs and replace them in the existing trace "
                         "file (the other runs, evaluations and prompt records are kept)")
    ap.add_argument("--resume", action="store_true",
                    help="reuse the runs a previous (killed) generation of this family finished")
    args = ap.parse_args()
    import yaml
    import fake_together

    global MODEL_ID
    MODEL_ID, out_name = FAMILIES[args.family]
    cfg, model, tok = fixture_model(args.family)
    if args.bf16_weights:
        round_weights_bf16(model)
    # c1long: beam search only, whose calls are recorded by their last 6 span log-probs
    backend = fake_together.Backend(fake_together.hf_model_for(model, cfg), tok,
                                    tail_positions=32 if args.family == "c1long" else None,
                                    kv_cache=64 if (args.family == "main128" or
                                                    (args.bf16_weights and args.family in TAILS))
                                    else 0)
    install(args.reference, backend)
    scen_path = (("configs", "main_body", "scenario_1.yaml") if args.family == "main128" else
                 ("configs", "appendix", "llama", "scenario_1", "beam_search.yaml"))
    scen = yaml.safe_load(open(os.path.join(args.reference, *scen_path)))["scenario"]
    issue, opinions = scen["issue"], dict(scen["agent_opinions"])
    if args.family in ("wide", "gemma256"):
        texts = list(opinions.values())
        opinions = {f"Agent {i + 1}": f"{texts[i % len(texts)]} (participant {i + 1})"
                    for i in range(WIDE_AGENTS)}

    from src import utils as rutils                      # noqa: E402  (reference)
    from src.methods import beam_search, best_of_n, finite_lookahead, mcts  # noqa: E402
    from src.methods import get_method_generator         # noqa: E402

    calls = []

    def recorder(fn):
        def wrapped(model, system_prompt, user_prompt, *a, **k):
            toks, lps = fn(model, system_prompt, user_prompt, *a, **k)
            if backend.tail is not None:     # fail fast: a tail past the computed rows
                import math
                assert all(v is None or math.isfinite(v) for v in lps[-6:]), \
                    "a recorded tail reaches past the computed positions"
            calls.append({"system": system_prompt, "user": user_prompt, "n": len(lps),
                          "tail": lps[-6:]})
            return toks, lps
        return wrapped

    # mcts.py:615 formats `final_statement` (commented out at :593) in a debug f-string,
    # so every non-empty rollout raises NameError; bind the name in the module globals so
    # the reference's search runs to completion (its evident intent; see methods/mcts.py)
    mcts.final_statement = ""
    for mod in (beam_search, best_of_n, finite_lookahead, mcts):
        mod.get_prompt_logprobs = recorder(mod.get_prompt_logprobs)

    out = {"model_id": MODEL_ID, "weight_seed": WEIGHT_SEED, "preset": cfg.name,
           "family": ("llama3" if args.family in ("c1", "c1long", "fl4", "bpe", "main128")
                      else "gemma2" if args.family in ("wide", "gemma256") else args.family),
           "vocab": cfg.vocab, "issue": issue, "agent_opinions": opinions, "runs": []}
    if args.family in ("c1", "c1long", "fl4"):
        out["preset_overrides"] = dict(C1_OVERRIDES)
        out["tokenizer_vocab"] = cfg.vocab
    if args.family == "main128":
        out["preset_overrides"] = dict(MAIN128_OVERRIDES)
        out["tokenizer_vocab"] = cfg.vocab
    if args.bf16_weights:
        out["weights_bf16"] = True
    if args.family == "bpe":
        out["tokenizer"] = "bpe_fixture"
    if args.family == "wide":
        out["preset_overrides"] = dict(WIDE_OVERRIDES)
    if args.family == "gemma256":
        out["preset_overrides"] = dict(GEMMA256_OVERRIDES)
    runs = (C1_RUNS if args.family == "c1" else C1_LONG_RUNS if args.family == "c1long"
            else FL4_RUNS if args.family == "fl4"
            else MAIN128_RUNS if args.family == "main128"
            else GEMMA256_RUNS if args.family == "gemma256"
            else BPE_RUNS if args.family == "bpe"
            else WIDE_RUNS if args.family == "wide" else None) or [
        ("best_of_n", {"n": 4, "max_tokens": 24, "seed": 7, "temperature": 1.0, "api_delay": 0,
                       "log_level": "WARNING"}),
        ("finite_lookahead", {"branching_factor": 2, "max_depth": 2, "max_tokens": 6, "seed": 11,
                              "api_delay": 0, "log_level": "WARNING"}),
        ("beam_search", {"beam_width": 2, "max_tokens": 8, "max_sampling_attempts": 4, "seed": 42,
                         "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
        ("beam_search", {"beam_width": 3, "max_tokens": 6, "max_sampling_attempts": 5, "seed": 5,
                         "api_delay": 0, "brushup": False, "log_level": "WARNING"}),
        ("mcts", {"num_simulations": 5, "max_tokens": 4, "expansion_sample_width": 2,
                  "max_sampling_attempts": 6, "rollout_depth": 5, "gamma": 0.99, "seed": 13,
                  "exploration_constant": 1.414, "api_delay": 0, "log_level": "WARNING"}),
        ("mcts", {"num_simulations": 4, "max_tokens": 3, "expansion_sample_width": 3,
                  "max_sampling_attempts": 20, "rollout_depth": 3, "gamma": 0.5, "seed": 2,
                  "api_delay": 0, "log_level": "WARNING"}),
    ]
    # --resume: the runs a killed generation finished (written after every run)
    partial = os.path.join(tempfile.gettempdir(), f"make_method_traces_{args.family}.partial.json")
    done = []
    if args.resume and os.path.exists(partial):
        with open(partial) as f:
            done = json.load(f)
    if args.only:
        prev = load_existing(out_name)
        assert prev.get("weights_bf16") == bool(args.bf16_weights), "weights differ from the file's"
        runs = [(m, c) for m, c in runs if m == args.only]
    for ri, (method, mcfg) in enumerate(runs):
        if ri < len(done) and done[ri]["method"] == method and done[ri]["config"] == mcfg:
            out["runs"].append(done[ri])
            print(f"{method}: resumed ({len(done[ri]['calls'])} scoring calls)")
            continue
        calls.clear()
        if args.family in TAILS and (args.family == "main128" or args.bf16_weights):
            backend.tail = TAILS[args.family][method]
        gen = get_method_generator(method, dict(mcfg), MODEL_ID)
        extra = {}
        if method == "best_of_n":
            orig_rewards = gen._calculate_candidate_rewards
            orig_welfare = gen._calculate_egalitarian_welfare

            def rec_rewards(*a, **k):
                r = orig_rewards(*a, **k)
                extra["candidates"] = list(k.get("candidate_statements", a[2] if len(a) > 2 else []))
                extra["agent_rewards"] = {aid: [float(x) for x in v]
                                          for aid, v in r["agent_rewards"].items()}
                return r

            def rec_welfare(*a, **k):
                w = orig_welfare(*a, **k)
                extra["welfare"] = [float(x) for x in w]
                return w

            gen._calculate_candidate_rewards = rec_rewards
            gen._calculate_egalitarian_welfare = rec_welfare
            if args.bf16_weights:
                # every candidate's draws (ids incl. the stop id, with the Gumbel-max margin of
                # each), keyed by its seed: a free-running bf16 replay that draws another token
                # must do so only where the reference's draw was a near-tie
                extra["bon_draws"] = []
                orig_bon_gen = best_of_n.generate_text

                def rec_bon_text(*a, **k):
                    out_text = orig_bon_gen(*a, **k)
                    extra["bon_draws"].append({"seed": k.get("seed"), "ids": backend.last_drawn,
                                               "margins": backend.last_margins})
                    return out_text
                best_of_n.generate_text = rec_bon_text
        if method == "finite_lookahead" and args.family in ("fl4", "gemma256", "main128"):
            # the reference's tree of every step and every one-token draw, so the bf16 replay
            # can teacher-force the tree (its draws from bf16 logits could flip near-ties of
            # the Gumbel argmax): each draw keyed by (statement + path so far, seed) -- the
            # draw is a function of that prompt and seed (finite_lookahead.py:296-334)
            static = gen._create_reference_continuation_prompt(issue, opinions, "")
            extra["fl_steps"], extra["fl_draws"] = [], []
            orig_tree = gen._generate_tree_paths
            orig_first = gen._get_first_token_of_best_path
            orig_gen_text = finite_lookahead.generate_text

            def rec_tree(issue_, ops_, current, *a, **k):
                paths = orig_tree(issue_, ops_, current, *a, **k)
                extra["fl_steps"].append({"current": current, "paths": [list(p) for p in paths]})
                return paths

            def rec_first(*a, **k):
                t = orig_first(*a, **k)
                extra["fl_steps"][-1]["next_token"] = t
                return t

            def rec_gen_text(*a, **k):
                out_text = orig_gen_text(*a, **k)
                up = k.get("user_prompt")
                assert up is not None and up.startswith(static) and k.get("max_tokens") == 1
                extra["fl_draws"].append({"suffix": up[len(static):], "seed": k.get("seed"),
                                          "text": out_text,
                                          "margin": (backend.last_margins[0]
                                                     if backend.last_margins else None)})
                return out_text

            gen._generate_tree_paths = rec_tree
            gen._get_first_token_of_best_path = rec_first
            finite_lookahead.generate_text = rec_gen_text
        if method == "beam_search" and args.bf16_weights:
            # every proposal draw (beam_search.py:251-266) with its Gumbel-max margin, keyed
            # by (statement so far, seed): a free-running bf16 replay that draws another
            # token must do so only where the reference's draw was a near-tie
            rs, ru = gen._create_reference_prompt(issue, opinions, "")
            beam_static = f"{rs}\n\n{ru}" if rs else ru
            backend.draw_log = []
        if method == "mcts":
            extra["steps"] = []
            orig_best = gen._select_best_child

            def rec_best(node):
                b = orig_best(node)
                extra["steps"].append({"visits": {t: c.visits for t, c in node.children.items()},
                                       "chosen": None if b is None else b.token})
                return b

            gen._select_best_child = rec_best
        stmt = gen.generate_statement(issue, opinions)
        if method == "best_of_n" and "bon_draws" in extra:
            best_of_n.generate_text = orig_bon_gen
        if method == "beam_search" and args.bf16_weights:
            assert all(d["prompt"].startswith(beam_static) for d in backend.draw_log)
            extra["draws"] = [{"suffix": d["prompt"][len(beam_static):], "seed": d["seed"],
                               "id": d["id"], "margin": d["margin"]} for d in backend.draw_log]
        if method == "finite_lookahead" and "fl_draws" in extra:
            finite_lookahead.generate_text = orig_gen_text
        out["runs"].append({"method": method, "config": mcfg, "statement": stmt,
                            "pre_brushup": getattr(gen, "pre_brushup_statement", None),
                            "calls": list(calls), **extra})
        print(f"{method}: {stmt!r} ({len(calls)} scoring calls)")
        with open(partial, "w") as f:
            json.dump(out["runs"], f)

    if args.family == "main128" or (args.only and args.family in TAILS):
        import math
        assert all(math.isfinite(v) for r in out["runs"] for c in r["calls"] for v in c["tail"]
                   if v is not None), "a recorded tail reaches past the computed positions"
    if args.only:
        # the new runs replace the file's runs of that method (same configs, in order)
        new = iter(out["runs"])
        prev["runs"] = [next(new) if r["method"] == args.only else r for r in prev["runs"]]
        write_traces(out_name, prev)
        return
    if args.family in ("c1long", "fl4"):   # method runs only (no evaluator pass)
        import math
        assert all(math.isfinite(v) for r in out["runs"] for c in r["calls"] for v in c["tail"]
                   if v is not None), "a recorded tail reaches past the computed positions"
        write_traces(out_name, out)
        return

    # post-hoc evaluation (src/evaluation.py:128-634) on fixed statements
    from src.evaluation import StatementEvaluator  # noqa: E402
    if args.family in TAILS and (args.family == "main128" or args.bf16_weights):
        backend.tail = TAILS[args.family]["eval"]
    ev = StatementEvaluator(MODEL_ID, include_comparative_ranking=False, verbose=False)
    stmts = [out["runs"][0]["statement"],
             "Genetic information should stay private unless the person consents to research.",
             "A"]
    out["evaluations"] = []
    for s in stmts:
        r = ev.evaluate_statement(s, issue, opinions)
        keep = {k: (None if v is None else float(v)) for k, v in r.items()
                if k != "statement_embedding" and not isinstance(v, str)}
        out["evaluations"].append({"statement": s, "result": keep})

    if args.family == "main128":
        import math
        # (the *_cosine welfares are NaN in every family: no embedding model here)
        bad = [(e["statement"][:20], k, v) for e in out["evaluations"]
               for k, v in e["result"].items()
               if v is not None and not math.isfinite(v) and not k.endswith("_cosine")]
        assert not bad, f"non-finite evaluation values: {bad}"
        backend.tail = None

    # text-compat scoring primitive (src/utils.py:201-373), incl. marker cases
    out["prompt_logprobs"] = []
    for system, user in [("You are a judge.", "The statement is fair."),
                         ("Context: genes.", "Ends with a space "),
                         ("Context: genes.", "Ends with a newline\n"),
                         (None, "No system prompt at all."),
                         ("Issue: privacy", "privacy")]:
        toks, lps = rutils.get_prompt_logprobs(MODEL_ID, system, user)
        out["prompt_logprobs"].append({"system": system, "user": user, "tokens": toks,
                                       "logprobs": lps})
    write_traces(out_name, out)


if __name__ == "__main__":
    main()
