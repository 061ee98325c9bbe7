"""The SHIPPED bf16 path pinned to the reference's own traces.

Every bench number and every bf16 checkpoint runs the stream-kernel path -- DecodeState
(static per-stream K/V, cs_prefix_attention, captured hipGraphs) behind the beam search's
_LiveBeams, and _score_fused for Best-of-N / the evaluator -- while the fp32 fixture
replays of test_methods_gpu.py exercise the eager path (fused_ok() needs bf16).  Here the
fixture weights of the traces whose heads the stream kernels serve (head_dim 64: the C1
and 16-agent traces) are rounded once to bf16 and the reference's recorded decisions are
replayed through that path:

  * beam search, teacher-forced: the generator runs with the reference's proposals (its
    recorded candidates, in its insertion order) and continues from the reference's kept
    beams; every (agent, candidate) increment it computes is compared with the
    reference's recorded last log-prob (beam_search.py:335-404), and the beams its own
    walk would keep must be the reference's wherever the reference's welfare gap between
    the differing candidates exceeds 2 x TOL_BF16 (beam_search.py:558-600);
  * Best-of-N: the reference's candidates scored by score_candidates (_score_fused):
    rewards vs the recorded rewards (best_of_n.py:240-327), argmax vs the reference's
    wherever its top-2 welfare gap exceeds 2 x TOL_BF16 (best_of_n.py:198);
  * the evaluator's per-agent avg log-probs (src/evaluation.py:177-230).

TOL_BF16 is the absolute per-agent log-prob tolerance of the bf16 forward (weights and
activations rounded to bf16, fp32 accumulation) against the reference's fp32 forward.
The measured maxima are printed (pytest -s) and recorded in DESIGN.md.

Each trace runs twice: with the projection / LM-head GEMMs as the shipped dispatch table
routes them (hipBLASLt for these fixture shapes) and with EVERY eligible GEMM forced onto
cs_gemm_bf16 (csrc/gemm.hip), so the hand-written GEMM is pinned to the reference's traces
at the same tolerance, not only to an fp32 product.
"""
import importlib
import json
import os

import pytest
import torch

import method_parity as mp

pytestmark = pytest.mark.gpu

# absolute per-agent log-prob tolerance of the bf16 path against the fp32 reference
TOL_BF16 = 0.06
# ... and of its MEAN over a trace (absolute and signed): bf16 rounding scatters the errors
# around zero, so a systematic error of a few 1e-2 that TOL_BF16 alone would let through
# moves the mean (measured means are printed and recorded in DESIGN.md)
TOL_BF16_MEAN = 0.01
# The traces made with --bf16-weights (weights_bf16: c1, gemma256, main128) hold weights
# that bf16 represents exactly, so the reference's fp32 run and this bf16 replay hold
# IDENTICAL weights and the difference is the bf16 forward alone; both tolerances above are
# a priori (set before any of these traces was measured) and the same for every trace.
# A free-running replay (the product's own proposals and walk) may draw another token than
# the reference only where the reference's draw was a near-tie: its Gumbel-max margin (best
# perturbed score minus the runner-up, recorded by make_method_traces.py) within the
# difference two perturbed scores can have when each is within TOL_BF16
MARGIN_TOL = 2 * TOL_BF16


def _tols(traces):
    """(per-value tolerance, mean |delta| tolerance) of a trace file."""
    return TOL_BF16, TOL_BF16_MEAN


BF16_TRACE_FILES = ["method_traces_c1.json", "method_traces_wide.json",
                    # Gemma-2 head_dim 256 (C3's head shape), soft-caps, sliding window
                    "method_traces_gemma256.json",
                    # C1 at 50 tokens: the bf16 step graphs over two V^T tiles of history
                    "method_traces_c1_long.json",
                    # lookahead branching 2 / depth 4, teacher-forced on the reference's trees
                    "method_traces_fl4.json",
                    # head_dim 128 (Llama-3.1-8B / 3.3-70B: C2, C4, C5) and the reference's
                    # main-body experiment: BoN 4 x 200 tokens, lookahead bf 2 / d 4, beam 4
                    # over 100 tokens, 5 agents
                    "method_traces_main128.json.gz"]
_REPORT = {}


class _EveryShape(dict):
    """A dispatch table that routes every shape cs_gemm_bf16 takes onto it."""

    def get(self, key, default=None):
        M, N, K, g = (int(v) for v in key.split(","))
        if N % 128 or K % 64:
            return default
        return {"variant": 2 if N % 256 == 0 else 3, "splits": 1}


class _EveryShapePacked(_EveryShape):
    """Every shape cs_gemm_bf16 takes, on the packed-weight form (cs_gemm_pack'ed copies,
    cs_gemm_bf16_packed)."""

    def get(self, key, default=None):
        e = super().get(key, default)
        return {"packed": e} if e is not default else default

    def packs(self, N, K, gated):
        return N % 128 == 0 and K % 64 == 0


@pytest.fixture(scope="module", params=[(f, r) for f in BF16_TRACE_FILES
                                        for r in ("dispatch", "cs_gemm", "packed")],
                ids=lambda p: f"{p[0]}-{p[1]}")
def bf16_traces(request, dev):
    fname, route = request.param
    if not mp.trace_exists(fname):
        pytest.skip(f"{fname} not generated (tests/golden/make_method_traces.py)")
    ops = importlib.import_module(mp.PKG + ".ops")
    t = mp.load_traces(fname)
    t["_fname"] = fname
    t["_file"] = fname if route == "dispatch" else (
        f"{fname} (every GEMM on cs_gemm)" if route == "cs_gemm" else
        f"{fname} (every GEMM on cs_gemm, packed weights)")
    eng, tok = mp.register_fixture_engine(t, dev, dtype=torch.bfloat16)
    assert eng.model.fused_ok(), "fixture heads must be served by the stream kernels"
    saved_table, saved_gemm = ops._gemm_table, ops.gemm
    saved_packed = ops.gemm_packed
    calls = [0]
    if route in ("cs_gemm", "packed"):
        def counted(fn):
            def run(*a, **k):
                calls[0] += 1
                return fn(*a, **k)
            return run
        ops._gemm_table = _EveryShape() if route == "cs_gemm" else _EveryShapePacked()
        if route == "cs_gemm":
            ops.gemm = counted(saved_gemm)
        else:
            ops.gemm_packed = counted(saved_packed)
    try:
        yield t, eng, tok
    finally:
        ops._gemm_table, ops.gemm, ops.gemm_packed = saved_table, saved_gemm, saved_packed
        importlib.import_module(mp.PKG + ".runtime").clear_engines()
    if route != "dispatch" and fname == "method_traces_c1.json":
        assert calls[0] > 0, f"no GEMM of the C1 fixture went through the {route} route"


def _report(name, key, value):
    _REPORT.setdefault(name, {})[key] = value
    print(f"bf16 parity {name}: {key} = {value}")
    out = os.environ.get("CS_BF16_PARITY_JSON")
    if out:
        with open(out, "w") as f:
            json.dump(_REPORT, f, indent=1)


def test_beam_fused_path_teacher_forced_against_reference(bf16_traces):
    traces, eng, tok = bf16_traces
    methods = importlib.import_module(mp.PKG + ".methods")
    for run in traces["runs"]:
        if run["method"] != "beam_search":
            continue
        ref_steps, users = mp.beam_reference_steps(traces, run, tok)
        tol, tol_mean = _tols(traces)
        A = len(users)
        gen = methods.get_method_generator("beam_search", dict(run["config"]), traces["model_id"])
        orig_walk = gen._walk
        orig_final = gen._final
        st = {"step": 0, "beams": [""], "R_ref": {"": [0.0] * A}, "R_bf": {"": [0.0] * A},
              "U_ref_of": {}, "max_err": 0.0, "sum_err": 0.0, "sum_signed": 0.0, "checked": 0,
              "sel_checked": 0,
              "sel_waived": 0, "errs": []}

        def propose(s_, ref_idx, bias, seed, tok_):
            cands = ref_steps[st["step"]]
            out = []
            for b in st["beams"]:
                ids = []
                for text, _lp in cands:
                    enc = tok.encode(text)
                    if tok.decode(enc[:-1]) == b:
                        ids.append(enc[-1])
                out.append(ids)
            return out + [[] for _ in range(s_.n_beams - len(out))]

        def walk(order, seq_of, tok_str_of, rewards_of, completed):
            n = len(order)
            lp_ref = dict(ref_steps[st["step"]])
            texts = [seq_of(i) for i in range(n)]
            assert sorted(texts) == sorted(lp_ref), "the generator scored other candidates"
            par = [t[:len(t) - len(tok_str_of(i))] for i, t in enumerate(texts)]
            U_bf = [list(rewards_of(i)) for i in range(n)]
            U_ref, U_mix = [], []
            for i in range(n):
                inc = [U_bf[i][a] - st["R_bf"][par[i]][a] for a in range(A)]
                ref = [lp_ref[texts[i]][a] for a in range(A)]
                for a in range(A):
                    e = abs(inc[a] - ref[a])
                    st["max_err"] = max(st["max_err"], e)
                    st["sum_err"] += e
                    st["sum_signed"] += inc[a] - ref[a]
                    st["checked"] += 1
                    if e > tol:
                        st["errs"].append(f"step {st['step']} cand {texts[i][-8:]!r} agent {a}: "
                                          f"{inc[a]:.5f} vs reference {ref[a]:.5f}")
                U_ref.append([st["R_ref"][par[i]][a] + ref[a] for a in range(A)])
                U_mix.append([st["R_ref"][par[i]][a] + inc[a] for a in range(A)])
            W_ref = [min(u) for u in U_ref]
            W_mix = [min(u) for u in U_mix]
            o_ref = sorted(range(n), key=lambda i: -W_ref[i])        # stable: ties in order
            o_mix = sorted(range(n), key=lambda i: -W_mix[i])
            scratch = []
            nb_mix, idx_mix = orig_walk(o_mix, seq_of, tok_str_of, rewards_of, scratch)
            nb_ref, idx_ref = orig_walk(o_ref, seq_of, tok_str_of, rewards_of, completed)
            for i in range(n):
                st["U_ref_of"][texts[i]] = U_ref[i]
            # the bf16 walk keeps the reference's beams unless the candidates it swaps are
            # within 2 x tol of each other in the reference's welfare
            only_ref = set(idx_ref) - set(idx_mix)
            only_mix = set(idx_mix) - set(idx_ref)
            st["sel_checked"] += 1
            if only_ref or only_mix:
                gap = min(abs(W_ref[x] - W_ref[y]) for x in only_ref for y in only_mix) \
                    if only_ref and only_mix else 0.0
                assert gap <= 2 * tol, (st["step"], gap, [texts[i] for i in only_ref],
                                             [texts[i] for i in only_mix])
                st["sel_waived"] += 1
            # teacher forcing: continue from the reference's kept beams
            for i in idx_ref:
                st["R_ref"][texts[i]] = U_ref[i]
                st["R_bf"][texts[i]] = U_bf[i]
            st["beams"] = [texts[i] for i in idx_ref]
            # the reference's next step scores exactly these beams' extensions
            if st["step"] + 1 < len(ref_steps):
                nxt = {tok.decode(tok.encode(t)[:-1]) for t, _ in ref_steps[st["step"] + 1]}
                assert nxt == set(st["beams"]), st["step"]
            st["step"] += 1
            return nb_ref, idx_ref

        def final(completed, beams, dev, A_loc, shard):
            out = orig_final(completed, beams, dev, A_loc, shard)
            pool = completed + beams
            pool = [(s, r) for s, r in pool if len(s.strip().split()) >= 5] or pool
            w = sorted((min(st["U_ref_of"].get(s, st["R_ref"].get(s))) for s, _ in pool),
                       reverse=True)
            st["final_gap"] = (w[0] - w[1]) if len(w) > 1 else float("inf")
            return out

        gen._propose = propose
        gen._walk = walk
        gen._final = final
        stmt = gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        assert gen.decode_path == "fused", gen.decode_path
        assert st["step"] == len(ref_steps)
        tag = f"{traces['_file']} beam {run['config']['beam_width']}"
        _report(tag, "max_abs_increment_err", st["max_err"])
        mean_abs = st["sum_err"] / max(1, st["checked"])
        mean_signed = st["sum_signed"] / max(1, st["checked"])
        _report(tag, "mean_abs_increment_err", mean_abs)
        _report(tag, "mean_signed_increment_err", mean_signed)
        _report(tag, "increments_checked", st["checked"])
        _report(tag, "selections_checked", st["sel_checked"])
        _report(tag, "selections_within_2tol_differing", st["sel_waived"])
        assert not st["errs"], "\n".join(st["errs"][:20])
        # bf16 rounding errors scatter around zero: a systematic error shows in the mean
        assert mean_abs <= tol_mean and abs(mean_signed) <= TOL_BF16_MEAN, (mean_abs, mean_signed)
        # the final choice over cumulative rewards (errors add up over the steps)
        if st["final_gap"] > 2 * tol * st["step"]:
            assert stmt == run["statement"], (stmt, run["statement"], st["final_gap"])


def test_beam_fused_path_free_running_against_reference(bf16_traces):
    """The shipped bf16 beam search running on its OWN proposals (cs_vocab_sample on its
    bf16 reference rows) and its OWN walk over its own cumulative rewards, on weights
    identical to the reference's (weights_bf16 traces).  Every step is compared with the
    reference's (beam_search.py:444-600): each proposal draw, attempt by attempt, against
    the reference's recorded draw (same prompt, same seed); every (agent, candidate)
    increment against the reference's recorded log-prob; the kept beams, in order, against
    the reference's walk.  The replay follows the reference only where it must to stay
    comparable -- a draw that differs where the reference's Gumbel margin is within
    MARGIN_TOL, or kept beams that differ -- and every such point is counted and reported;
    a draw differing at a larger margin fails the test."""
    traces, eng, tok = bf16_traces
    runs = [r for r in traces["runs"] if r["method"] == "beam_search" and "draws" in r]
    if not traces.get("weights_bf16") or not runs:
        pytest.skip("trace not made on bf16-representable weights with recorded draws")
    methods = importlib.import_module(mp.PKG + ".methods")
    ops = importlib.import_module(mp.PKG + ".ops")
    for run in runs:
        ref_steps, users = mp.beam_reference_steps(traces, run, tok)
        draws = {(d["suffix"], d["seed"]): (d["id"], d["margin"]) for d in run["draws"]}
        tol, tol_mean = _tols(traces)
        A = len(users)
        cfg = dict(run["config"])
        n_att = int(cfg["max_sampling_attempts"])
        gen = methods.get_method_generator("beam_search", cfg, traces["model_id"])
        orig_propose, orig_walk, orig_final = gen._propose, gen._walk, gen._final
        st = {"step": 0, "beams": [""], "R_ref": {"": [0.0] * A}, "R_bf": {"": [0.0] * A},
              "U_ref_of": {}, "U_bf_of": {}, "max_err": 0.0, "sum_err": 0.0, "sum_signed": 0.0,
              "checked": 0, "draws_checked": 0, "draw_resyncs": [], "walk_resyncs": [],
              "max_cum_err": 0.0, "first_resync": None, "errs": []}

        def ref_props(n_beams):
            cands = ref_steps[st["step"]]
            out = []
            for b in st["beams"]:
                ids = []
                for text, _lp in cands:
                    enc = tok.encode(text)
                    if tok.decode(enc[:-1]) == b:
                        ids.append(enc[-1])
                out.append(ids)
            return out + [[] for _ in range(n_beams - len(out))]

        def propose(s_, ref_idx, bias, seed, tok_):
            raw = []
            saved = ops.vocab_sample

            def capture(*a, **k):
                ids, lp = saved(*a, **k)
                raw.append(ids.cpu())
                return ids, lp
            ops.vocab_sample = capture
            try:
                got = orig_propose(s_, ref_idx, bias, seed, tok_)
            finally:
                ops.vocab_sample = saved
            raw = torch.cat(raw, dim=1).tolist() if raw else []
            want = ref_props(s_.n_beams)
            # the reference's draws of every live beam, attempt by attempt (its attempt seed
            # base + beam + a, beam_search.py:251, 471-473; the product's the same)
            differ = None
            for b, text in enumerate(st["beams"]):
                for a in range(1, n_att + 1):
                    rec = draws.get((text, seed + b + a))
                    if rec is None:               # the reference stopped drawing this beam
                        break
                    st["draws_checked"] += 1
                    if raw[b][a - 1] != rec[0]:
                        differ = (b, a, rec[1])
                        break
                if differ:
                    break
            if differ is None:
                assert [g for g in got[:len(st["beams"])]] == want[:len(st["beams"])], \
                    (st["step"], "identical draws gave other proposals")
                return got
            b, a, margin = differ
            if margin is None or margin > MARGIN_TOL:
                st["errs"].append(f"step {st['step']} beam {b} attempt {a}: drew "
                                  f"another token where the reference's margin is {margin}")
            st["draw_resyncs"].append((st["step"], margin))
            if st["first_resync"] is None:
                st["first_resync"] = st["step"]
            return want

        def walk(order, seq_of, tok_str_of, rewards_of, completed):
            n = len(order)
            lp_ref = dict(ref_steps[st["step"]])
            texts = [seq_of(i) for i in range(n)]
            assert sorted(texts) == sorted(lp_ref), "the generator scored other candidates"
            par = [t[:len(t) - len(tok_str_of(i))] for i, t in enumerate(texts)]
            U_bf = [list(rewards_of(i)) for i in range(n)]
            U_ref = []
            for i in range(n):
                inc = [U_bf[i][a] - st["R_bf"][par[i]][a] for a in range(A)]
                ref = [lp_ref[texts[i]][a] for a in range(A)]
                for a in range(A):
                    e = abs(inc[a] - ref[a])
                    st["max_err"] = max(st["max_err"], e)
                    st["sum_err"] += e
                    st["sum_signed"] += inc[a] - ref[a]
                    st["checked"] += 1
                    if e > tol:
                        st["errs"].append(f"step {st['step']} cand {texts[i][-8:]!r} agent {a}: "
                                          f"{inc[a]:.5f} vs reference {ref[a]:.5f}")
                U_ref.append([st["R_ref"][par[i]][a] + ref[a] for a in range(A)])
            W_ref = [min(u) for u in U_ref]
            W_bf = [min(u) for u in U_bf]
            st["max_cum_err"] = max([st["max_cum_err"]] +
                                    [abs(x - y) for x, y in zip(W_bf, W_ref)])
            o_ref = sorted(range(n), key=lambda i: -W_ref[i])        # stable: ties in order
            scratch = []
            nb_bf, idx_bf = orig_walk(list(order), seq_of, tok_str_of, rewards_of, scratch)
            nb_ref, idx_ref = orig_walk(o_ref, seq_of, tok_str_of, rewards_of, completed)
            for i in range(n):
                st["U_ref_of"][texts[i]] = U_ref[i]
                st["U_bf_of"][texts[i]] = U_bf[i]
            if idx_bf != idx_ref:
                # the first position where the kept lists differ: its two candidates' gap in
                # the reference's welfare (the product's cumulative welfare ordered them the
                # other way)
                j = next(k for k in range(min(len(idx_bf), len(idx_ref)) + 1)
                         if k >= len(idx_bf) or k >= len(idx_ref) or idx_bf[k] != idx_ref[k])
                gap = (abs(W_ref[idx_ref[j]] - W_ref[idx_bf[j]])
                       if j < len(idx_bf) and j < len(idx_ref) else 0.0)
                st["walk_resyncs"].append((st["step"], gap))
                if st["first_resync"] is None:
                    st["first_resync"] = st["step"]
            for i in idx_ref:
                st["R_ref"][texts[i]] = U_ref[i]
                st["R_bf"][texts[i]] = U_bf[i]
            st["beams"] = [texts[i] for i in idx_ref]
            if st["step"] + 1 < len(ref_steps):
                nxt = {tok.decode(tok.encode(t)[:-1]) for t, _ in ref_steps[st["step"] + 1]}
                assert nxt == set(st["beams"]), st["step"]
            st["step"] += 1
            return nb_ref, idx_ref

        def final(completed, beams, dev, A_loc, shard):
            out = orig_final(completed, beams, dev, A_loc, shard)
            pool = completed + beams
            pool = [(s, r) for s, r in pool if len(s.strip().split()) >= 5] or pool
            w = sorted((min(st["U_ref_of"].get(s, st["R_ref"].get(s))) for s, _ in pool),
                       reverse=True)
            st["final_gap"] = (w[0] - w[1]) if len(w) > 1 else float("inf")
            return out

        gen._propose, gen._walk, gen._final = propose, walk, final
        stmt = gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        assert gen.decode_path == "fused", gen.decode_path
        assert st["step"] == len(ref_steps), (st["step"], len(ref_steps))
        tag = f"{traces['_file']} beam {cfg['beam_width']} x {cfg['max_tokens']} free-running"
        mean_abs = st["sum_err"] / max(1, st["checked"])
        mean_signed = st["sum_signed"] / max(1, st["checked"])
        for k, v in (("steps", st["step"]), ("draws_checked", st["draws_checked"]),
                     ("increments_checked", st["checked"]),
                     ("max_abs_increment_err", st["max_err"]),
                     ("mean_abs_increment_err", mean_abs),
                     ("mean_signed_increment_err", mean_signed),
                     ("max_abs_cumulative_welfare_err", st["max_cum_err"]),
                     ("first_step_followed_reference", st["first_resync"]),
                     ("draw_near_ties_followed", st["draw_resyncs"]),
                     ("walks_followed", st["walk_resyncs"]),
                     ("final_gap", st["final_gap"]),
                     ("statement_identical", stmt == run["statement"])):
            _report(tag, k, v)
        assert not st["errs"], "\n".join(st["errs"][:20])
        assert mean_abs <= tol_mean and abs(mean_signed) <= TOL_BF16_MEAN, (mean_abs, mean_signed)
        # kept beams differ only where the reference's welfare gap is within the measured
        # cumulative welfare error (twice: both candidates' errors)
        for s_, gap in st["walk_resyncs"]:
            assert gap <= 2 * st["max_cum_err"], (s_, gap, st["max_cum_err"])
        # the final choice: the reference's unless its top-2 gap is within that error
        if st["final_gap"] > 2 * st["max_cum_err"]:
            assert stmt == run["statement"], (stmt, run["statement"], st["final_gap"])


def test_best_of_n_scoring_fused_against_reference(bf16_traces):
    traces, eng, tok = bf16_traces
    methods = importlib.import_module(mp.PKG + ".methods")
    for run in traces["runs"]:
        if run["method"] != "best_of_n":
            continue
        gen = methods.get_method_generator("best_of_n", dict(run["config"]), traces["model_id"])
        cands = run["candidates"]
        U = gen.score_candidates(traces["issue"], dict(traces["agent_opinions"]), cands)
        ref = torch.tensor([run["agent_rewards"][aid] for aid in traces["agent_opinions"]],
                           dtype=torch.float64)
        tol, _ = _tols(traces)
        err = float((U.double().cpu() - ref).abs().max())
        _report(f"{traces['_file']} best_of_n", "max_abs_reward_err", err)
        assert err <= tol, err
        W = U.double().cpu().min(dim=0).values
        w_ref = torch.tensor(run["welfare"], dtype=torch.float64)
        top2 = torch.topk(w_ref, 2).values if w_ref.numel() > 1 else None
        if top2 is None or float(top2[0] - top2[1]) > 2 * tol:
            assert int(W.argmax()) == int(w_ref.argmax())


def test_best_of_n_free_running_against_reference(bf16_traces):
    """The whole shipped Best-of-N -- its OWN seeded candidates (runtime.generate on the
    bf16 stream path, cs_vocab_sample per token), then _score_fused and the welfare argmax
    -- against the reference's run (best_of_n.py:104-136 generate_text(seed=seed+i) per
    candidate, :198 argmax).  Every drawn token is compared with the reference's draw of the
    same (candidate seed, t); a different token is accepted only where the reference's
    Gumbel-max margin was a near-tie (<= MARGIN_TOL), and the replay then follows the
    reference's token.  The candidates must then be the reference's, their rewards within
    TOL_BF16, and the chosen statement the reference's wherever its top-2 welfare gap
    exceeds 2 x TOL_BF16."""
    traces, eng, tok = bf16_traces
    runs = [r for r in traces["runs"] if r["method"] == "best_of_n" and "bon_draws" in r]
    if not runs:
        pytest.skip("trace has no recorded Best-of-N draws (make_method_traces.py --bf16-weights)")
    methods = importlib.import_module(mp.PKG + ".methods")
    runtime = importlib.import_module(mp.PKG + ".runtime")
    ops = importlib.import_module(mp.PKG + ".ops")
    tol, _ = _tols(traces)
    for run in runs:
        ref_draw = {}
        for d in run["bon_draws"]:
            for t, (i, m) in enumerate(zip(d["ids"], d["margins"])):
                ref_draw[runtime.to_i64(runtime.draw_seed(int(d["seed"]), t))] = (int(i), float(m))
        stats = {"draws": 0, "resynced": 0, "max_resync_margin": 0.0}
        saved = ops.vocab_sample

        def follow(logits, sd, *a, **k):
            ids, rest = saved(logits, sd, *a, **k)
            ids_h = ids[:, 0].tolist()
            fixed = False
            for j, s in enumerate(sd[:, 0].tolist()):
                assert s in ref_draw, "a draw the reference never made (stream ran past its end)"
                ref_id, margin = ref_draw[s]
                stats["draws"] += 1
                if ids_h[j] != ref_id:
                    assert margin <= MARGIN_TOL, (
                        f"drew {ids_h[j]} where the reference drew {ref_id} at margin {margin}")
                    stats["resynced"] += 1
                    stats["max_resync_margin"] = max(stats["max_resync_margin"], margin)
                    ids_h[j], fixed = ref_id, True
            if fixed:
                ids = ids.clone()
                ids[:, 0] = torch.tensor(ids_h, dtype=ids.dtype, device=ids.device)
            return ids, rest

        gen = methods.get_method_generator("best_of_n", dict(run["config"]), traces["model_id"])
        ops.vocab_sample = follow
        try:
            stmt = gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        finally:
            ops.vocab_sample = saved
        assert stats["draws"] == sum(len(d["ids"]) for d in run["bon_draws"]), stats
        assert gen.last_candidates == run["candidates"]
        U = torch.tensor([gen.last_agent_rewards[aid] for aid in traces["agent_opinions"]],
                         dtype=torch.float64)
        ref = torch.tensor([run["agent_rewards"][aid] for aid in traces["agent_opinions"]],
                           dtype=torch.float64)
        err = float((U - ref).abs().max())
        name = f"{traces['_file']} best_of_n free-running"
        _report(name, "max_abs_reward_err", err)
        _report(name, "draws", stats)
        assert err <= tol, err
        w_ref = torch.tensor(run["welfare"], dtype=torch.float64)
        top2 = torch.topk(w_ref, 2).values if w_ref.numel() > 1 else None
        if top2 is None or float(top2[0] - top2[1]) > 2 * tol:
            assert stmt == run["pre_brushup"] or stmt == run["statement"], (stmt, run["statement"])


def test_evaluator_fused_against_reference(bf16_traces):
    traces, eng, tok = bf16_traces
    ev_mod = importlib.import_module(mp.PKG + ".evaluation")
    ev = ev_mod.StatementEvaluator(traces["model_id"], include_comparative_ranking=False,
                                   verbose=False)
    tol, _ = _tols(traces)
    worst = 0.0
    for rec in traces.get("evaluations", []):     # (absent from the beam-only c1long trace)
        got = ev.evaluate_statement(rec["statement"], traces["issue"], dict(traces["agent_opinions"]))
        for k, ref in rec["result"].items():
            if not k.startswith("avg_logprob") or ref is None or ref != ref:
                continue
            e = abs(float(got[k]) - ref)
            worst = max(worst, e)
            assert e <= tol, (rec["statement"][:20], k, got[k], ref)
    _report(f"{traces['_file']} evaluator", "max_abs_avg_logprob_err", worst)


class _FLTeacher:
    """Teacher forcing of the finite-lookahead stream path (FiniteLookaheadGenerator._teacher)
    onto a reference trace that recorded its tree and draws (make_method_traces.py fl4 /
    gemma256): every one-token draw is the reference's (keyed by statement + path so far and
    the reference's seed, finite_lookahead.py:296-334, 375-377), so the stream path scores
    the reference's own trees; per step the product's per-(agent, path) rewards are compared
    with the reference's (mean of the last len(path) span log-probs of its recorded calls,
    finite_lookahead.py:490-520) and its choice with the reference's max-min (:527), then
    the reference's path is committed."""

    def __init__(self, traces, run, tok, dev, free=False):
        prompts = importlib.import_module(mp.PKG + ".methods.prompts")
        self.tok, self.dev = tok, dev
        # free: the product's own draws are compared with the reference's and kept unless
        # they differ, which they may only where the reference's Gumbel margin is within
        # MARGIN_TOL (then the reference's draw is followed and counted)
        self.free = free
        self.margins = {(d["suffix"], d["seed"]): d.get("margin") for d in run["fl_draws"]}
        self.draws_checked, self.draw_resyncs = 0, []
        self.tol, self.tol_mean = _tols(traces)
        self.steps = run["fl_steps"]
        self.table = {(d["suffix"], d["seed"]): d["text"] for d in run["fl_draws"]}
        self.users = [prompts.FL["agent_user"].format(issue=traces["issue"], opinion=op)
                      for op in traces["agent_opinions"].values()]
        self.tail = {c["user"]: c["tail"] for c in run["calls"]}
        self.k = 0
        self.max_err, self.checked, self.differing, self.errs = 0.0, 0, 0, []
        self.sum_err = self.sum_signed = 0.0

    def draws(self, frontier, bf, depth, kid):
        cur = self.steps[self.k]["current"]
        out = []
        for n in frontier:
            row = []
            for i in range(bf):
                seed = n.seed + i * (depth + 1)
                text = self.table[(cur + "".join(n.strs), seed)]
                if text == "":
                    row.append(self.tok.eos_ids[0])
                else:
                    ids = self.tok.encode(text)
                    assert len(ids) == 1, (text, ids)
                    row.append(ids[0])
            out.append(row)
        if self.free:
            got = kid.cpu().tolist()
            eos = set(self.tok.eos_ids)
            for r, n in enumerate(frontier):
                for i in range(bf):
                    self.draws_checked += 1
                    g, w = got[r][i], out[r][i]
                    if g == w or (g in eos and w in eos):
                        continue
                    key = (cur + "".join(n.strs), n.seed + i * (depth + 1))
                    margin = self.margins.get(key)
                    self.draw_resyncs.append((self.k, margin))
                    if margin is None or margin > MARGIN_TOL:
                        self.errs.append(f"step {self.k} draw {key[1]}: {g} vs reference {w} "
                                         f"at margin {margin}")
        return torch.tensor(out, dtype=kid.dtype, device=kid.device)

    def choose(self, chains, U, W, b):
        st = self.steps[self.k]
        paths = [ch[-1].strs for ch in chains]
        assert paths == st["paths"], (self.k, "the forced tree is not the reference's")
        Uc = U.double().cpu()
        W_ref = []
        for p, path in enumerate(paths):
            stmt = st["current"] + "".join(path)
            u_ref = []
            for a, u in enumerate(self.users):
                tail = self.tail[u + stmt]
                vals = tail[-len(path):]
                ref = sum(vals) / len(vals)
                u_ref.append(ref)
                e = abs(float(Uc[a, p]) - ref)
                self.max_err = max(self.max_err, e)
                self.sum_err += e
                self.sum_signed += float(Uc[a, p]) - ref
                self.checked += 1
                if e > self.tol:
                    self.errs.append(f"step {self.k} path {p} agent {a}: {float(Uc[a, p]):.5f} "
                                     f"vs reference {ref:.5f}")
            W_ref.append(min(u_ref))
        b_ref = max(range(len(paths)), key=lambda i: W_ref[i])       # first max (:527)
        assert paths[b_ref][0] == st["next_token"], (self.k, paths[b_ref], st["next_token"])
        if b != b_ref:
            self.differing += 1
            gap = W_ref[b_ref] - W_ref[b]
            assert gap <= 2 * self.tol, (self.k, b, b_ref, gap)
        self.k += 1
        return b_ref


def test_lookahead_stream_teacher_forced_against_reference(bf16_traces):
    traces, eng, tok = bf16_traces
    methods = importlib.import_module(mp.PKG + ".methods")
    runs = [r for r in traces["runs"] if r["method"] == "finite_lookahead" and "fl_draws" in r]
    if not runs:
        pytest.skip("trace records no lookahead tree")
    for run in runs:
        gen = methods.get_method_generator("finite_lookahead", dict(run["config"]),
                                           traces["model_id"])
        teacher = gen._teacher = _FLTeacher(traces, run, tok, eng.device)
        stmt = gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        assert gen.decode_path == "stream-tree", gen.decode_path
        assert teacher.k == len(run["fl_steps"]), (teacher.k, len(run["fl_steps"]))
        assert stmt == run["statement"], (stmt, run["statement"])
        tag = f"{traces['_file']} lookahead bf {run['config']['branching_factor']} " \
              f"d {run['config']['max_depth']}"
        _report(tag, "max_abs_reward_err", teacher.max_err)
        mean_abs = teacher.sum_err / max(1, teacher.checked)
        mean_signed = teacher.sum_signed / max(1, teacher.checked)
        _report(tag, "mean_abs_reward_err", mean_abs)
        _report(tag, "mean_signed_reward_err", mean_signed)
        _report(tag, "rewards_checked", teacher.checked)
        _report(tag, "choices_within_2tol_differing", teacher.differing)
        assert not teacher.errs, "\n".join(teacher.errs[:20])
        assert mean_abs <= teacher.tol_mean and abs(mean_signed) <= TOL_BF16_MEAN, \
            (mean_abs, mean_signed)


def test_lookahead_stream_free_running_against_reference(bf16_traces):
    """The lookahead stream path drawing its OWN trees (cs_vocab_sample on its bf16
    reference rows, the reference's seed schedule finite_lookahead.py:296-334, 375-377) on
    weights identical to the reference's: every draw compared with the reference's; a
    differing draw is allowed only at a reference Gumbel margin within MARGIN_TOL (the
    reference's draw is then followed, and counted), and the per-(agent, path) rewards and
    choices are checked as in the teacher-forced replay."""
    traces, eng, tok = bf16_traces
    runs = [r for r in traces["runs"] if r["method"] == "finite_lookahead" and "fl_draws" in r
            and all("margin" in d for d in r["fl_draws"])]
    if not traces.get("weights_bf16") or not runs:
        pytest.skip("trace not made on bf16-representable weights with recorded margins")
    methods = importlib.import_module(mp.PKG + ".methods")
    for run in runs:
        gen = methods.get_method_generator("finite_lookahead", dict(run["config"]),
                                           traces["model_id"])
        teacher = gen._teacher = _FLTeacher(traces, run, tok, eng.device, free=True)
        stmt = gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        assert gen.decode_path == "stream-tree", gen.decode_path
        assert teacher.k == len(run["fl_steps"]), (teacher.k, len(run["fl_steps"]))
        tag = f"{traces['_file']} lookahead bf {run['config']['branching_factor']} " \
              f"d {run['config']['max_depth']} free-running"
        mean_abs = teacher.sum_err / max(1, teacher.checked)
        for k, v in (("draws_checked", teacher.draws_checked),
                     ("draw_near_ties_followed", teacher.draw_resyncs),
                     ("max_abs_reward_err", teacher.max_err), ("mean_abs_reward_err", mean_abs),
                     ("choices_within_2tol_differing", teacher.differing),
                     ("statement_identical", stmt == run["statement"])):
            _report(tag, k, v)
        assert not teacher.errs, "\n".join(teacher.errs[:20])
        assert stmt == run["statement"], (stmt, run["statement"])
