"""Method-level parity on the MI355X: the product's generators, evaluator and
text-compat scoring primitive, running through the HIP C-ABI library on the GPU,
replay the reference's golden traces (tests/golden/method_traces.json, recorded by
running the reference's own code, see make_method_traces.py)."""
import importlib

import pytest
import torch

import method_parity as mp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=mp.GPU_TRACE_FILES)
def traces(request, dev):
    if not mp.trace_exists(request.param):
        pytest.skip(f"{request.param} not generated (tests/golden/make_method_traces.py)")
    t = mp.load_traces(request.param)
    mp.register_fixture_engine(t, dev)
    yield t
    importlib.import_module(mp.PKG + ".runtime").clear_engines()


def test_native_library_is_the_path(traces):
    ops = importlib.import_module(mp.PKG + ".ops")
    assert ops.logsoftmax_gather.__module__ == mp.PKG + ".ops"
    lib = importlib.import_module(mp.PKG + "._lib")
    assert lib._lib is not None or lib.load() is not None


def test_methods_match_reference_traces(traces):
    failures = mp.check_methods(traces)
    assert not failures, "\n".join(failures)


def test_beam_candidate_logprobs_match_reference_calls(traces):
    failures, n = mp.check_beam_increments(traces)
    assert n > 0 or not any(r["method"] == "beam_search" for r in traces["runs"])
    assert not failures, "\n".join(failures[:20])


def test_evaluator_matches_reference(traces):
    failures = mp.check_evaluations(traces)
    assert not failures, "\n".join(failures)


def test_prompt_logprobs_match_reference(traces):
    failures = mp.check_prompt_logprobs(traces)
    assert not failures, "\n".join(failures)


def test_beam_topk_proposer_runs(traces):
    """The deterministic top-K proposer (BASELINE 'top-k tokens per beam') end to end."""
    methods = importlib.import_module(mp.PKG + ".methods")
    gen = methods.get_method_generator("beam_search", {"beam_width": 4, "max_tokens": 6,
                                                       "proposer": "topk", "top_k": 10,
                                                       "seed": 1}, traces["model_id"])
    s1 = gen.generate_statement(traces["issue"], traces["agent_opinions"])
    s2 = methods.get_method_generator("beam_search", {"beam_width": 4, "max_tokens": 6,
                                                      "proposer": "topk", "top_k": 10, "seed": 1},
                                      traces["model_id"]).generate_statement(
        traces["issue"], traces["agent_opinions"])
    assert s1 == s2 and isinstance(s1, str)
    assert all(len(st["candidates"]) <= 4 * 10 for st in gen.step_log)


def test_score_tree_matches_per_path_scoring(traces):
    """engine.score_tree (each token-tree node once, tree attention mask) gives the same
    log-probs as scoring every root-to-node path as its own continuation."""
    R = importlib.import_module(mp.PKG + ".runtime")
    engine, tok = R.get_engine(traces["model_id"])
    g = torch.Generator().manual_seed(3)
    prefixes = [tok.encode("Issue: genes. Opinion " + str(a) + ":") for a in range(3)]
    prefixes = [[tok.bos_id] + p for p in prefixes]
    cache = engine.prefill(prefixes)
    # a random tree: 3 roots, branching 2-3, depth 3
    tokens, parents, paths = [], [], []
    frontier = [(-1, [])]
    for _ in range(3):
        nxt = []
        for p, path in frontier:
            for _b in range(int(torch.randint(2, 4, (1,), generator=g))):
                t = int(torch.randint(40, 200, (1,), generator=g))
                tokens.append(t)
                parents.append(p)
                paths.append(path + [t])
                nxt.append((len(tokens) - 1, path + [t]))
        frontier = nxt
    node_lp = engine.score_tree(cache, [0, 1, 2], tokens, parents)          # [3, N]
    for a in range(3):
        lp = engine.score(cache, [a] * len(paths), paths)
        offs = engine.offsets(paths, engine.device)
        last = lp[offs[1:].long() - 1]                                       # each path's last token
        assert torch.max(torch.abs(last - node_lp[a])).item() < 1e-4


def test_batched_span_sums_match_per_call_reference_semantics(traces):
    """utils.user_span_sums (id-level fast path + the batched text-compat path, with the
    engine's prefix reuse) == the sum of get_prompt_logprobs per (system, user) call, the
    reference's own per-call primitive (src/utils.py:201-373; mcts.py:270-320, 343-368),
    including spans the first-occurrence find lands on inside the system text, the
    U+200B marker, empty and absent user prompts."""
    utils = importlib.import_module(mp.PKG + ".utils")
    mid = traces["model_id"]
    op = next(iter(traces["agent_opinions"].values()))
    sysA = f"You are a participant.\n\nIssue: {traces['issue']}\nOpinion: {op}\nStatement: We"
    sysB = sysA + " should act"
    pairs = [(sysA, " should"), (sysB, "e"), (sysA, "a "), (sysB, " together\n"),
             (None, "hello there"), (sysA, ""), (sysB, op[:12]), (sysA, " act now"),
             (sysB, "ct")]
    systems, users = [p[0] for p in pairs], [p[1] for p in pairs]
    want = []
    for s, u in pairs:
        _, lps = utils.get_prompt_logprobs(mid, s, u)
        want.append(float(sum(lps)) if lps and all(v is not None for v in lps) else float("nan"))
    got = utils.user_span_sums(mid, systems, users).tolist()
    got2 = utils.user_span_sums(mid, systems, users).tolist()     # served from the store
    for w, g, g2 in zip(want, got, got2):
        assert (w != w) == (g != g) == (g2 != g2)
        if w == w:
            assert abs(w - g) <= 1e-3 and abs(w - g2) <= 1e-3, (w, g, g2)


def test_methods_match_reference_traces_without_prefix_reuse(traces):
    """The same replays with the engine's prefix reuse off (every prompt encoded in full,
    as the reference does): reuse changes how much is encoded, not what is decided."""
    runtime = importlib.import_module(mp.PKG + ".runtime")
    eng, _ = runtime.get_engine(traces["model_id"])
    keep = eng.reuse_caches
    eng.reuse_caches = 0
    eng.reset_prefix_store()
    try:
        failures = mp.check_methods(traces)
    finally:
        eng.reuse_caches = keep
    assert not failures, "\n".join(failures)


def test_prefix_reuse_prefill_matches_full_prefill_on_gpu(traces):
    """An extending prefill (stored K/V + only the new tokens) equals a full prefill on the
    device's attention / GEMM kernels (fp32 fixture model)."""
    runtime = importlib.import_module(mp.PKG + ".runtime")
    E = importlib.import_module(mp.PKG + ".engine")
    eng, _ = runtime.get_engine(traces["model_id"])
    g = torch.Generator().manual_seed(9)
    V = traces["vocab"]
    base = [torch.randint(3, V, (n,), generator=g).tolist() for n in (70, 41, 96)]
    new = [base[0] + [5, 6, 7], base[2][:80] + [9] * 11, base[1][:30], base[0][:69] + [4]]
    ref = E.ScoringEngine(eng.model, reuse_caches=0).prefill(new)
    e2 = E.ScoringEngine(eng.model, reuse_caches=4, reuse_min_tokens=4)
    e2.prefill(base)
    got = e2.prefill(new)
    assert e2.reuse_stats["reused"] == 1
    v = ref.valid
    torch.testing.assert_close(got.last_hidden, ref.last_hidden, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(got.hidden[v], ref.hidden[v], atol=1e-4, rtol=1e-4)
    for (ka, va), (kb, vb) in zip(got.kv, ref.kv):
        m = v[:, None, :, None].expand_as(ka)
        torch.testing.assert_close(ka[m], kb[m], atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(va[m], vb[m], atol=1e-4, rtol=1e-4)


def test_score_matches_full_forward_of_prefix_plus_continuation(traces):
    """engine.score (prefix K/V once per agent, continuations batched as streams with free
    key slots, chunked) == the log-probs of a plain full forward over prefix +
    continuation for every stream (ragged lengths, several owners, tiny chunks)."""
    R = importlib.import_module(mp.PKG + ".runtime")
    E = importlib.import_module(mp.PKG + ".engine")
    base, tok = R.get_engine(traces["model_id"])
    eng = E.ScoringEngine(base.model, max_rows_per_chunk=23, max_streams_per_chunk=3,
                          reuse_caches=0)
    g = torch.Generator().manual_seed(8)
    V = traces["vocab"]
    prefixes = [[tok.bos_id] + torch.randint(3, V, (n,), generator=g).tolist() for n in (9, 30, 17)]
    conts = [torch.randint(3, V, (n,), generator=g).tolist() for n in (1, 7, 12, 3, 1, 9, 5)]
    owner = [0, 1, 2, 1, 0, 2, 0]
    cache = eng.prefill(prefixes)
    lp = eng.score(cache, owner, conts).double().cpu()
    offs = [0]
    for c in conts:
        offs.append(offs[-1] + len(c))
    for r, (o, c) in enumerate(zip(owner, conts)):
        ids = torch.as_tensor(prefixes[o] + c, device=eng.device)[None]
        _, h, _ = eng.model.prefill(ids, torch.tensor([ids.shape[1]], device=eng.device))
        P = len(prefixes[o])
        rows = h[0, P - 1:P - 1 + len(c)]
        z = eng.model.lm_head(rows).double()
        if eng.softcap:                          # gemma-2 final logit soft-cap
            z = eng.softcap * torch.tanh(z / eng.softcap)
        want = torch.log_softmax(z, -1)
        want = want[torch.arange(len(c)), torch.as_tensor(c, device=eng.device)].cpu()
        assert torch.max(torch.abs(lp[offs[r]:offs[r + 1]] - want)).item() < 1e-4, r


@pytest.mark.parametrize("preset", ["tiny-llama", "tiny-gemma"])
def test_bf16_methods_select_the_same_with_and_without_prefix_reuse(dev, preset):
    """Prefix reuse (on by default) changes a prefill's bf16 rounding only at the level of
    a different batch padding; on bf16 models Best-of-N and finite lookahead select the same
    statement with reuse on and off, and their per-agent rewards agree within 2e-2 (bf16
    forward, 150-token scale)."""
    R = importlib.import_module(mp.PKG + ".runtime")
    methods = importlib.import_module(mp.PKG + ".methods")
    opinions = {"Agent 1": "We should fund public transit first.",
                "Agent 2": "Lower the city's taxes before anything else.",
                "Agent 3": "Protect parks and the environment above all."}
    issue = "How should the city spend its budget?"
    results = []
    for reuse in (4, 0):
        eng, tok = R.random_engine(preset, dev, dtype=torch.bfloat16, seed=3, reuse_caches=reuse)
        R.register_engine("test/bf16-reuse", eng, tok)
        try:
            bon = methods.get_method_generator("best_of_n", {"n": 6, "max_tokens": 12, "seed": 5},
                                               "test/bf16-reuse")
            s_bon = bon.generate_statement(issue, opinions)
            fl = methods.get_method_generator("finite_lookahead",
                                              {"branching_factor": 2, "max_depth": 2,
                                               "max_tokens": 6, "seed": 5}, "test/bf16-reuse")
            s_fl = fl.generate_statement(issue, opinions)
            results.append((s_bon, bon.last_welfare, s_fl, eng.reuse_stats["reused"]))
        finally:
            R.clear_engines()
    (b1, w1, f1, used1), (b0, w0, f0, used0) = results
    assert used0 == 0 and used1 > 0
    assert b1 == b0 and f1 == f0
    assert len(w1) == len(w0) and all(abs(x - y) < 2e-2 for x, y in zip(w1, w0))
