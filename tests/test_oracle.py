"""CPU tests: the C oracle is pinned to golden vectors produced by the reference
itself (tests/golden/core_golden.npz via make_golden.py) and to the reference's
published evaluation CSVs (tests/golden/eval_welfare_published.csv)."""
import os

import numpy as np
import pandas as pd
import pytest


@pytest.fixture(scope="module")
def core_golden(golden_dir):
    return np.load(os.path.join(golden_dir, "core_golden.npz"))


@pytest.mark.parametrize("name", ["ls_small", "ls_wide", "ls_big"])
def test_oracle_log_softmax_rows_matches_reference(orc, core_golden, name):
    M = core_golden[f"{name}_in"]
    ref = core_golden[f"{name}_out"]
    n, B = M.shape
    tgt = np.tile(np.arange(B, dtype=np.int32), (n, 1))
    # oracle reads f32; compare the f32-rounded input through the fp64 numpy formula too
    tok, lse = orc.logsoftmax_gather(M.astype(np.float32), tgt)
    np.testing.assert_allclose(tok, ref, atol=1e-5)
    np.testing.assert_allclose(tok, orc.log_softmax_rows_np(M.astype(np.float32)), atol=1e-12)


def _utilities_via_oracle(orc, v, w, rho):
    """core.compute_utilities restated as rows -> oracle log-softmax/gather -> segment sums."""
    L, B, d = v.shape
    n = w.shape[0]
    import itertools
    leaves = np.array(list(itertools.product(range(B), repeat=L)))
    m = len(leaves)
    chosen = v[np.arange(L)[None, :], leaves]            # [m, L, d]
    z = np.cumsum(chosen, axis=1) - chosen
    X = z[:, :, None, :] + v[None]                       # [m, L, B, d]
    logits = rho * np.einsum("id,mtbd->imtb", w, X)      # [n, m, L, B]
    rows = np.ascontiguousarray(logits.reshape(-1, B), dtype=np.float32)
    tgt = np.broadcast_to(leaves[None], (n, m, L)).reshape(-1, 1).astype(np.int32)
    tok, _ = orc.logsoftmax_gather(rows, tgt)
    seg = orc.segment_reduce(tok, np.arange(0, n * m * L + 1, L))
    logu = seg["sum_lp"].reshape(n, m)
    return np.exp(logu - logu.max(axis=1, keepdims=True)) + 1e-300


def test_oracle_compute_utilities_matches_reference(orc, core_golden):
    for s in core_golden["seeds"]:
        v, w = core_golden[f"v_{s}"], core_golden[f"w_{s}"]
        for ri, rho in zip((0, 9, 19), core_golden["rho"]):
            U = _utilities_via_oracle(orc, v, w, rho)
            np.testing.assert_allclose(U, core_golden[f"U_{s}_{ri}"], rtol=1e-5, atol=1e-12)


def test_oracle_point_mass_welfare_and_selection(orc, core_golden):
    for s in core_golden["seeds"]:
        for ri in (0, 9, 19):
            U = core_golden[f"U_{s}_{ri}"]
            F = orc.welfare(U, orc.SUMLOG, eps=1e-320)
            np.testing.assert_allclose(F, core_golden[f"Fpoint_{s}_{ri}"], rtol=1e-12)
            assert orc.topk(orc.welfare(U, orc.SUM), 1)[0, 0] == core_golden[f"jutil_{s}_{ri}"]
            assert orc.topk(orc.welfare(U, orc.MIN), 1)[0, 0] == core_golden[f"jegal_{s}_{ri}"]
            assert orc.topk(F, 1)[0, 0] == core_golden[f"jnash_{s}_{ri}"]


def test_oracle_perplexity_welfare_matches_published_results(orc, golden_dir):
    """src/evaluation.py:367-381 identities on all 749 published rows."""
    df = pd.read_csv(os.path.join(golden_dir, "eval_welfare_published.csv"))
    assert len(df) == 749
    for n_agents, g in df.groupby("n_agents"):
        lp = g[[f"avg_logprob_{j}" for j in range(n_agents)]].to_numpy().T   # [A, rows]
        ppl = np.exp(-lp)
        np.testing.assert_allclose(ppl, g[[f"perplexity_{j}" for j in range(n_agents)]].to_numpy().T,
                                   rtol=1e-12)
        np.testing.assert_allclose(orc.welfare(ppl, orc.MAX),
                                   g["egalitarian_welfare_perplexity"], rtol=1e-12)
        np.testing.assert_allclose(orc.welfare(ppl, orc.SUM),
                                   g["utilitarian_welfare_perplexity"], rtol=1e-12)
        inv = 1.0 / np.maximum(ppl, 1e-9)
        np.testing.assert_allclose(orc.welfare(inv, orc.SUMLOG, eps=1e-300),
                                   g["log_nash_welfare_perplexity"], rtol=1e-10, atol=1e-12)


def test_oracle_topk_is_python_stable_sort(orc):
    rng = np.random.default_rng(3)
    for _ in range(20):
        W = rng.integers(-3, 3, size=37).astype(np.float64)   # many ties
        W[rng.integers(0, 37, size=3)] = np.nan
        idx = orc.topk(W, 37)[0]
        finite = [i for i in range(37) if not np.isnan(W[i])]
        expect = sorted(finite, key=lambda i: W[i], reverse=True)
        expect += [i for i in range(37) if np.isnan(W[i])]
        assert list(idx) == expect


def test_oracle_segment_reduce_skips_none(orc):
    lp = np.array([-1.0, np.nan, -2.0, -0.5, np.nan], dtype=np.float64)
    out = orc.segment_reduce(lp, np.array([0, 3, 3, 5]))
    np.testing.assert_allclose(out["sum_lp"], [-3.0, 0.0, -0.5])
    assert list(out["count"]) == [2, 0, 1]
    np.testing.assert_allclose(out["sum_p"], [np.exp(-1) + np.exp(-2), 0.0, np.exp(-0.5)])
    assert out["last"][0] == -2.0 and np.isnan(out["last"][1]) and np.isnan(out["last"][2])


def test_oracle_welfare_nonfinite_modes(orc):
    U = np.array([[1.0, np.nan, -np.inf], [2.0, 3.0, np.inf]])
    np.testing.assert_allclose(orc.welfare(U, orc.MIN), [1.0, 3.0, np.nan])  # all-non-finite column -> NaN
    W = orc.welfare(U, orc.MIN, nonfinite=1, nan_val=-10, posinf_val=20, neginf_val=-20)
    np.testing.assert_allclose(W, [1.0, -10.0, -20.0])


def test_oracle_bf16_and_f16_decoding(orc):
    rng = np.random.default_rng(5)
    x = (rng.normal(size=(3, 300)) * 4).astype(np.float32)
    tgt = rng.integers(0, 300, size=(3, 2)).astype(np.int32)
    bits = orc.bf16_bits(x)
    tok_b, _ = orc.logsoftmax_gather(bits, tgt, bf16=True)
    tok_ref, _ = orc.logsoftmax_gather(orc.bf16_to_f32(bits), tgt)
    np.testing.assert_allclose(tok_b, tok_ref, atol=1e-12)
    tok_h, _ = orc.logsoftmax_gather(x.astype(np.float16), tgt)
    tok_h_ref, _ = orc.logsoftmax_gather(x.astype(np.float16).astype(np.float32), tgt)
    np.testing.assert_allclose(tok_h, tok_h_ref, atol=1e-12)


def test_oracle_softcap_and_out_of_range(orc):
    rng = np.random.default_rng(6)
    x = (rng.normal(size=(2, 50)) * 40).astype(np.float32)
    tgt = np.array([[3, -1], [50, 7]], dtype=np.int32)
    tok, _ = orc.logsoftmax_gather(x, tgt, softcap=30.0)
    capped = 30.0 * np.tanh(x.astype(np.float64) / 30.0)
    ref = orc.log_softmax_rows_np(capped)
    assert abs(tok[0, 0] - ref[0, 3]) < 1e-12 and abs(tok[1, 1] - ref[1, 7]) < 1e-12
    assert np.isnan(tok[0, 1]) and np.isnan(tok[1, 0])


def test_oracle_uniform_is_strictly_inside_unit_interval(orc):
    u = orc.cs_uniform(123456789, np.arange(1 << 20))
    assert u.dtype == np.float32 and u.min() > 0 and u.max() < 1
    assert abs(float(u.mean()) - 0.5) < 2e-3
    assert np.array_equal(u, orc.cs_uniform(123456789, np.arange(1 << 20)))
    assert not np.array_equal(u[:100], orc.cs_uniform(123456790, np.arange(100)))
