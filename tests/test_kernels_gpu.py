"""GPU parity: every C-ABI kernel vs the CPU oracle on identical seeded inputs.

Tolerances (north_star): per-token / per-agent log-probs within 1e-3 absolute
(fp32 accumulation on the GPU vs fp64 oracle); selected indices bit-exact given
identical scores.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LP_TOL = 1e-3


def _bits(t: torch.Tensor) -> np.ndarray:
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


def _host_logits(t: torch.Tensor):
    """(numpy array, bf16 flag) of a CPU/GPU logits tensor for the oracle."""
    if t.dtype == torch.bfloat16:
        return _bits(t), True
    if t.dtype == torch.float16:
        return t.cpu().numpy(), False
    return t.cpu().numpy(), False


CASES = [
    # dtype, rows, vocab, ld_pad, k, softcap           path exercised
    (torch.bfloat16, 64, 4096, 0, 1, 0.0),            # split-V, aligned
    (torch.bfloat16, 3, 128256, 0, 10, 0.0),          # split-V, Llama-3 vocab, beam-style k
    (torch.float32, 16, 128256, 0, 10, 0.0),          # C1 shape (fp32), split-V
    (torch.bfloat16, 2, 256000, 0, 50, 30.0),         # Gemma-2 vocab + soft-cap, k=50
    (torch.float16, 33, 5003, 3, 2, 0.0),             # odd vocab, padded ld -> misaligned rows
    (torch.bfloat16, 2500, 1000, 1, 1, 0.0),          # single pass, odd ld (every row misaligned)
    (torch.float32, 1, 7, 0, 7, 0.0),                 # tiny row, k = vocab
    (torch.bfloat16, 4096, 4096, 0, 1, 0.0),          # single pass, many rows
    (torch.float32, 2049, 515, 0, 3, 5.0),            # single pass, soft-cap, scalar tail
    (torch.bfloat16, 300, 256000, 1, 4, 30.0),        # single pass, soft-cap table, misaligned
    (torch.bfloat16, 7, 77, 0, 3, 50.0),              # tiny rows through the soft-cap table
]


def _lsg_fuzz(n=30, seed=77):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        dtype = [torch.float32, torch.bfloat16, torch.float16][rng.integers(0, 3)]
        rows = int(rng.choice([1, 2, 5, 31, 255, 256, 257, 1023, 2048, 3001]))
        vocab = int(rng.choice([1, 2, 9, 64, 1000, 4097, 32000, 128256, 256000]))
        if rows * vocab > 40_000_000:
            rows = max(1, 40_000_000 // vocab)
        out.append((dtype, rows, vocab, int(rng.integers(0, 9)), int(rng.integers(0, 9)),
                    float(rng.choice([0.0, 0.0, 30.0, 50.0])) if dtype != torch.float16 else 0.0))
    return out


@pytest.mark.parametrize("dtype,rows,vocab,ld_pad,k,softcap", CASES + _lsg_fuzz())
def test_logsoftmax_gather_matches_oracle(ops, orc, dev, dtype, rows, vocab, ld_pad, k, softcap):
    g = torch.Generator().manual_seed(rows * 7 + vocab)
    full = (torch.randn(rows, vocab + ld_pad, generator=g) * 3.0).to(dtype)
    logits = full[:, :vocab]  # row stride vocab + ld_pad
    tgt = torch.randint(0, vocab, (rows, k), generator=g, dtype=torch.int32)
    tok, lse = ops.logsoftmax_gather(full.to(dev)[:, :vocab], tgt.to(dev), softcap=softcap,
                                     want_lse=True)
    host, bf16 = _host_logits(full)
    o_tok, o_lse = orc.logsoftmax_gather(np.ascontiguousarray(host), tgt.numpy(), softcap=softcap,
                                         bf16=bf16, vocab=vocab)
    if k:
        assert np.max(np.abs(tok.cpu().numpy() - o_tok)) < LP_TOL
    assert np.max(np.abs(lse.cpu().numpy() - o_lse)) < LP_TOL
    del logits


@pytest.mark.parametrize("cap", [30.0, 50.0, 2.5])
def test_bf16_softcap_table_covers_every_bit_pattern(ops, orc, dev, cap):
    """bf16 + soft-cap looks exp(cap*tanh(x/cap)) up in an LDS table (magnitudes clamped at
    2^-24 and 512).  Rows hold every non-NaN bf16 bit pattern (+-0, subnormals, +-inf, the
    largest finite values) in order and shuffled, rows of one pattern class, and a NaN row:
    lse and gathered targets against the fp64 oracle and the fp32 (transcendental) path."""
    bits = np.arange(65536, dtype=np.uint32)
    fin = bits[(bits & 0x7FFF) <= 0x7F80].astype(np.uint16)        # 65,282 patterns
    rng = np.random.default_rng(int(cap * 10))
    V = fin.size
    tiny = fin[(fin & 0x7FFF) < (104 << 7)]
    huge = fin[(fin & 0x7FFF) >= (135 << 7)]
    rows = [fin, rng.permutation(fin), np.resize(rng.permutation(tiny), V),
            np.resize(rng.permutation(huge), V), rng.permutation(fin)]
    rows[4][12345] = 0x7FC1                                         # a NaN
    host = np.ascontiguousarray(np.stack(rows))
    x = torch.from_numpy(host.view(np.int16)).view(torch.bfloat16)
    tgt = torch.from_numpy(rng.integers(0, V, size=(len(rows), 6), dtype=np.int32))
    tgt[0, :3] = torch.tensor([0, V // 2, V - 1], dtype=torch.int32)
    tok, lse = ops.logsoftmax_gather(x.to(dev), tgt.to(dev), softcap=cap, want_lse=True)
    o_tok, o_lse = orc.logsoftmax_gather(host, tgt.numpy(), softcap=cap, bf16=True)
    lse, tok = lse.cpu().numpy(), tok.cpu().numpy()
    assert np.isnan(lse[4]) and np.all(np.isnan(tok[4])) and np.isnan(o_lse[4])
    assert np.max(np.abs(lse[:4] - o_lse[:4])) < LP_TOL
    assert np.max(np.abs(tok[:4] - o_tok[:4])) < LP_TOL
    f_tok, f_lse = ops.logsoftmax_gather(x.float().to(dev), tgt.to(dev), softcap=cap, want_lse=True)
    assert np.max(np.abs(lse[:4] - f_lse.cpu().numpy()[:4])) < 2e-5
    # misaligned rows (odd element offset) exercise the table's scalar head / tail
    xs = x.to(dev)[:4, 1:]
    t2 = torch.clamp(tgt[:4].to(dev) - 1, min=0)
    m_tok, m_lse = ops.logsoftmax_gather(xs, t2, softcap=cap, want_lse=True)
    o2_tok, o2_lse = orc.logsoftmax_gather(np.ascontiguousarray(host[:4, 1:]), t2.cpu().numpy(),
                                           softcap=cap, bf16=True)
    assert np.max(np.abs(m_lse.cpu().numpy() - o2_lse)) < LP_TOL
    assert np.max(np.abs(m_tok.cpu().numpy() - o2_tok)) < LP_TOL


def test_out_of_range_targets_are_nan_and_masked_vocab(ops, orc, dev):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(5, 3000, generator=g) * 2
    x[:, 100:200] = -float("inf")  # logit-bias style masked tokens
    tgt = torch.tensor([[0, -1], [150, 5], [2999, 3000], [7, 8], [9, 10]], dtype=torch.int32)
    tok, _ = ops.logsoftmax_gather(x.to(dev), tgt.to(dev))
    o_tok, _ = orc.logsoftmax_gather(x.numpy(), tgt.numpy())
    t = tok.cpu().numpy()
    assert np.isnan(t[0, 1]) and np.isnan(t[2, 1])
    assert t[1, 0] == -np.inf and o_tok[1, 0] == -np.inf
    m = np.isfinite(o_tok)
    assert np.max(np.abs(t[m] - o_tok[m])) < LP_TOL


def test_zero_rows_is_noop(ops, dev):
    x = torch.empty(0, 128, device=dev, dtype=torch.bfloat16)
    t = torch.empty(0, 1, device=dev, dtype=torch.int32)
    tok, _ = ops.logsoftmax_gather(x, t)
    assert tok.shape == (0, 1)


@pytest.mark.parametrize("rows", [8, 3000])
def test_bitwise_deterministic(ops, dev, rows):
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(rows, 32000, generator=g) * 3).to(torch.bfloat16).to(dev)
    t = torch.randint(0, 32000, (rows, 4), generator=g, dtype=torch.int32).to(dev)
    a, la = ops.logsoftmax_gather(x, t, want_lse=True)
    b, lb = ops.logsoftmax_gather(x, t, want_lse=True)
    assert torch.equal(a, b) and torch.equal(la, lb)


def test_row_shift_invariance(ops, dev):
    """log-softmax is invariant to adding a constant to a row (size-independent property)."""
    g = torch.Generator().manual_seed(8)
    x = torch.randn(40, 50000, generator=g, dtype=torch.float32) * 2
    c = torch.linspace(-20, 20, 40)[:, None]
    t = torch.randint(0, 50000, (40, 3), generator=g, dtype=torch.int32).to(dev)
    a, _ = ops.logsoftmax_gather(x.to(dev), t)
    b, _ = ops.logsoftmax_gather((x + c).to(dev), t)
    assert torch.max(torch.abs(a - b)).item() < 1e-4


def test_full_vocab_probabilities_sum_to_one(ops, dev):
    x = (torch.randn(6, 128256, device=dev) * 4).to(torch.bfloat16)
    t = torch.arange(128256, dtype=torch.int32, device=dev).repeat(6, 1)
    tok, _ = ops.logsoftmax_gather(x, t)
    s = torch.exp(tok.double()).sum(dim=1)
    assert torch.max(torch.abs(s - 1)).item() < 1e-4


def test_segment_reduce_matches_oracle(ops, orc, dev):
    rng = np.random.default_rng(2)
    lens = rng.integers(0, 300, size=257)
    lens[[3, 100]] = 0
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    lp = -np.abs(rng.normal(size=int(off[-1]))).astype(np.float32) * 3
    lp[rng.integers(0, off[-1], size=40)] = np.nan
    out = ops.segment_reduce(torch.as_tensor(lp, device=dev), torch.as_tensor(off, device=dev))
    ref = orc.segment_reduce(lp.astype(np.float64), off)
    assert np.max(np.abs(out["sum_lp"].cpu().numpy() - ref["sum_lp"])) < 1e-3
    assert np.max(np.abs(out["sum_p"].cpu().numpy() - ref["sum_p"])) < 1e-4
    assert np.array_equal(out["count"].cpu().numpy(), ref["count"])
    lo, lr = out["last"].cpu().numpy(), ref["last"]
    assert np.array_equal(np.isnan(lo), np.isnan(lr))
    assert np.array_equal(lo[~np.isnan(lo)], lr[~np.isnan(lr)].astype(np.float32))


@pytest.mark.parametrize("kind", ["min", "sum", "sumlog", "max"])
@pytest.mark.parametrize("nonfinite", ["skip", "replace"])
def test_welfare_matches_oracle(ops, orc, dev, kind, nonfinite):
    rng = np.random.default_rng(4)
    U = rng.uniform(-5, 1, size=(37, 1000)).astype(np.float32)
    U[0, :5] = [np.nan, np.inf, -np.inf, 0.0, 1e-12]
    U[:, 7] = np.nan  # an all-None column
    codes = {"min": orc.MIN, "sum": orc.SUM, "sumlog": orc.SUMLOG, "max": orc.MAX}
    W = ops.welfare(torch.as_tensor(U, device=dev), kind, eps=1e-9, nonfinite=nonfinite)
    ref = orc.welfare(U.astype(np.float64), codes[kind], eps=1e-9,
                      nonfinite=0 if nonfinite == "skip" else 1)
    w = W.cpu().numpy()
    assert np.array_equal(np.isnan(w), np.isnan(ref))
    m = ~np.isnan(ref)
    np.testing.assert_allclose(w[m], ref[m], rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("seg_len", [1, 2, 7, 64, 800, 1000, 4096, 16384])
def test_topk_matches_stable_sort(ops, orc, dev, seg_len):
    rng = np.random.default_rng(seg_len)
    n_seg = 3
    W = rng.integers(-20, 20, size=(n_seg, seg_len)).astype(np.float32)  # heavy ties
    W[:, rng.integers(0, seg_len, size=max(1, seg_len // 50))] = np.nan
    if seg_len > 2:
        W[0, 1] = -0.0
        W[0, 2] = 0.0
    k = seg_len if seg_len <= 1000 else 64
    idx, val = ops.topk(torch.as_tensor(W, device=dev), k)
    ref = orc.topk(W.astype(np.float64), k)
    assert np.array_equal(idx.cpu().numpy(), ref)
    v = val.cpu().numpy()
    assert np.array_equal(np.isnan(v), np.isnan(np.take_along_axis(W, ref, 1)))


@pytest.mark.parametrize("seg_len", [65, 256, 800, 4096, 16384])
@pytest.mark.parametrize("k", [1, 16, 255, 256])
@pytest.mark.parametrize("case", ["ties", "clustered", "all_nan", "constant"])
def test_topk_selection_path(ops, orc, dev, seg_len, k, case):
    """k <= 256 of more than 64 values goes through the radix-select kernel: the exact
    stable order (value desc, index asc, NaN last) under ties, one exponent bin, all-NaN
    and constant segments, with a leading-dimension stride."""
    if k > seg_len:
        pytest.skip("k > seg_len")
    rng = np.random.default_rng(seg_len * 31 + k)
    n_seg, ld = 3, seg_len + 5
    if case == "ties":
        W = rng.integers(-3, 3, size=(n_seg, ld)).astype(np.float32)
        W[:, rng.integers(0, seg_len, size=max(1, seg_len // 20))] = np.nan
    elif case == "clustered":
        W = (-2.5e6 - rng.random((n_seg, ld))).astype(np.float32)
    elif case == "all_nan":
        W = np.full((n_seg, ld), np.nan, dtype=np.float32)
    else:
        W = np.full((n_seg, ld), 1.25, dtype=np.float32)
    Wt = torch.as_tensor(W, device=dev)[:, :seg_len]
    idx, val = ops.topk(Wt, k)
    ref = orc.topk(W[:, :seg_len].astype(np.float64), k)
    assert np.array_equal(idx.cpu().numpy(), ref)
    v = val.cpu().numpy()
    r = np.take_along_axis(W[:, :seg_len], ref, 1)
    assert np.array_equal(np.isnan(v), np.isnan(r)) and np.array_equal(v[~np.isnan(v)], r[~np.isnan(r)])


def test_core_drop_in_matches_reference_golden(pkg, golden_dir, dev):
    import importlib
    core = importlib.import_module(pkg.__name__ + ".core")
    g = np.load(os.path.join(golden_dir, "core_golden.npz"))
    for name in ("ls_small", "ls_wide", "ls_big"):
        np.testing.assert_allclose(core.log_softmax_rows(g[f"{name}_in"]), g[f"{name}_out"],
                                   atol=1e-4)
    for s in g["seeds"]:
        v, w = g[f"v_{s}"], g[f"w_{s}"]
        for ri, rho in zip((0, 9, 19), g["rho"]):
            U, leaves = core.compute_utilities(v, w, rho)
            np.testing.assert_allclose(U, g[f"U_{s}_{ri}"], rtol=1e-4, atol=1e-12)
            assert [tuple(x) for x in g["leaves"]] == leaves
            # selection bit-exact given identical scores (the reference's U)
            Uref = g[f"U_{s}_{ri}"]
            assert core.point_mass_select(Uref, "utilitarian") == g[f"jutil_{s}_{ri}"]
            assert core.point_mass_select(Uref, "egalitarian") == g[f"jegal_{s}_{ri}"]
            F = core.point_mass_welfare(Uref, "nash")
            np.testing.assert_allclose(F, g[f"Fpoint_{s}_{ri}"], rtol=1e-5)


def test_published_perplexity_welfare_on_gpu(ops, golden_dir, dev):
    import pandas as pd
    df = pd.read_csv(os.path.join(golden_dir, "eval_welfare_published.csv"))
    for n_agents, g in df.groupby("n_agents"):
        lp = g[[f"avg_logprob_{j}" for j in range(n_agents)]].to_numpy().T.astype(np.float32)
        ppl = torch.exp(-torch.as_tensor(lp, device=dev))
        np.testing.assert_allclose(ops.welfare(ppl, "max").cpu().numpy(),
                                   g["egalitarian_welfare_perplexity"], rtol=1e-5)
        np.testing.assert_allclose(ops.welfare(ppl, "sum").cpu().numpy(),
                                   g["utilitarian_welfare_perplexity"], rtol=1e-5)
        inv = 1.0 / torch.clamp(ppl, min=1e-9)
        np.testing.assert_allclose(ops.welfare(inv, "sumlog", eps=1e-30).cpu().numpy(),
                                   g["log_nash_welfare_perplexity"], rtol=1e-5, atol=1e-4)


def test_c2_full_size_sampled_rows(ops, orc, dev):
    """BASELINE C2 at full size (76,800 x 128,256 bf16 = 19.7 GB): sampled rows vs oracle,
    every row's log-sum-exp vs torch, and run-to-run bitwise determinism."""
    rows, V = 76_800, 128_256
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.empty(rows, V, dtype=torch.bfloat16, device=dev)
    for r0 in range(0, rows, 4096):
        x[r0:r0 + 4096] = (torch.randn(min(4096, rows - r0), V, generator=g, device=dev) * 3)
    t = torch.randint(0, V, (rows, 1), generator=g, device=dev, dtype=torch.int32)
    tok, lse = ops.logsoftmax_gather(x, t, want_lse=True)
    tok2, _ = ops.logsoftmax_gather(x, t)
    assert torch.equal(tok, tok2)
    pick = torch.tensor([0, 1, 4095, 4096, 38_400, 76_799], device=dev)
    host = _bits(x[pick])
    o_tok, o_lse = orc.logsoftmax_gather(host, t[pick].cpu().numpy(), bf16=True)
    assert np.max(np.abs(tok[pick].cpu().numpy() - o_tok)) < LP_TOL
    ref_lse = torch.cat([torch.logsumexp(x[r0:r0 + 2048].float(), dim=1)
                         for r0 in range(0, rows, 2048)])
    assert torch.max(torch.abs(ref_lse - lse)).item() < LP_TOL
    del x
    torch.cuda.empty_cache()


def test_c4_full_size_lookahead_nash(ops, orc, dev):
    """BASELINE C4 at full size: R = 256 paths x depth 4 x A = 32 agents = 32,768 rows x
    128,256 bf16 (8.4 GB).  Sampled rows vs the oracle; the full pipeline (mean of each
    path's 4 log-probs -> U [32, 256] -> Nash welfare -> argmax) vs the oracle's folds on
    the kernel's own token log-probs (size-independent: exact fold order and tie-break)."""
    A, R, D, V = 32, 256, 4, 128_256
    rows = A * R * D
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.empty(rows, V, dtype=torch.bfloat16, device=dev)
    for r0 in range(0, rows, 4096):
        x[r0:r0 + 4096] = (torch.randn(min(4096, rows - r0), V, generator=g, device=dev) * 3)
    t = torch.randint(0, V, (rows, 1), generator=g, device=dev, dtype=torch.int32)
    tok, _ = ops.logsoftmax_gather(x, t)
    pick = torch.tensor([0, 3, 4, 16_383, 16_384, rows - 1], device=dev)
    o_tok, _ = orc.logsoftmax_gather(_bits(x[pick]), t[pick].cpu().numpy(), bf16=True)
    assert np.max(np.abs(tok[pick].cpu().numpy().reshape(-1) - o_tok.reshape(-1))) < LP_TOL
    del x
    torch.cuda.empty_cache()
    offs = torch.arange(0, rows + 1, D, dtype=torch.int32, device=dev)
    seg = ops.segment_reduce(tok, offs)
    U = (seg["sum_lp"] / seg["count"].float()).view(A, R)
    # Nash welfare of log-prob utilities needs positive utilities: exp(mean lp) as in the
    # evaluator's avg-prob welfare (evaluation.py:337-349)
    P = torch.exp(U).contiguous()
    W = ops.welfare(P, "sumlog")
    best, _ = ops.topk(W, 1)
    h = tok.cpu().numpy().reshape(-1)
    o_seg = orc.segment_reduce(h, offs.cpu().numpy())
    o_U = (o_seg["sum_lp"] / o_seg["count"]).reshape(A, R)
    assert np.max(np.abs(U.cpu().numpy() - o_U)) < LP_TOL
    o_W = orc.welfare(P.cpu().double().numpy(), orc.SUMLOG, eps=1e-9)
    assert np.max(np.abs(W.cpu().numpy() - o_W)) < 1e-3 * A
    assert int(best.item()) == int(orc.topk(W.cpu().double().numpy(), 1)[0, 0])


BEAM_CASES = [
    # dtype, A, B, K, vocab, softcap, kind          shape exercised
    (torch.float32, 4, 4, 10, 128256, 0.0, "min"),     # C1 (fp32 Llama-3.2-1B vocab)
    (torch.bfloat16, 16, 16, 50, 256000, 30.0, "min"),  # C3 (Gemma-2 vocab, soft-cap)
    (torch.bfloat16, 64, 8, 32, 128256, 0.0, "min"),    # C5 (64 agents, beam 8, top-32)
    (torch.bfloat16, 64, 40, 3, 4099, 0.0, "sum"),      # single-pass rows (A*B >= 2048)
    (torch.float16, 5, 3, 7, 5003, 0.0, "sumlog"),      # odd vocab
    (torch.bfloat16, 3, 1, 1, 777, 0.0, "max"),         # first step: one beam, one token
    (torch.bfloat16, 4, 16, 64, 3001, 0.0, "min"),      # B*K = 1024: largest in-launch sort
]


@pytest.mark.parametrize("dtype,A,B,K,vocab,softcap,kind", BEAM_CASES)
def test_beam_step_matches_oracle_and_unfused_path(ops, orc, dev, dtype, A, B, K, vocab, softcap,
                                                   kind):
    g = torch.Generator().manual_seed(A * 131 + B * 7 + K)
    logits = (torch.randn(A * B, vocab, generator=g) * 3.0).to(dtype)
    tgt = torch.randint(0, vocab, (B, K), generator=g, dtype=torch.int32)
    if B > 1 and K > 2:
        tgt[1, K - 2:] = -1                  # a ragged beam: padded candidate slots
    tgt[0, 0] = tgt[0, min(1, K - 1)]        # duplicate token in one beam
    R = (-torch.rand(A, B, generator=g) * 20.0)
    if kind == "sumlog":
        R = torch.rand(A, B, generator=g) * 2.0 + 10.0   # positive utilities for the log
    lg, tg, Rg = logits.to(dev), tgt.to(dev), R.to(dev)
    U, W, order, oval = ops.beam_step(lg, tg, Rg, kind, softcap=softcap)
    C = B * K

    # 1) bit-identical to the unfused kernels on the same device inputs
    tok, _ = ops.logsoftmax_gather(lg, tg.repeat(A, 1), softcap=softcap)
    U2 = (Rg[:, :, None] + tok.view(A, B, K)).reshape(A, C)
    W2 = ops.welfare(U2.contiguous(), kind)
    o2, v2 = ops.topk(W2, C)
    assert torch.equal(torch.nan_to_num(U, nan=7.0), torch.nan_to_num(U2, nan=7.0))
    assert torch.equal(torch.nan_to_num(W, nan=7.0), torch.nan_to_num(W2, nan=7.0))
    assert torch.equal(order, o2) and torch.equal(torch.nan_to_num(oval, nan=7.0),
                                                  torch.nan_to_num(v2, nan=7.0))
    # partial orders (threshold-selection path): the first n of the full order
    for n in sorted({1, B, min(C, 256), min(C, 257)}):
        kept = torch.empty(A, n, device=dev) if C <= 1024 else None
        _, Wn, on, vn = ops.beam_step(lg, tg, Rg, kind, n_order=n, softcap=softcap, kept_out=kept)
        assert torch.equal(on, order[:n]), f"n_order={n}"
        if kept is not None:
            assert torch.equal(torch.nan_to_num(kept, nan=7.0),
                               torch.nan_to_num(U[:, on.long()], nan=7.0))
        assert torch.equal(torch.nan_to_num(vn, nan=7.0), torch.nan_to_num(oval[:n], nan=7.0))
        assert torch.equal(torch.nan_to_num(Wn, nan=7.0), torch.nan_to_num(W, nan=7.0))

    # 2) the CPU oracle: per-agent log-probs within 1e-3, order bit-exact given the scores
    host, bf16 = _host_logits(logits)
    o_tok, _ = orc.logsoftmax_gather(np.ascontiguousarray(host), tgt.repeat(A, 1).numpy(),
                                     softcap=softcap, bf16=bf16, vocab=vocab)
    o_U = (R.double().numpy()[:, :, None] + o_tok.reshape(A, B, K)).reshape(A, C)
    u = U.cpu().numpy()
    assert np.array_equal(np.isnan(u), np.isnan(o_U))
    assert np.nanmax(np.abs(u - o_U)) < LP_TOL
    codes = {"min": orc.MIN, "sum": orc.SUM, "sumlog": orc.SUMLOG, "max": orc.MAX}
    o_W = orc.welfare(o_U, codes[kind], eps=1e-9)
    w = W.cpu().numpy()
    tol = LP_TOL * (A if kind in ("sum",) else 1)
    assert np.nanmax(np.abs(w - o_W)) < tol
    assert np.array_equal(order.cpu().numpy(), orc.topk(w.astype(np.float64), C)[0])


def test_beam_step_sort_skipped_for_sharded_runs(ops, dev):
    A, B, K, V = 2, 4, 5, 3000
    x = torch.randn(A * B, V, device=dev)
    t = torch.randint(0, V, (B, K), device=dev, dtype=torch.int32)
    R = torch.zeros(A, B, device=dev)
    U, W, order, _ = ops.beam_step(x, t, R, "min", n_order=0)
    assert order is None and U.shape == (A, B * K) and torch.isfinite(W).all()
    with pytest.raises(ops.CSError):
        ops.beam_step(x, t, torch.zeros(A, B + 1, device=dev), "min")


@pytest.mark.parametrize("C,n,case", [(40, 4, "rand"), (256, 8, "rand"), (800, 16, "rand"),
                                      (1024, 300, "rand"), (800, 16, "ties"), (512, 64, "clustered"),
                                      (97, 97, "rand"), (1, 1, "rand")])
def test_beam_select_is_topk_plus_keep(ops, orc, dev, C, n, case):
    """cs_beam_select (sharded tail: unfill, stable top-n, kept columns) == the unfused
    where + cs_segmented_topk + index_select, and == the oracle's stable order."""
    g = torch.Generator(device=dev).manual_seed(C * 7 + n)
    A = 3
    U = torch.randn(A, C, generator=g, device=dev) * 4.0
    if case == "ties":
        U = torch.round(U)
    if case == "clustered":
        U = U * 1e-3 - 2.5e6
    W = U.min(0).values
    if C > 4:   # columns without a usable utility: filled with +inf before the MIN all-reduce
        W[3] = float("nan")
        W[C // 2] = float("nan")
    Wx = torch.where(torch.isnan(W), torch.full_like(W, float("inf")), W)
    kept = torch.empty(A, n, device=dev)
    W_out = torch.empty_like(W)
    order, val = ops.beam_select(Wx, n, U=U, unfill="min", kept_out=kept, W_out=W_out,
                                 with_values=True)
    Wn = torch.where(torch.isinf(Wx) & (Wx > 0), torch.full_like(Wx, float("nan")), Wx)
    ref_order, ref_val = ops.topk(Wn, n)
    assert torch.equal(order, ref_order)
    assert torch.equal(torch.nan_to_num(val, nan=1234.5), torch.nan_to_num(ref_val, nan=1234.5))
    assert torch.equal(kept, U.index_select(1, ref_order.long()))
    assert torch.equal(torch.isnan(W_out), torch.isnan(W)) and \
        torch.equal(torch.nan_to_num(W_out), torch.nan_to_num(W))
    assert np.array_equal(order.cpu().numpy(), orc.topk(Wn.cpu().numpy().astype(np.float64), n)[0])
    o2, v2 = ops.beam_select(Wn, n)                 # no unfill, no kept
    assert torch.equal(o2, ref_order) and v2 is None


def test_beam_select_rejects_bad_arguments(ops, dev):
    W = torch.randn(2000, device=dev)
    with pytest.raises(ops.CSError):
        ops.beam_select(W, 4)                        # C > 1024
    with pytest.raises(ops.CSError):
        ops.beam_select(W[:10], 11)                  # n_order > C
    with pytest.raises(ops.CSError):
        ops.beam_select(W[:10], 0)


def test_beam_step_partial_order_with_ties_and_nan(ops, dev):
    """Every candidate ties (constant rows, equal rewards) except a few NaN slots: the
    threshold-selection order must still be index order with NaN last."""
    A, B, K, V = 3, 8, 16, 2048
    x = torch.zeros(A * B, V, device=dev, dtype=torch.bfloat16)
    t = torch.randint(0, V, (B, K), device=dev, dtype=torch.int32)
    t[2, 5] = -1
    t[0, 0] = V + 3
    R = torch.zeros(A, B, device=dev)
    U, W, full, _ = ops.beam_step(x, t, R, "min")
    for n in (1, 7, 64, B * K):
        _, _, part, _ = ops.beam_step(x, t, R, "min", n_order=n)
        assert torch.equal(part, full[:n])
    ref = [c for c in range(B * K) if c not in (0, 2 * K + 5)] + [0, 2 * K + 5]
    assert full.cpu().tolist() == ref


@pytest.mark.parametrize("offset", [-1000.0, -3.0e6])
def test_beam_step_partial_order_clustered_rewards(ops, dev, offset):
    """Cumulative rewards far from zero put every welfare value in one exponent bin: the
    selection refines digit by digit and must still return the exact stable order."""
    A, B, K, V = 8, 16, 50, 4099
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(A * B, V, generator=g, device=dev) * 3.0
    t = torch.randint(0, V, (B, K), generator=g, device=dev, dtype=torch.int32)
    R = offset - torch.rand(A, B, generator=g, device=dev)
    _, W, full, _ = ops.beam_step(x, t, R, "min")
    o2, _ = ops.topk(W, B * K)
    assert torch.equal(full, o2)
    for n in (1, B, 100, 256):
        _, _, part, _ = ops.beam_step(x, t, R, "min", n_order=n)
        assert torch.equal(part, full[:n]), n


def test_vocab_topk_clustered_values(ops, orc, dev):
    """Logits that share one exponent (the histogram's first digit) and exact ties."""
    g = torch.Generator().manual_seed(9)
    x = 1000.0 + torch.randint(0, 50, (4, 30000), generator=g).float() / 64.0
    ids, vals = ops.vocab_topk(x.to(dev), 64)
    o_ids, o_vals = orc.vocab_topk(x.double().numpy(), 64)
    assert np.array_equal(ids.cpu().numpy(), o_ids)


@pytest.mark.parametrize("dtype,A,B,K,vocab,softcap,kind", [
    (torch.float32, 4, 4, 10, 128256, 0.0, "min"),      # C1
    (torch.bfloat16, 16, 16, 50, 256000, 30.0, "min"),  # C3
    (torch.bfloat16, 64, 8, 32, 128256, 0.0, "min"),    # C5
    (torch.bfloat16, 8, 3, 256, 70000, 0.0, "sum"),     # max K, split rows, fold path
    (torch.float16, 5, 2, 7, 777, 0.0, "max"),          # one proposer chunk
])
def test_beam_decode_step_is_topk_plus_beam_step(ops, dev, dtype, A, B, K, vocab, softcap, kind):
    """cs_beam_decode_step (proposer + scoring in one launch) is bit-identical to
    cs_vocab_topk followed by cs_beam_step, for full and partial orders and kept rewards."""
    g = torch.Generator(device=dev).manual_seed(A * 7 + B + K)
    ref = (torch.randn(B, vocab, generator=g, device=dev) * 3.0).to(dtype)
    ref[0, 11] = ref[0, 12] = ref[0].max()          # a tie at the top of beam 0
    x = (torch.randn(A * B, vocab, generator=g, device=dev) * 3.0).to(dtype)
    R = -torch.rand(A, B, generator=g, device=dev) * 30.0
    ids, _ = ops.vocab_topk(ref, K, softcap=softcap)
    U, W, o, v = ops.beam_step(x, ids, R, kind, softcap=softcap)
    for rep in range(2):   # the workspace is reused (counters left at zero)
        ids2, U2, W2, o2, v2 = ops.beam_decode_step(ref, x, R, K, kind, softcap=softcap)
        assert torch.equal(ids, ids2)
        assert torch.equal(torch.nan_to_num(U, nan=7.0), torch.nan_to_num(U2, nan=7.0))
        assert torch.equal(torch.nan_to_num(W, nan=7.0), torch.nan_to_num(W2, nan=7.0))
        assert torch.equal(o, o2)
    n = min(B, B * K)
    kept = torch.empty(A, n, device=dev) if B * K <= 1024 else None
    _, _, _, on, _ = ops.beam_decode_step(ref, x, R, K, kind, n_order=n, softcap=softcap,
                                          kept_out=kept)
    assert torch.equal(on, o[:n])
    if kept is not None:
        assert torch.equal(kept, U[:, on.long()])


@pytest.mark.parametrize("case", ["constant", "masked", "nan", "chunk_ties", "random"])
@pytest.mark.parametrize("K", [1, 10, 16])
def test_beam_decode_proposer_edge_rows(ops, orc, dev, case, K):
    """Small K takes the decode proposer's wave-bound selection (lane maxima -> per-wave
    k-th -> block bound -> rank the few keys above it), with the radix path as fallback
    for massive ties: constant rows, masked (-inf) rows with fewer finite values than K,
    NaN rows and ties straddling chunk boundaries give the oracle's ids and cs_vocab_topk's
    ids (radix path) exactly."""
    g = torch.Generator().manual_seed(17 + K)
    B, V, A = 3, 20000, 2
    ref = torch.randn(B, V, generator=g) * 3.0
    if case == "constant":
        ref[:] = 1.25
        ref[1, 5000:9000] = 0.0
    elif case == "masked":
        ref[:, 6:] = float("-inf")
        ref[2] = float("-inf")
    elif case == "nan":
        ref[0, ::3] = float("nan")
        ref[1, :] = float("nan")
        ref[1, 17] = 2.0
    elif case == "chunk_ties":
        ref[:] = -5.0
        for c in (4095, 4096, 8191, 8192, 12287, 19999, 1023, 1024, 2047):
            ref[:, c] = 7.0
    x = torch.randn(A * B, V, generator=g) * 3.0
    R = torch.zeros(A, B)
    ids, *_ = ops.beam_decode_step(ref.to(dev), x.to(dev), R.to(dev), K, "min")
    o_ids, _ = orc.vocab_topk(ref.double().numpy(), K)
    t_ids, _ = ops.vocab_topk(ref.to(dev), K)
    assert np.array_equal(ids.cpu().numpy(), o_ids)
    assert torch.equal(ids, t_ids)


def test_fused_beam_launches_stress_shared_workspace(ops, dev):
    """Hand-offs under repetition: 40 fused decode / beam launches of alternating shapes on
    ONE workspace (counters must return to zero every call), each checked word for word
    against the unfused kernels, with a large stream kernel queued in between so that the
    launches start on a busy device."""
    shapes = [(16, 16, 50, 64000, 30.0, torch.bfloat16), (64, 8, 32, 32000, 0.0, torch.bfloat16),
              (4, 4, 10, 128256, 0.0, torch.float32)]
    g = torch.Generator(device=dev).manual_seed(77)
    data = []
    for A, B, K, V, cap, dt in shapes:
        ref = (torch.randn(B, V, generator=g, device=dev) * 3.0).to(dt)
        x = (torch.randn(A * B, V, generator=g, device=dev) * 3.0).to(dt)
        ids, _ = ops.vocab_topk(ref, K, softcap=cap)
        data.append((A, B, K, cap, ref, x, ids))
    busy = torch.randn(8192, 32000, device=dev, dtype=torch.bfloat16)
    wd, wb = ops.Workspace(zeroed=True), ops.Workspace(zeroed=True)
    for it in range(40):
        A, B, K, cap, ref, x, ids = data[it % len(data)]
        R = -torch.rand(A, B, generator=g, device=dev) * (1 + it)
        ops.logsoftmax_gather(busy, None, want_lse=True)       # uneven load ahead
        U, W, o, _ = ops.beam_step(x, ids, R, "min", softcap=cap, workspace=wb)
        ids2, U2, W2, o2, _ = ops.beam_decode_step(ref, x, R, K, "min", softcap=cap,
                                                   workspace=wd, n_order=B * K if it % 2 else B)
        assert torch.equal(ids, ids2), it
        assert torch.equal(U, U2) and torch.equal(W, W2), it
        assert torch.equal(o[:o2.numel()], o2), it


def test_fused_beam_decode_graph_replays_stress(ops, dev):
    """The arrival-counter hand-offs under back-to-back hipGraph replays (no host gap between
    launches, the counters of one replay reset by its last arrivers just before the next
    replay's first arrivals): 300 replays of the C3-shaped decode step, every 50th compared
    word for word with the eager unfused kernels."""
    A, B, K, V, cap = 16, 16, 50, 64000, 30.0
    g = torch.Generator(device=dev).manual_seed(5)
    ref = (torch.randn(B, V, generator=g, device=dev) * 3.0).to(torch.bfloat16)
    x = (torch.randn(A * B, V, generator=g, device=dev) * 3.0).to(torch.bfloat16)
    R = -torch.rand(A, B, generator=g, device=dev) * 10.0
    ids, _ = ops.vocab_topk(ref, K, softcap=cap)
    U, W, o, _ = ops.beam_step(x, ids, R, "min", softcap=cap)
    ws = ops.Workspace(zeroed=True)
    out_ids = torch.empty(B, K, dtype=torch.int32, device=dev)
    out_o = torch.empty(B * K, dtype=torch.int32, device=dev)
    U2 = torch.empty(A, B * K, device=dev)
    W2 = torch.empty(B * K, device=dev)
    kw = dict(softcap=cap, workspace=ws, out_ids=out_ids, out_order=out_o, out_U=U2, out_W=W2)
    ops.beam_decode_step(ref, x, R, K, "min", **kw)           # sizes the workspace
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            ops.beam_decode_step(ref, x, R, K, "min", **kw)
    torch.cuda.current_stream().wait_stream(s)
    for it in range(300):
        graph.replay()
        if it % 50 == 49:
            torch.cuda.synchronize()
            assert torch.equal(ids, out_ids), it
            assert torch.equal(U, U2) and torch.equal(W, W2), it
            assert torch.equal(o, out_o), it
    assert int(ws.buf[:4096].count_nonzero()) == 0     # counters left at zero


def _fuzz_cases(n=24, seed=2024):
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(n):
        dtype = [torch.float32, torch.bfloat16, torch.float16][rng.integers(0, 3)]
        A = int(rng.integers(1, 40))
        B = int(rng.integers(1, 20))
        vocab = int(rng.choice([97, 1000, 4099, 33333, 70001, 128256]))
        K = int(min(rng.integers(1, 65), vocab, 16384 // B))
        softcap = float(rng.choice([0.0, 0.0, 30.0, 50.0])) if dtype != torch.float16 else 0.0
        kind = ["min", "min", "max", "sum", "sumlog"][rng.integers(0, 5)]
        pattern = ["randn", "ties", "masked"][rng.integers(0, 3)]
        cases.append((i, dtype, A, B, K, vocab, softcap, kind, pattern))
    return cases


@pytest.mark.parametrize("i,dtype,A,B,K,vocab,softcap,kind,pattern", _fuzz_cases())
def test_beam_decode_fuzz(ops, orc, dev, i, dtype, A, B, K, vocab, softcap, kind, pattern):
    """Seeded random shapes (dtype, agents, beams, K, vocab, soft-cap, welfare kind, tie /
    mask patterns): the fused decode step equals cs_vocab_topk + cs_beam_step bit for bit,
    its proposer equals the oracle's top-K, and its partial order + kept rewards equal the
    full order's prefix."""
    if A * B > 65536:
        pytest.skip("shape outside the launch limits")
    g = torch.Generator().manual_seed(1000 + i)
    ref = torch.randn(B, vocab, generator=g) * 3.0
    x = torch.randn(A * B, vocab, generator=g) * 3.0
    if pattern == "ties":
        ref = torch.round(ref)
        x = torch.round(x * 2) / 2
    elif pattern == "masked":
        m = torch.rand(B, vocab, generator=g) < 0.5
        ref[m] = float("-inf")
    ref, x = ref.to(dtype).to(dev), x.to(dtype).to(dev)
    R = (-torch.rand(A, B, generator=g) * 20.0).to(dev)
    ids, _ = ops.vocab_topk(ref, K, softcap=softcap)
    o_ids, _ = orc.vocab_topk(ref.double().cpu().numpy() if softcap == 0.0 else
                              (softcap * torch.tanh(ref.double().cpu() / softcap)).numpy(), K)
    U, W, o, _ = ops.beam_step(x, ids, R, kind, softcap=softcap)
    ids2, U2, W2, o2, _ = ops.beam_decode_step(ref, x, R, K, kind, softcap=softcap)
    assert torch.equal(ids, ids2)
    if softcap == 0.0:   # (soft-capped ties can merge differently in fp64 -> checked via ids)
        assert np.array_equal(ids.cpu().numpy(), o_ids)
    assert torch.equal(torch.nan_to_num(U, nan=7.0), torch.nan_to_num(U2, nan=7.0))
    assert torch.equal(torch.nan_to_num(W, nan=7.0), torch.nan_to_num(W2, nan=7.0))
    assert torch.equal(o, o2)
    n = min(B, B * K)
    kept = torch.empty(A, n, device=dev) if B * K <= 1024 else None
    _, _, _, on, _ = ops.beam_decode_step(ref, x, R, K, kind, n_order=n, softcap=softcap,
                                          kept_out=kept)
    assert torch.equal(on, o[:n])
    if kept is not None:
        assert torch.equal(kept, U[:, on.long()])
