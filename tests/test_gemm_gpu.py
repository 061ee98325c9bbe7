"""cs_gemm_bf16 (csrc/gemm.hip) on the MI355X: the decode-step projection GEMM against an
fp32 product of the same bf16 operands (a floating-point kernel: torch fp32 is its
reference, SURVEY.md §8(d) "parity gates"), the gated gate|up form against cs_gated_act of
the rounded GEMM halves, K splits against no split, and bitwise run-to-run determinism.

Tolerance: |y - ref| <= 2^-7 |ref| + 1e-3 * max|ref| — one bf16 rounding of the output
(relative 2^-8) plus fp32 accumulation-order differences over K <= 14336."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [
    # M, N, K            what it covers
    (1, 128, 64),        # one row, one K step, one tile
    (20, 3072, 2048),    # C1 q|k|v (one 32-row block)
    (33, 256, 192),      # ragged rows (padded rows of the last tile dropped), K = 3 steps
    (272, 8192, 3584),   # C3 q|k|v: 17 row tiles, split K
    (272, 3584, 14336),  # C3 down: long K, split K
    (300, 384, 640),     # > 288 rows: two row blocks
    (520, 1024, 1024),   # C5 row count: two row blocks
]


def _tol(ref):
    return ref.abs() * 2.0 ** -7 + 1e-3 * ref.abs().max()


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_matches_fp32_product(ops, dev, M, N, K, variant):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    ref = x.float() @ w.float().t()
    if variant in (2, 4) and N % 256:
        pytest.skip("256-column tiles")
    y = ops.gemm(x, w, variant=variant)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert torch.all((y.float() - ref).abs() <= _tol(ref)), (y.float() - ref).abs().max().item()
    # every K split gives the same result up to accumulation order, and each is reproducible
    for sp in (1, 2, 4):
        if K % (64 * sp):
            continue
        a = ops.gemm(x, w, splits=sp, variant=variant)
        b = ops.gemm(x, w, splits=sp, variant=variant)
        assert torch.equal(a, b), f"splits={sp} not bitwise reproducible"
        assert torch.all((a.float() - ref).abs() <= _tol(ref)), sp


def test_gemm_strided_operands_and_out(ops, dev):
    """x a column slice of a wider buffer (ld > K), out a slice of a wider buffer."""
    M, N, K = 40, 256, 128
    big = torch.randn(M, K + 64, device=dev).to(torch.bfloat16)
    x = big[:, :K]
    w = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
    ob = torch.zeros(M, N + 128, device=dev, dtype=torch.bfloat16)
    ops.gemm(x, w, out=ob[:, :N])
    ref = x.float() @ w.float().t()
    assert torch.all((ob[:, :N].float() - ref).abs() <= _tol(ref))
    assert torch.all(ob[:, N:] == 0)


@pytest.mark.parametrize("col0", [0, 4])
def test_gemm_split_k_into_strided_out(ops, dev, col0):
    """A K split folds its partials with 16-byte stores: an out whose rows are only 8-byte
    aligned (ld % 8 == 4, or a 4-column offset) must still get the split's exact result."""
    M, N, K = 24, 256, 512
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.1).to(dev, torch.bfloat16)
    want = ops.gemm(x, w, splits=4, variant=2)
    ob = torch.zeros(M, N + 132, device=dev, dtype=torch.bfloat16)     # ld % 8 == 4
    view = ob[:, col0:col0 + N]
    ops.gemm(x, w, splits=4, variant=2, out=view)
    assert torch.equal(view, want)
    assert torch.all(ob[:, :col0] == 0) and torch.all(ob[:, col0 + N:] == 0)


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
@pytest.mark.parametrize("M,F,K", [(20, 512, 256), (272, 1024, 448), (300, 256, 128),
                                   # 2F % 256 != 0: variant 3's 128-row (64-feature) gated
                                   # tiles; variants 2 / 4 resolve to variant 1 there
                                   (48, 192, 512)])
def test_gated_gemm_equals_gemm_then_gated_act(ops, dev, act, M, F, K, variant):
    """gated = 1 is act(gate) * up of the ROUNDED GEMM halves with cs_gated_act's rounding:
    bitwise equal to cs_gated_act applied to the unsplit cs_gemm output.  Variant 3 is the
    four-wave gated form (64 gate + 64 up features per workgroup) the dispatch table runs
    for the C1 / per-rank C3 gate|up projections."""
    g = torch.Generator(device="cpu").manual_seed(F + K)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(2 * F, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    gu = ops.gemm(x, w, splits=1)
    want = ops.gated_act(gu[:, :F], gu[:, F:], act)
    got = ops.gemm(x, w, gated=True, act=act, variant=variant)
    assert got.shape == (M, F)
    assert torch.equal(got, want)


THIN_SHAPES = [
    # M, N, K            what it covers
    (1, 128, 64),        # one row, one K step: 7 of the 8 waves have no step
    (5, 256, 640),       # 10 K steps over 8 / 16 waves (uneven slices)
    (20, 3072, 2048),    # C1 q|k|v
    (48, 3584, 4096),    # C3 output projection at 8 ranks
    (72, 1024, 8192),    # C5's 8-rank row count, long K
    (80, 384, 14336),    # the thin form's row limit, C3 down's K
]


@pytest.mark.parametrize("variant", [5, 6, 7])
@pytest.mark.parametrize("M,N,K", THIN_SHAPES)
def test_thin_gemm_matches_fp32_product(ops, dev, M, N, K, variant):
    """Variants 5-7 (M <= 80: each wave streams its own K slice, waves folded in order)."""
    g = torch.Generator(device="cpu").manual_seed(M * 11 + N + K)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    ref = x.float() @ w.float().t()
    y = ops.gemm(x, w, variant=variant)
    assert y.shape == (M, N)
    assert torch.all((y.float() - ref).abs() <= _tol(ref)), (y.float() - ref).abs().max().item()
    assert torch.equal(y, ops.gemm(x, w, variant=variant)), "not bitwise reproducible"


@pytest.mark.parametrize("variant", [5, 7])
@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
@pytest.mark.parametrize("M,F,K", [(20, 512, 256), (48, 1024, 448), (72, 256, 1024)])
def test_thin_gated_gemm_equals_thin_gemm_then_gated_act(ops, dev, act, M, F, K, variant):
    """The thin gated form rounds the same fp32 sums as the thin plain form with the same
    wave count (16 waves only up to 3 row tiles, else 8), then applies cs_gated_act."""
    g = torch.Generator(device="cpu").manual_seed(F + K + M)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(2 * F, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    plain = variant if (variant != 7 or M <= 48) else 5
    gu = ops.gemm(x, w, variant=plain)
    want = ops.gated_act(gu[:, :F], gu[:, F:], act)
    got = ops.gemm(x, w, gated=True, act=act, variant=variant)
    assert torch.equal(got, want)


def test_thin_gemm_rejects_more_than_80_rows(ops, dev):
    x = torch.zeros(81, 128, device=dev, dtype=torch.bfloat16)
    w = torch.zeros(128, 128, device=dev, dtype=torch.bfloat16)
    with pytest.raises(ops.CSError):
        ops.gemm(x, w, variant=5)


@pytest.mark.parametrize("variant", [2, 3, 4])
@pytest.mark.parametrize("M,N,K,gated", [
    (20, 3072, 2048, 0), (48, 3584, 4096, 0), (72, 1024, 8192, 0), (272, 8192, 3584, 0),
    (300, 512, 640, 0), (48, 1024, 448, 1), (272, 2048, 512, 1),
    # 65-80 rows: the packed launch takes a 5-tile row block, the unpacked one 8 tiles
    (65, 1024, 512, 0), (72, 2048, 1024, 1),
    # packed gated, <= 80 rows, 2F % 224 == 0: the 7-wave form (112 features per workgroup),
    # bitwise the unpacked 8-wave kernel -- one row block of 2, 4 and 5 tiles
    (20, 3584, 256, 1), (48, 1792, 512, 1), (72, 1792, 1024, 1), (80, 3584, 192, 1),
])
def test_packed_weight_gemm_is_bitwise_the_unpacked(ops, dev, M, N, K, gated, variant):
    """cs_gemm_pack + cs_gemm_bf16_packed: the same fragments reach the same MFMAs, only
    their addresses change -- bitwise the unpacked cs_gemm_bf16, for every K split."""
    if variant in (2, 4) and N % 256:
        pytest.skip("256-column tiles")
    g = torch.Generator(device="cpu").manual_seed(M + N + K + gated)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    pw = ops.gemm_pack(w)
    for sp in ((1,) if gated else (0, 1, 2, 4)):
        if sp > 1 and K % (64 * sp):
            continue
        want = ops.gemm(x, w, gated=bool(gated), splits=sp, variant=variant)
        got = ops.gemm_packed(x, pw, gated=bool(gated), splits=sp, variant=variant)
        assert torch.equal(got, want), sp


def test_gemm_pack_is_the_documented_permutation(ops, dev):
    N, K = 32, 128
    w = torch.arange(N * K, device=dev, dtype=torch.float32).view(N, K).to(torch.bfloat16)
    p = ops.gemm_pack(w).data.view(-1)
    T, s, h, lane, e = 1, 1, 1, 37, 5
    at = ((T * (K // 64) + s) * 2 + h) * 512 + 8 * lane + e
    assert p[at] == w[16 * T + lane % 16, 64 * s + 32 * h + 8 * (lane // 16) + e]
    assert torch.equal(p.sort().values, w.view(-1).sort().values)


def test_linear_runs_the_packed_copy_where_the_table_says_so(ops, dev):
    """ops.linear with a cs_gemm_pack'ed copy takes the table's packed entry (plain, gated and
    the unfolded K-split partials), bitwise the unpacked kernel of the same variant / split;
    without the copy the unpacked entry; gemm_packs names the packed weights."""
    M, N, K = 48, 1024, 512
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    pw = ops.gemm_pack(w)
    table = {f"{M},{N},{K},0": {"variant": 3, "splits": 2, "packed": {"variant": 3, "splits": 2}},
             f"{M},{N},{K},1": {"packed": {"variant": 2, "splits": 1}}}
    saved = ops._gemm_table
    ops._gemm_table = table
    try:
        assert ops.gemm_choice(M, N, K)["packed"] is False
        assert ops.gemm_choice(M, N, K, packed=True)["packed"] is True
        assert ops.gemm_choice(M, N, K, True) is None            # no unpacked gated entry
        assert ops.gemm_packs(N, K) and ops.gemm_packs(N, K, True) and not ops.gemm_packs(N, 2 * K)
        assert torch.equal(ops.linear(x, w, packed=pw), ops.linear(x, w))
        assert torch.equal(ops.linear(x, w, fold=False, packed=pw).part,
                           ops.linear(x, w, fold=False).part)
        got = ops.linear(x, w, gated=True, act="silu", packed=pw)
        assert torch.equal(got, ops.gemm(x, w, gated=True, act="silu", variant=2))
        # no gated entry: the plain GEMM's packed entry + cs_gated_act
        del table[f"{M},{N},{K},1"]
        got = ops.linear(x, w, gated=True, act="silu", packed=pw)
        gu = ops.gemm_packed(x, pw, splits=2, variant=3)
        assert torch.equal(got, ops.gated_act(gu[:, :N // 2], gu[:, N // 2:], "silu"))
    finally:
        ops._gemm_table = saved


def test_gemm_rejects_unsupported_shapes(ops, dev):
    x = torch.zeros(4, 100, device=dev, dtype=torch.bfloat16)
    w = torch.zeros(128, 100, device=dev, dtype=torch.bfloat16)
    assert not ops.gemm_ok(x, w)
    with pytest.raises(ops.CSError):
        ops.gemm(x, w)


@pytest.mark.parametrize("M,d,K,splits,variant", [(272, 3584, 2048, 8, 3), (37, 2048, 1024, 2, 2),
                                                  (72, 8192, 1024, 4, 4), (520, 8192, 1024, 4, 2),
                                                  # d = 8192 (1024-thread rows) with > 8 splits:
                                                  # the two 8-split batches of the fold
                                                  (72, 8192, 2048, 16, 2), (48, 8192, 1536, 12, 2)])
@pytest.mark.parametrize("plus_one,post_norm", [(False, False), (True, True)])
def test_split_partials_folded_by_add_rms_norm_is_bitwise(ops, dev, M, d, K, splits, variant,
                                                          plus_one, post_norm):
    """cs_gemm_bf16(y = NULL) + cs_add_rms_norm_splitk == cs_gemm_bf16's own fold followed by
    cs_add_rms_norm (the down projection + residual add of a decode step), bit for bit."""
    g = torch.Generator(device="cpu").manual_seed(M + d + splits)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(d, K, generator=g) * 0.05).to(dev, torch.bfloat16)
    a = (torch.randn(M, d, generator=g) * 2).to(dev, torch.bfloat16)
    wt = (torch.randn(d, generator=g) * 0.1).to(dev, torch.bfloat16)
    wb = (torch.randn(d, generator=g) * 0.1).to(dev, torch.bfloat16) if post_norm else None
    y = ops.gemm(x, w, splits=splits, variant=variant)
    a_ref, a_got = a.clone(), a.clone()
    ref = ops.add_rms_norm(a_ref, wt, 1e-6, b=y, b_weight=wb, s_out=a_ref, plus_one=plus_one)
    part = ops.gemm_partials(x, w, splits=splits, variant=variant)
    assert tuple(part.part.shape) == (splits, M, d)
    got = ops.add_rms_norm(a_got, wt, 1e-6, b=part, b_weight=wb, s_out=a_got, plus_one=plus_one)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert torch.equal(a_got, a_ref)


def _table_keys():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd",
                        "tuned", "gemm_dispatch_mi355x.json")
    with open(path) as f:
        return sorted(json.load(f)["table"], key=lambda k: [int(v) for v in k.split(",")])


@pytest.mark.parametrize("key", _table_keys())
def test_every_dispatched_production_shape_matches_fp32_product(ops, dev, key):
    """Every shape the committed dispatch table routes onto cs_gemm (the production decode
    GEMMs of C1-C5 at 1 GPU and per rank at 8: e.g. the 70B per-rank gate|up 72 x 57,344 x
    8,192 in the 7-wave packed gated form, its down 72 x 8,192 x 28,672, Gemma-2's per-rank
    gate|up 48 x 28,672 x 3,584, the 520-row C5 shapes, the LM heads), through ops.linear as
    the model calls it -- with and without the packed copy -- against the fp32 product of
    the same bf16 operands.  Plain: |y - ref| <= 2^-7 |ref| + 1e-3 max|ref| (one bf16
    rounding + accumulation order, _tol); gated: act(gate) * up of the ROUNDED halves, so
    three bf16 roundings (gate, up, product): 2^-6 |ref| + 2e-3 max|ref|."""
    M, N, K, gated = (int(v) for v in key.split(","))
    gated = bool(gated)
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    if gated:
        F_ = N // 2
        ref = torch.nn.functional.silu(ref[:, :F_]) * ref[:, F_:]
        tol = ref.abs() * 2.0 ** -6 + 2e-3 * ref.abs().max()
    else:
        tol = _tol(ref)
    pw = ops.gemm_pack(w) if ops.gemm_choice(M, N, K, gated, packed=True) is not None else None
    routes = {"unpacked": ops.linear(x, w, gated=gated, act="silu")}
    if pw is not None:
        routes["packed"] = ops.linear(x, w, gated=gated, act="silu", packed=pw)
    del w
    for name, y in routes.items():
        assert y.shape == ref.shape, name
        err = (y.float() - ref).abs()
        assert bool((err <= tol).all()), (name, float(err.max()), float(ref.abs().max()))
