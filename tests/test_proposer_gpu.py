"""GPU parity of the candidate-proposer kernels (cs_vocab_topk, cs_vocab_sample)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,rows,vocab,k,softcap", [
    (torch.bfloat16, 4, 128256, 10, 0.0),     # C1/C3-style beam proposer, Llama vocab
    (torch.float32, 3, 256000, 50, 30.0),     # Gemma vocab + soft-cap, top-50
    (torch.bfloat16, 16, 5000, 256, 0.0),     # max k
    (torch.float32, 2, 4096, 1, 0.0),         # greedy
    (torch.float16, 1, 77, 77, 0.0),          # k = vocab, single partial chunk
])
def test_vocab_topk_matches_oracle(ops, orc, dev, dtype, rows, vocab, k, softcap):
    g = torch.Generator().manual_seed(vocab + k)
    x = torch.round(torch.randn(rows, vocab, generator=g) * 4) / 2   # heavy ties
    x = x.to(dtype)
    ids, vals = ops.vocab_topk(x.to(dev), k, softcap=softcap)
    xf = x.float().double().numpy()
    if softcap:
        xf = softcap * np.tanh(xf / softcap)
        # the kernel computes the cap in fp32; compare ids on the fp32-capped values
        xf = (softcap * torch.tanh(x.float() / softcap)).double().numpy()
    o_ids, o_vals = orc.vocab_topk(xf, k)
    got = ids.cpu().numpy()
    if softcap:
        # fp32 tanh of the kernel vs torch may split a tie: require identical value multisets
        np.testing.assert_allclose(np.sort(vals.cpu().numpy(), 1), np.sort(o_vals, 1), atol=1e-5)
    else:
        assert np.array_equal(got, o_ids)
        np.testing.assert_array_equal(vals.cpu().numpy(), o_vals.astype(np.float32))


@pytest.mark.parametrize("case", ["constant", "masked", "nan", "chunk_ties", "gemma_c3"])
def test_vocab_topk_edge_rows(ops, orc, dev, case):
    """Rows that defeat the histogram threshold (massive ties -> full-sort fallback) or
    carry -inf / NaN, and ties straddling the 4096-element chunk boundaries."""
    g = torch.Generator().manual_seed(7)
    rows, V, k, cap = 3, 20000, 40, 0.0
    x = torch.randn(rows, V, generator=g) * 3.0
    if case == "constant":
        x[:] = 1.25
        x[1, 5000:9000] = 0.0             # a row whose chunks are partly constant
    elif case == "masked":
        x[:, 100:] = float("-inf")        # logit-bias mask: fewer finite values than k
        x[2] = float("-inf")
    elif case == "nan":
        x[0, ::3] = float("nan")
        x[1, :] = float("nan")
        x[1, 17] = 2.0
    elif case == "chunk_ties":
        x[:] = -5.0
        for c in (4095, 4096, 8191, 8192, 12287, 19999):
            x[:, c] = 7.0
    elif case == "gemma_c3":
        rows, V, k, cap = 16, 256000, 50, 30.0
        x = torch.randn(rows, V, generator=g) * 3.0
    xd = x.to(torch.bfloat16 if case == "gemma_c3" else torch.float32)
    ids, vals = ops.vocab_topk(xd.to(dev), k, softcap=cap)
    xf = xd.float()
    if cap:
        xf = cap * torch.tanh(xf / cap)
    o_ids, o_vals = orc.vocab_topk(xf.double().numpy(), k)
    if cap:   # fp32 tanh of the kernel vs torch: compare value multisets, then ids by value
        np.testing.assert_allclose(vals.cpu().numpy(), o_vals, atol=1e-5)
    else:
        assert np.array_equal(ids.cpu().numpy(), o_ids)
        np.testing.assert_array_equal(vals.cpu().numpy(), o_vals.astype(np.float32))


def test_vocab_sample_matches_oracle(ops, orc, dev):
    rng = np.random.default_rng(12)
    rows, V, n_draw = 6, 50000, 8
    x = torch.as_tensor(rng.normal(size=(rows, V)).astype(np.float32) * 2.5)
    seeds = torch.as_tensor(rng.integers(0, 2**62, size=(rows, n_draw)), dtype=torch.int64)
    ids, lp = ops.vocab_sample(x.to(dev), seeds.to(dev))
    ids, lp = ids.cpu().numpy(), lp.cpu().numpy()
    mism = 0
    for r in range(rows):
        for d in range(n_draw):
            i, l = orc.gumbel_sample(x[r].numpy(), int(seeds[r, d]))
            if ids[r, d] != i:
                mism += 1
            else:
                assert abs(lp[r, d] - l) < 1e-3
    assert mism == 0


def test_vocab_sample_temperature_and_bf16(ops, orc, dev):
    rng = np.random.default_rng(13)
    rows, V = 3, 128256
    xb = torch.as_tensor(rng.normal(size=(rows, V)).astype(np.float32) * 3).to(torch.bfloat16)
    seeds = torch.arange(rows * 4, dtype=torch.int64).reshape(rows, 4) * 7919 + 5
    ids, lp = ops.vocab_sample(xb.to(dev), seeds.to(dev), temperature=0.7)
    xf = xb.float().numpy()
    for r in range(rows):
        for d in range(4):
            i, l = orc.gumbel_sample(xf[r], int(seeds[r, d]), temperature=0.7)
            assert ids[r, d].item() == i
            assert abs(lp[r, d].item() - l) < 1e-3


def test_vocab_sample_distribution(ops, dev):
    """Gumbel-max draws follow softmax(x): empirical frequencies over many seeds."""
    V = 16
    x = torch.linspace(-2, 2, V)
    rows = 4096
    seeds = torch.arange(rows * 16, dtype=torch.int64).reshape(rows, 16)
    ids, _ = ops.vocab_sample(x.repeat(rows, 1).to(dev), seeds.to(dev))
    freq = torch.bincount(ids.reshape(-1).long().cpu(), minlength=V).double() / ids.numel()
    p = torch.softmax(x.double(), 0)
    assert torch.max(torch.abs(freq - p)).item() < 0.01
