"""CPU tests of the methods' HOST logic against the reference's golden traces.

The HIP kernels are not available on this CPU-only host, so these tests replace the
package's C-ABI ops *explicitly, inside the test* with the CPU oracle (test
infrastructure).  This checks everything around the kernels — prompt layouts, seed
schedules, tree order, dedupe/EOS walks, reward folding, selection — on the same
fixture model the reference traces were recorded with.  The product itself has no
CPU path: tests/test_methods_gpu.py replays the same traces through the real HIP
library on an MI355X.
"""
import importlib

import numpy as np
import pytest
import torch

import method_parity as mp

PKG = mp.PKG


@pytest.fixture(scope="module")
def emulated(orc):
    ops = importlib.import_module(PKG + ".ops")
    R = importlib.import_module(PKG + ".runtime")
    saved = {n: getattr(ops, n) for n in ("logsoftmax_gather", "segment_reduce", "welfare",
                                          "topk", "vocab_sample", "vocab_topk")}

    def lsg(logits, targets, *, vocab=None, softcap=0.0, workspace=None, want_lse=False, **kw):
        x = logits.detach().float().contiguous().numpy()
        t = targets.reshape(logits.shape[0], -1).numpy().astype(np.int32)
        tok, lse = orc.logsoftmax_gather(x, t, softcap=softcap, vocab=vocab)
        return torch.as_tensor(tok, dtype=torch.float32), torch.as_tensor(lse, dtype=torch.float32)

    def seg(tok, offsets):
        o = orc.segment_reduce(tok.double().numpy(), offsets.numpy())
        return {"sum_lp": torch.as_tensor(o["sum_lp"], dtype=torch.float32),
                "sum_p": torch.as_tensor(o["sum_p"], dtype=torch.float32),
                "count": torch.as_tensor(o["count"]),
                "last": torch.as_tensor(o["last"], dtype=torch.float32)}

    def wel(U, kind, *, eps=1e-9, nonfinite="skip", nan_val=-10.0, posinf_val=20.0,
            neginf_val=-20.0, out=None):
        code = {"min": orc.MIN, "egalitarian": orc.MIN, "sum": orc.SUM, "utilitarian": orc.SUM,
                "sumlog": orc.SUMLOG, "nash": orc.SUMLOG, "max": orc.MAX}[kind]
        W = orc.welfare(U.double().numpy(), code, eps=eps,
                        nonfinite=0 if nonfinite == "skip" else 1, nan_val=nan_val,
                        posinf_val=posinf_val, neginf_val=neginf_val)
        return torch.as_tensor(W, dtype=torch.float32)

    def tk(W, k, with_values=True):
        W32 = W.float().double().numpy()
        idx = orc.topk(W32, k)
        out = torch.as_tensor(idx)
        vals = torch.as_tensor(np.take_along_axis(np.atleast_2d(W32), idx, 1), dtype=torch.float32)
        return (out[0], vals[0]) if W.dim() == 1 else (out, vals)

    def vs(logits, seeds, *, temperature=1.0, vocab=None, softcap=0.0, workspace=None):
        x = logits.detach().float().double().numpy()
        sd = seeds.reshape(x.shape[0], -1).numpy().astype(np.int64)
        ids = np.zeros(sd.shape, dtype=np.int32)
        lps = np.zeros(sd.shape, dtype=np.float32)
        for r in range(sd.shape[0]):
            for d in range(sd.shape[1]):
                ids[r, d], lps[r, d] = orc.gumbel_sample(x[r], int(sd[r, d]) & ((1 << 64) - 1),
                                                         temperature)
        return torch.as_tensor(ids), torch.as_tensor(lps)

    def vt(logits, k, *, vocab=None, softcap=0.0, workspace=None):
        ids, vals = orc.vocab_topk(logits.detach().double().numpy(), k)
        return torch.as_tensor(ids), torch.as_tensor(vals, dtype=torch.float32)

    for n, f in (("logsoftmax_gather", lsg), ("segment_reduce", seg), ("welfare", wel),
                 ("topk", tk), ("vocab_sample", vs), ("vocab_topk", vt)):
        setattr(ops, n, f)
    traces = mp.load_traces()
    mp.register_fixture_engine(traces, torch.device("cpu"))
    yield traces
    for n, f in saved.items():
        setattr(ops, n, f)
    R.clear_engines()


def test_methods_match_reference_traces(emulated):
    failures = mp.check_methods(emulated)
    assert not failures, "\n".join(failures)


def test_evaluator_matches_reference(emulated):
    failures = mp.check_evaluations(emulated)
    assert not failures, "\n".join(failures)


def test_prompt_logprobs_match_reference(emulated):
    failures = mp.check_prompt_logprobs(emulated)
    assert not failures, "\n".join(failures)
