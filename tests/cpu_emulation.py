"""TEST INFRASTRUCTURE: CPU emulation of the package's C-ABI ops, backed by the oracle.

Used only by CPU tests that check HOST logic around the kernels (method control flow,
multi-rank welfare combination).  Installing it is explicit and reversible; the
product has no CPU path of its own.
"""
import importlib

import numpy as np
import torch

import oracle as orc

PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
NAMES = ("logsoftmax_gather", "segment_reduce", "welfare", "topk", "vocab_sample", "vocab_topk",
         "beam_step", "beam_decode_step", "beam_select")


def _lsg(logits, targets, *, vocab=None, softcap=0.0, workspace=None, want_lse=False, **kw):
    x = logits.detach().float().contiguous().numpy()
    t = targets.reshape(logits.shape[0], -1).numpy().astype(np.int32)
    tok, lse = orc.logsoftmax_gather(x, t, softcap=softcap, vocab=vocab)
    return torch.as_tensor(tok, dtype=torch.float32), torch.as_tensor(lse, dtype=torch.float32)


def _seg(tok, offsets):
    o = orc.segment_reduce(tok.double().numpy(), offsets.numpy())
    return {"sum_lp": torch.as_tensor(o["sum_lp"], dtype=torch.float32),
            "sum_p": torch.as_tensor(o["sum_p"], dtype=torch.float32),
            "count": torch.as_tensor(o["count"]),
            "last": torch.as_tensor(o["last"], dtype=torch.float32)}


def _wel(U, kind, *, eps=1e-9, nonfinite="skip", nan_val=-10.0, posinf_val=20.0,
         neginf_val=-20.0, out=None):
    code = {"min": orc.MIN, "egalitarian": orc.MIN, "sum": orc.SUM, "utilitarian": orc.SUM,
            "sumlog": orc.SUMLOG, "nash": orc.SUMLOG, "max": orc.MAX}[kind]
    W = orc.welfare(U.double().numpy(), code, eps=eps, nonfinite=0 if nonfinite == "skip" else 1,
                    nan_val=nan_val, posinf_val=posinf_val, neginf_val=neginf_val)
    return torch.as_tensor(W, dtype=torch.float32)


def _tk(W, k, with_values=True):
    W32 = W.float().double().numpy()
    idx = orc.topk(W32, k)
    out = torch.as_tensor(idx)
    vals = torch.as_tensor(np.take_along_axis(np.atleast_2d(W32), idx, 1), dtype=torch.float32)
    return (out[0], vals[0]) if W.dim() == 1 else (out, vals)


def _capped(logits, softcap):
    """The logits the kernels draw from: cap * tanh(x / cap) when soft-capped (Gemma-2)."""
    x = logits.detach().float().double().numpy()
    return softcap * np.tanh(x / softcap) if softcap and softcap > 0 else x


def _vs(logits, seeds, *, temperature=1.0, vocab=None, softcap=0.0, workspace=None):
    x = _capped(logits, softcap)
    sd = seeds.reshape(x.shape[0], -1).numpy().astype(np.int64)
    ids = np.zeros(sd.shape, dtype=np.int32)
    lps = np.zeros(sd.shape, dtype=np.float32)
    for r in range(sd.shape[0]):
        for d in range(sd.shape[1]):
            ids[r, d], lps[r, d] = orc.gumbel_sample(x[r], int(sd[r, d]) & ((1 << 64) - 1),
                                                     temperature)
    return torch.as_tensor(ids), torch.as_tensor(lps)


def _vt(logits, k, *, vocab=None, softcap=0.0, workspace=None):
    ids, vals = orc.vocab_topk(_capped(logits, softcap), k)
    return torch.as_tensor(ids), torch.as_tensor(vals, dtype=torch.float32)


def _bs(logits, targets, rewards, kind="min", *, n_order=None, vocab=None, softcap=0.0,
        eps=1e-9, workspace=None, kept_out=None):
    A, B = rewards.shape
    K = targets.shape[1]
    tok, _ = _lsg(logits, targets.repeat(A, 1), vocab=vocab, softcap=softcap)
    U = (rewards.float()[:, :, None] + tok.view(A, B, K)).reshape(A, B * K)
    W = _wel(U, kind, eps=eps)
    n = B * K if n_order is None else n_order
    if n == 0:
        return U, W, None, None
    order, val = _tk(W, n)
    if kept_out is not None:
        kept_out.copy_(U[:, order.long()])
    return U, W, order.to(torch.int32), val


def _bd(ref_logits, logits, rewards, k, kind="min", *, n_order=None, vocab=None, softcap=0.0,
        eps=1e-9, workspace=None, kept_out=None):
    ids, _ = _vt(ref_logits, k, vocab=vocab, softcap=softcap)
    ids = ids.to(torch.int32)
    U, W, order, val = _bs(logits, ids, rewards, kind, n_order=n_order, vocab=vocab,
                           softcap=softcap, eps=eps, kept_out=kept_out)
    return ids, U, W, order, val


def _sel(W, n_order, *, U=None, unfill=None, kept_out=None, W_out=None, with_values=False):
    fill = {None: None, "none": None, "+inf": np.inf, "min": np.inf, "-inf": -np.inf,
            "max": -np.inf}[unfill]
    Wn = W.clone()
    if fill is not None:
        Wn[Wn == fill] = float("nan")
    if W_out is not None:
        W_out.copy_(Wn)
    order, val = _tk(Wn, n_order)
    if kept_out is not None and U is not None:
        kept_out.copy_(U[:, order.long()])
    return order.to(torch.int32), (val if with_values else None)


_IMPL = {"beam_select": _sel, "logsoftmax_gather": _lsg, "segment_reduce": _seg, "welfare": _wel, "topk": _tk,
         "vocab_sample": _vs, "vocab_topk": _vt, "beam_step": _bs, "beam_decode_step": _bd}


def install():
    """Replace the ops with the emulation; returns the saved originals."""
    orc.lib()
    ops = importlib.import_module(PKG + ".ops")
    saved = {n: getattr(ops, n) for n in NAMES}
    for n in NAMES:
        setattr(ops, n, _IMPL[n])
    return saved


def uninstall(saved):
    ops = importlib.import_module(PKG + ".ops")
    for n, f in saved.items():
        setattr(ops, n, f)
