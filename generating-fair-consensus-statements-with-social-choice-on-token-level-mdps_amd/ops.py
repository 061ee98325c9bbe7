"""Torch-tensor front end of the C-ABI (``include/consensus_scoring.h``).

Every function here launches a hand-written gfx950 kernel through
``libconsensus_scoring.so`` on torch's *current* HIP stream and returns device
tensors.  Inputs must already live on the GPU; nothing is copied to the host and
nothing falls back to a CPU path (a missing library raises ``CSError``).

Reference semantics each op restates are cited on the op.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import json
import os
import threading
from typing import Dict, NamedTuple, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import CSError

WELFARE = {"min": _lib.WELFARE_MIN, "egalitarian": _lib.WELFARE_MIN,
           "sum": _lib.WELFARE_SUM, "utilitarian": _lib.WELFARE_SUM,
           "sumlog": _lib.WELFARE_SUMLOG, "nash": _lib.WELFARE_SUMLOG,
           "max": _lib.WELFARE_MAX}

# CS_DEBUG_TABLES=1: the row-layout history's slot tables are checked on the host against
# the K / V buffer they index before every (uncaptured) launch that reads them (read once)
_DEBUG_TABLES = os.environ.get("CS_DEBUG_TABLES") == "1"
_DTYPE = {torch.float32: _lib.CS_F32, torch.bfloat16: _lib.CS_BF16, torch.float16: _lib.CS_F16}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _require_cuda(*ts: torch.Tensor) -> None:
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise CSError("consensus_scoring ops take device tensors (got a CPU tensor); "
                          "there is no CPU path")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise CSError(f"tensors on different devices: {dev} vs {t.device}")


class Workspace:
    """Grow-only device scratch for split-V partials (allocation happens here, never
    inside a launch, so a captured graph can reuse a pre-sized workspace).

    ``zeroed=True`` allocates zero-filled memory: cs_beam_step keeps arrival counters in
    its workspace that must start at zero (every call leaves them at zero again)."""

    def __init__(self, zeroed: bool = False) -> None:
        self.buf: Optional[torch.Tensor] = None
        self.zeroed = zeroed

    def get(self, nbytes: int, device: torch.device) -> Optional[torch.Tensor]:
        if nbytes == 0:
            return None
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != device:
            alloc = torch.zeros if self.zeroed else torch.empty
            self.buf = alloc(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        return self.buf

    def reset(self) -> None:
        """Zero a zeroed workspace again (its arrival counters), e.g. after a failed launch
        that may have stopped with counters half-counted."""
        if self.zeroed and self.buf is not None and not torch.cuda.is_current_stream_capturing():
            self.buf.zero_()


_default_ws: dict = {}
_beam_ws: dict = {}
_decode_ws: dict = {}


def workspace_size(rows: int, vocab: int, k: int = 1) -> int:
    return int(_lib.load().cs_workspace_size(rows, vocab, k))


def logsoftmax_gather(logits: torch.Tensor, targets: Optional[torch.Tensor], *, vocab: Optional[int] = None,
                      softcap: float = 0.0, out: Optional[torch.Tensor] = None,
                      lse_out: Optional[torch.Tensor] = None, want_lse: bool = False,
                      workspace: Optional[Workspace] = None):
    """Fused log-softmax over the vocab + gather at ``targets``.

    logits  [rows, ld] bf16/f16/f32 with unit column stride (only the first
            ``vocab`` columns are used); targets [rows, k] int32 (ids outside
            [0, vocab) give NaN, the reference's ``None``).
    Returns (tok_lp [rows, k] f32, lse [rows] f32 or None).

    Restates: remote echo=True prompt log-probs read by get_prompt_logprobs
    (src/utils.py:249-263); core.log_softmax_rows + gather (core.py:64-68, 89-90).
    """
    L = _lib.load()
    if logits.dim() != 2 or logits.stride(1) != 1:
        raise CSError("logits must be 2-D with unit column stride")
    if logits.dtype not in _DTYPE:
        raise CSError(f"unsupported logits dtype {logits.dtype}")
    rows, ld = logits.shape[0], logits.stride(0) if logits.shape[0] > 1 else logits.shape[1]
    vocab = logits.shape[1] if vocab is None else int(vocab)
    if vocab > logits.shape[1]:
        raise CSError("vocab exceeds logits width")
    if targets is None:
        k = 0
        targets = torch.empty((rows, 0), dtype=torch.int32, device=logits.device)
    else:
        if targets.dtype != torch.int32:
            raise CSError("targets must be int32")
        if targets.dim() != 2 or targets.shape[0] != rows:
            if rows == 0 or targets.numel() % rows != 0:
                raise CSError("targets must be [rows, k]")
            targets = targets.reshape(rows, -1)
        if not targets.is_contiguous():
            targets = targets.contiguous()
        k = targets.shape[1]
    _require_cuda(logits, targets, out, lse_out)
    if out is None:
        out = torch.empty((rows, k), dtype=torch.float32, device=logits.device)
    elif out.dtype != torch.float32 or not out.is_contiguous() or out.numel() != rows * k:
        raise CSError("out must be contiguous float32 with rows*k elements")
    if lse_out is None and want_lse:
        lse_out = torch.empty(rows, dtype=torch.float32, device=logits.device)
    nbytes = workspace_size(rows, vocab, k)
    if workspace is None:
        workspace = _default_ws.setdefault(logits.device, Workspace())
    ws = workspace.get(nbytes, logits.device)
    rc = L.cs_logsoftmax_gather(
        logits.data_ptr(), _DTYPE[logits.dtype], rows, vocab, ld,
        targets.data_ptr() if k else None, k, float(softcap), out.data_ptr() if k else None,
        lse_out.data_ptr() if lse_out is not None else None,
        ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0, _stream())
    _lib.check(rc, "cs_logsoftmax_gather")
    return out, lse_out


def segment_reduce(tok_lp: torch.Tensor, offsets: torch.Tensor):
    """Per-segment Σlp, Σexp(lp), count of non-NaN, last value (fp64 accumulation).

    Restates best_of_n.py:303-305, finite_lookahead.py:508-520, evaluation.py:203-213,
    beam_search.py:389-390 and core.py:90.
    """
    L = _lib.load()
    tok = tok_lp.reshape(-1)
    if tok.dtype != torch.float32 or not tok.is_contiguous():
        raise CSError("tok_lp must be contiguous float32")
    if offsets.dtype != torch.int32 or offsets.dim() != 1 or not offsets.is_contiguous():
        raise CSError("offsets must be a contiguous 1-D int32 tensor")
    _require_cuda(tok, offsets)
    n_seg = offsets.numel() - 1
    dev = tok.device
    sum_lp = torch.empty(n_seg, dtype=torch.float32, device=dev)
    sum_p = torch.empty(n_seg, dtype=torch.float32, device=dev)
    cnt = torch.empty(n_seg, dtype=torch.int32, device=dev)
    last = torch.empty(n_seg, dtype=torch.float32, device=dev)
    rc = L.cs_segment_reduce(tok.data_ptr(), tok.numel(), offsets.data_ptr(), n_seg,
                             sum_lp.data_ptr(), sum_p.data_ptr(), cnt.data_ptr(), last.data_ptr(),
                             _stream())
    _lib.check(rc, "cs_segment_reduce")
    return {"sum_lp": sum_lp, "sum_p": sum_p, "count": cnt, "last": last}


def welfare(U: torch.Tensor, kind, *, eps: float = 1e-9, nonfinite: str = "skip",
            nan_val: float = -10.0, posinf_val: float = 20.0, neginf_val: float = -20.0,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Welfare over agents (rows of U [A, C]) for every candidate column.

    kind: 'min'|'egalitarian', 'sum'|'utilitarian', 'sumlog'|'nash', 'max'.
    Restates evaluation.py:337-381, beam_search.py:558-560, best_of_n.py:384-408,
    core.py:108-113 (point mass) and core.py:374.
    """
    L = _lib.load()
    if isinstance(kind, str):
        kind = WELFARE[kind]
    if U.dim() != 2 or U.dtype != torch.float32 or (U.stride(1) != 1 and U.shape[1] > 1):
        raise CSError("U must be 2-D float32 with unit column stride")
    _require_cuda(U, out)
    A, C = U.shape
    ldu = U.stride(0) if A > 1 else C
    if out is None:
        out = torch.empty(C, dtype=torch.float32, device=U.device)
    mode = {"skip": _lib.NONFINITE_SKIP, "replace": _lib.NONFINITE_REPLACE}[nonfinite]
    rc = L.cs_welfare_reduce(U.data_ptr(), A, C, ldu, int(kind), float(eps), mode, float(nan_val),
                             float(posinf_val), float(neginf_val), out.data_ptr(), _stream())
    _lib.check(rc, "cs_welfare_reduce")
    return out


def topk(W: torch.Tensor, k: int, *, with_values: bool = True):
    """Stable descending top-k per row of W [n_seg, seg_len] (value desc, index asc;
    NaN last).  Restates beam_search.py:558-560 (stable sorted, reverse=True),
    best_of_n.py:198 (np.argmax) and finite_lookahead.py:527 (max, first wins)."""
    L = _lib.load()
    W2 = W.reshape(1, -1) if W.dim() == 1 else W
    if W2.dim() != 2 or W2.dtype != torch.float32 or W2.stride(1) != 1:
        raise CSError("W must be float32 with unit column stride")
    _require_cuda(W2)
    n_seg, seg_len = W2.shape
    ld = W2.stride(0) if n_seg > 1 else seg_len
    idx = torch.empty((n_seg, k), dtype=torch.int32, device=W.device)
    val = torch.empty((n_seg, k), dtype=torch.float32, device=W.device) if with_values else None
    rc = L.cs_segmented_topk(W2.data_ptr(), n_seg, seg_len, ld, int(k), idx.data_ptr(),
                             val.data_ptr() if val is not None else None, _stream())
    _lib.check(rc, "cs_segmented_topk")
    if W.dim() == 1:
        return idx[0], (val[0] if val is not None else None)
    return idx, val


UNFILL = {None: 0, "none": 0, "+inf": 1, "min": 1, "-inf": 2, "max": 2}


def beam_select(W: torch.Tensor, n_order: int, *, U: Optional[torch.Tensor] = None,
                unfill=None, kept_out: Optional[torch.Tensor] = None, W_out: Optional[torch.Tensor] = None,
                with_values: bool = False):
    """Selection half of an agent-sharded beam step, one launch (cs_beam_select).

    W [C] float32 all-reduced welfare (C <= 1024); unfill '+inf'/'min' maps +inf back to
    NaN (the MIN combine's fill for columns without a usable utility), '-inf'/'max' -inf.
    Returns (order [n_order] int32 by (W desc, index asc), NaN last; values or None).
    With U [A, C] (this rank's agents) and kept_out [A, n_order]: kept_out[a, r] =
    U[a, order[r]], the kept beams' cumulative rewards.  W_out (nullable) receives W after
    unfill.  Bit-identical to topk(W) + U.index_select(1, order).
    Restates the stable sort + keep of beam_search.py:558-593 on one agent shard."""
    L = _lib.load()
    if W.dim() != 1 or W.dtype != torch.float32 or not W.is_contiguous():
        raise CSError("W must be a contiguous 1-D float32 tensor")
    _require_cuda(W)
    C = W.shape[0]
    A = 0
    if kept_out is not None:
        if U is None or U.dtype != torch.float32 or not U.is_contiguous() or U.dim() != 2 \
                or U.shape[1] != C:
            raise CSError("kept_out needs U [A, C] contiguous float32")
        A = U.shape[0]
        if kept_out.shape != (A, n_order) or kept_out.dtype != torch.float32 \
                or not kept_out.is_contiguous():
            raise CSError("kept_out must be [A, n_order] contiguous float32")
    order = torch.empty(n_order, dtype=torch.int32, device=W.device)
    val = torch.empty(n_order, dtype=torch.float32, device=W.device) if with_values else None
    rc = L.cs_beam_select(W.data_ptr(), C, UNFILL[unfill], U.data_ptr() if A else None, A,
                          int(n_order), W_out.data_ptr() if W_out is not None else None,
                          order.data_ptr(), val.data_ptr() if val is not None else None,
                          kept_out.data_ptr() if kept_out is not None else None, _stream())
    _lib.check(rc, "cs_beam_select")
    return order, val


def beam_step(logits: torch.Tensor, targets: torch.Tensor, rewards: torch.Tensor, kind="min", *,
              n_order: Optional[int] = None, vocab: Optional[int] = None, softcap: float = 0.0,
              eps: float = 1e-9, workspace: Optional[Workspace] = None,
              kept_out: Optional[torch.Tensor] = None,
              out_U: Optional[torch.Tensor] = None, out_W: Optional[torch.Tensor] = None):
    """One beam-search scoring step after the LM head, fused into one launch.

    logits  [A*B, ld] agent rows (row a*B + b = agent a, beam b);
    targets [B, K] int32 candidate tokens per beam (ids outside [0, vocab) = padding);
    rewards [A, B] float32 cumulative per-agent rewards of the beams.
    Returns (U [A, B*K], W [B*K], order [n_order] int32, order_val [n_order]) with
    U = rewards + log p(token), W = welfare over agents, order = stable descending
    (n_order defaults to B*K; 0 skips the sort and returns (U, W, None, None); up to 256
    the launch selects the n_order best without sorting the rest).
    kept_out [A, n_order] float32 (optional) receives U[:, order]: the cumulative rewards
    of the kept beams when the first n_order ranks are kept (B*K <= 1024).

    Restates beam_search.py:495-560 (per-candidate agent log-probs :335-404,
    cumulative rewards :534-536, stable sort by min over agents :558-560).
    """
    L = _lib.load()
    rows, ld, vocab = _logits_args(logits, vocab)
    if targets.dim() != 2 or targets.dtype != torch.int32:
        raise CSError("targets must be [B, K] int32")
    if rewards.dim() != 2 or rewards.dtype != torch.float32:
        raise CSError("rewards must be [A, B] float32")
    targets, rewards = targets.contiguous(), rewards.contiguous()
    A, B = rewards.shape
    K = targets.shape[1]
    if targets.shape[0] != B or rows != A * B:
        raise CSError(f"shape mismatch: logits rows {rows}, rewards {tuple(rewards.shape)}, "
                      f"targets {tuple(targets.shape)}")
    _require_cuda(logits, targets, rewards)
    if isinstance(kind, str):
        kind = WELFARE[kind]
    C = B * K
    n_order = C if n_order is None else int(n_order)
    dev = logits.device
    U = torch.empty((A, C), dtype=torch.float32, device=dev) if out_U is None else out_U
    W = torch.empty(C, dtype=torch.float32, device=dev) if out_W is None else out_W
    if (U.shape != (A, C) or W.shape != (C,) or U.dtype != torch.float32 or
            W.dtype != torch.float32 or not U.is_contiguous() or not W.is_contiguous()):
        raise CSError(f"out_U / out_W must be contiguous float32 [{A}, {C}] / [{C}]")
    order = torch.empty(max(n_order, 0), dtype=torch.int32, device=dev)
    oval = torch.empty(max(n_order, 0), dtype=torch.float32, device=dev)
    nbytes = int(L.cs_beam_step_workspace_size(rows, vocab))
    if workspace is None:
        workspace = _beam_ws.setdefault(dev, Workspace(zeroed=True))
    if not workspace.zeroed:
        raise CSError("beam_step needs a Workspace(zeroed=True) of its own (arrival counters)")
    ws = workspace.get(nbytes, dev)
    if kept_out is not None:
        if (kept_out.dtype != torch.float32 or not kept_out.is_contiguous()
                or tuple(kept_out.shape) != (A, n_order)):
            raise CSError(f"kept_out must be a contiguous float32 [{A}, {n_order}] tensor")
        _require_cuda(kept_out)
    rc = L.cs_beam_step(logits.data_ptr(), _DTYPE[logits.dtype], A, B, vocab, ld,
                        targets.data_ptr(), K, rewards.data_ptr(), float(softcap), int(kind),
                        float(eps), U.data_ptr(), W.data_ptr(), n_order,
                        order.data_ptr() if n_order else None, oval.data_ptr() if n_order else None,
                        kept_out.data_ptr() if kept_out is not None else None,
                        ws.data_ptr() if ws is not None else None,
                        ws.numel() if ws is not None else 0, _stream())
    if rc != 0:
        workspace.reset()
    _lib.check(rc, "cs_beam_step")
    if n_order == 0:
        return U, W, None, None
    return U, W, order, oval


def beam_decode_step(ref_logits: torch.Tensor, logits: torch.Tensor, rewards: torch.Tensor,
                     k: int, kind="min", *, n_order: Optional[int] = None,
                     vocab: Optional[int] = None, softcap: float = 0.0, eps: float = 1e-9,
                     workspace: Optional[Workspace] = None,
                     kept_out: Optional[torch.Tensor] = None,
                     out_U: Optional[torch.Tensor] = None, out_W: Optional[torch.Tensor] = None,
                     out_ids: Optional[torch.Tensor] = None,
                     out_order: Optional[torch.Tensor] = None):
    """Proposer + scoring of one beam decode step in ONE launch (cs_beam_decode_step).

    ref_logits [B, ld_ref] reference-policy rows; logits [A*B, ld] agent rows (row a*B+b);
    rewards [A, B] float32.  Returns (ids [B, k] int32, U [A, B*k], W [B*k], order, order_val)
    — identical to ``ids, _ = vocab_topk(ref_logits, k)`` followed by
    ``beam_step(logits, ids, rewards, ...)``.  Restates beam_search.py:439-560.
    """
    L = _lib.load()
    rows, ld, vocab = _logits_args(logits, vocab)
    B_ref, ld_ref, _ = _logits_args(ref_logits, vocab)
    if rewards.dim() != 2 or rewards.dtype != torch.float32:
        raise CSError("rewards must be [A, B] float32")
    if ref_logits.dtype != logits.dtype:
        raise CSError("ref_logits and logits must share a dtype")
    rewards = rewards.contiguous()
    A, B = rewards.shape
    if B_ref != B or rows != A * B:
        raise CSError(f"shape mismatch: ref rows {B_ref}, agent rows {rows}, rewards {tuple(rewards.shape)}")
    _require_cuda(ref_logits, logits, rewards, out_ids, out_order)
    if isinstance(kind, str):
        kind = WELFARE[kind]
    k = int(k)
    C = B * k
    n_order = C if n_order is None else int(n_order)
    dev = logits.device
    ids = torch.empty((B, k), dtype=torch.int32, device=dev) if out_ids is None else out_ids
    if ids.shape != (B, k) or ids.dtype != torch.int32 or not ids.is_contiguous():
        raise CSError(f"out_ids must be a contiguous int32 [{B}, {k}] tensor")
    U = torch.empty((A, C), dtype=torch.float32, device=dev) if out_U is None else out_U
    W = torch.empty(C, dtype=torch.float32, device=dev) if out_W is None else out_W
    if (U.shape != (A, C) or W.shape != (C,) or U.dtype != torch.float32 or
            W.dtype != torch.float32 or not U.is_contiguous() or not W.is_contiguous()):
        raise CSError(f"out_U / out_W must be contiguous float32 [{A}, {C}] / [{C}]")
    order = (torch.empty(max(n_order, 0), dtype=torch.int32, device=dev) if out_order is None
             else out_order)
    if order.shape != (max(n_order, 0),) or order.dtype != torch.int32 or not order.is_contiguous():
        raise CSError(f"out_order must be a contiguous int32 [{n_order}] tensor")
    oval = torch.empty(max(n_order, 0), dtype=torch.float32, device=dev)
    nbytes = int(L.cs_beam_decode_workspace_size(A, B, vocab, k))
    if workspace is None:
        workspace = _decode_ws.setdefault(dev, Workspace(zeroed=True))
    if not workspace.zeroed:
        raise CSError("beam_decode_step needs a Workspace(zeroed=True) of its own (arrival counters)")
    ws = workspace.get(nbytes, dev)
    if kept_out is not None:
        if (kept_out.dtype != torch.float32 or not kept_out.is_contiguous()
                or tuple(kept_out.shape) != (A, n_order)):
            raise CSError(f"kept_out must be a contiguous float32 [{A}, {n_order}] tensor")
        _require_cuda(kept_out)
    rc = L.cs_beam_decode_step(ref_logits.data_ptr(), ld_ref, logits.data_ptr(), ld,
                               _DTYPE[logits.dtype], A, B, vocab, k, float(softcap),
                               rewards.data_ptr(), int(kind), float(eps), ids.data_ptr(),
                               U.data_ptr(), W.data_ptr(), n_order,
                               order.data_ptr() if n_order else None,
                               oval.data_ptr() if n_order else None,
                               kept_out.data_ptr() if kept_out is not None else None,
                               ws.data_ptr(), ws.numel(), _stream())
    if rc != 0:
        workspace.reset()
    _lib.check(rc, "cs_beam_decode_step")
    if n_order == 0:
        return ids, U, W, None, None
    return ids, U, W, order, oval


def _logits_args(logits: torch.Tensor, vocab: Optional[int]):
    if logits.dim() != 2 or logits.stride(1) != 1:
        raise CSError("logits must be 2-D with unit column stride")
    if logits.dtype not in _DTYPE:
        raise CSError(f"unsupported logits dtype {logits.dtype}")
    rows = logits.shape[0]
    ld = logits.stride(0) if rows > 1 else logits.shape[1]
    vocab = logits.shape[1] if vocab is None else int(vocab)
    if vocab > logits.shape[1]:
        raise CSError("vocab exceeds logits width")
    return rows, ld, vocab


def vocab_topk(logits: torch.Tensor, k: int, *, vocab: Optional[int] = None, softcap: float = 0.0,
               workspace: Optional[Workspace] = None):
    """Top-k token ids (value desc, id asc) of every logits row -> (ids [rows, k] int32,
    values [rows, k] f32).  The deterministic beam-candidate proposer replacing the
    reference's repeated one-token sampling (beam_search.py:199-333)."""
    L = _lib.load()
    rows, ld, vocab = _logits_args(logits, vocab)
    _require_cuda(logits)
    ids = torch.empty((rows, k), dtype=torch.int32, device=logits.device)
    vals = torch.empty((rows, k), dtype=torch.float32, device=logits.device)
    nbytes = int(L.cs_vocab_topk_workspace_size(rows, vocab, k))
    if workspace is None:
        workspace = _default_ws.setdefault(logits.device, Workspace())
    ws = workspace.get(nbytes, logits.device)
    rc = L.cs_vocab_topk(logits.data_ptr(), _DTYPE[logits.dtype], rows, vocab, ld, int(k),
                         float(softcap), ids.data_ptr(), vals.data_ptr(),
                         ws.data_ptr() if ws is not None else None,
                         ws.numel() if ws is not None else 0, _stream())
    _lib.check(rc, "cs_vocab_topk")
    return ids, vals


def vocab_sample(logits: torch.Tensor, seeds: torch.Tensor, *, temperature: float = 1.0,
                 vocab: Optional[int] = None, softcap: float = 0.0,
                 workspace: Optional[Workspace] = None):
    """Seeded Gumbel-max draws: seeds [rows, n_draw] int64 (bit pattern used as uint64) ->
    (ids [rows, n_draw] int32, log-probs [rows, n_draw] f32)."""
    L = _lib.load()
    rows, ld, vocab = _logits_args(logits, vocab)
    seeds = seeds.reshape(rows, -1)
    if seeds.dtype != torch.int64 or not seeds.is_contiguous():
        raise CSError("seeds must be a contiguous int64 tensor [rows, n_draw]")
    _require_cuda(logits, seeds)
    n_draw = seeds.shape[1]
    ids = torch.empty((rows, n_draw), dtype=torch.int32, device=logits.device)
    lp = torch.empty((rows, n_draw), dtype=torch.float32, device=logits.device)
    nbytes = int(L.cs_vocab_sample_workspace_size(rows, vocab, n_draw))
    if workspace is None:
        workspace = _default_ws.setdefault(logits.device, Workspace())
    ws = workspace.get(nbytes, logits.device)
    rc = L.cs_vocab_sample(logits.data_ptr(), _DTYPE[logits.dtype], rows, vocab, ld,
                           float(temperature), float(softcap), seeds.data_ptr(), n_draw,
                           ids.data_ptr(), lp.data_ptr(), ws.data_ptr() if ws is not None else None,
                           ws.numel() if ws is not None else 0, _stream())
    _lib.check(rc, "cs_vocab_sample")
    return ids, lp


class AttnPlan:
    """A cs_prefix_attention work plan on the device (entries, counts) and the split
    partials' workspace it needs; built once per (prefix-length bounds, shape) and reused by
    every launch (and graph replay) of that shape."""

    def __init__(self, entries: Optional[torch.Tensor], n_attn: int, n_merge: int,
                 workspace: Optional[torch.Tensor]) -> None:
        self.entries, self.n_attn, self.n_merge, self.workspace = entries, n_attn, n_merge, workspace


_attn_plans: "collections.OrderedDict" = collections.OrderedDict()
_ATTN_PLAN_CACHE = 64
_plan_sinks = threading.local()


@contextlib.contextmanager
def retain_plans(holder: dict):
    """Every AttnPlan handed out inside the block is also stored in ``holder`` (keyed by
    id).  A captured graph keeps the raw device pointers of its plans' entries and
    workspace; the owner of the graph keeps the plans alive through ``holder`` so that
    an eviction from the LRU cache above cannot free memory a later replay uses."""
    stack = getattr(_plan_sinks, "stack", None)
    if stack is None:
        stack = _plan_sinks.stack = []
    stack.append(holder)
    try:
        yield holder
    finally:
        stack.pop()


def _retain(plan: "AttnPlan") -> "AttnPlan":
    for holder in getattr(_plan_sinks, "stack", ()):
        holder[id(plan)] = plan
    return plan


def attention_plan(prefix_len_host: Sequence[int], group_prefix_host: Optional[Sequence[int]],
                   n_groups: int, n_str: int, T: int, H: int, Hkv: int, D: int, ld_hist: int,
                   device) -> AttnPlan:
    """The work plan of cs_prefix_attention_plan for host bounds of the prefix lengths
    (cached; the device copy is made outside any graph capture)."""
    key = (tuple(int(x) for x in prefix_len_host),
           None if group_prefix_host is None else tuple(int(x) for x in group_prefix_host),
           n_groups, n_str, T, H, Hkv, D, ld_hist, str(device))
    plan = _attn_plans.get(key)
    if plan is not None:
        _attn_plans.move_to_end(key)
        return _retain(plan)
    if torch.cuda.is_current_stream_capturing():
        raise CSError("cs_prefix_attention: the work plan of this shape must be built before "
                      "graph capture (run the step once eagerly)")
    L = _lib.load()
    lens = np.ascontiguousarray(np.asarray(key[0], dtype=np.int32))
    gp = None if key[1] is None else np.ascontiguousarray(np.asarray(key[1], dtype=np.int32))
    n_a, n_m = ctypes.c_int32(0), ctypes.c_int32(0)
    wsb = ctypes.c_size_t(0)
    args = (lens.ctypes.data, lens.size, None if gp is None else gp.ctypes.data, n_groups, n_str,
            T, H, Hkv, D, ld_hist)
    total = int(L.cs_prefix_attention_plan(*args, None, 0, ctypes.byref(n_a), ctypes.byref(n_m),
                                           ctypes.byref(wsb)))
    if total < 0:
        _lib.check(total, "cs_prefix_attention_plan")
    if total == 0:
        plan = AttnPlan(None, 0, 0, None)
    else:
        host = np.zeros((total, 4), dtype=np.int32)
        rc = int(L.cs_prefix_attention_plan(*args, host.ctypes.data, total, ctypes.byref(n_a),
                                            ctypes.byref(n_m), ctypes.byref(wsb)))
        if rc != total:
            _lib.check(rc if rc < 0 else -1, "cs_prefix_attention_plan")
        plan = AttnPlan(torch.from_numpy(host).to(device), n_a.value, n_m.value,
                        torch.empty(max(int(wsb.value), 16), dtype=torch.uint8, device=device))
    _attn_plans[key] = plan
    while len(_attn_plans) > _ATTN_PLAN_CACHE:
        _attn_plans.popitem(last=False)
    return _retain(plan)


def prefix_attention(q: torch.Tensor, k_prefix: torch.Tensor, vt_prefix: torch.Tensor,
                     prefix_off: torch.Tensor, prefix_len: torch.Tensor, max_prefix_len: int,
                     k_hist: torch.Tensor, vt_hist: torch.Tensor, hist_base: torch.Tensor,
                     n_str: int, T: int, *, scale: float, softcap: float = 0.0, window: int = 0,
                     group_prefix: Optional[torch.Tensor] = None,
                     prefix_len_host: Optional[Sequence[int]] = None,
                     group_prefix_host: Optional[Sequence[int]] = None,
                     out: Optional[torch.Tensor] = None, plan: Optional[AttnPlan] = None,
                     hist_rows: Optional[torch.Tensor] = None):
    """Cascade attention of candidate streams over shared per-agent prefix K/V
    (cs_prefix_attention; layouts in include/consensus_scoring.h).  hist_rows [S, ldh] int32:
    the history is row-layout (vt_hist is V [S, Hkv, ldh, D] like k_hist) and slot j of
    stream s lives in row hist_rows[s, j] (cs_prefix_attention_rows: beams without copies).

    q [n_groups*n_str*T, H, D] bf16; k_prefix [Hkv, Lp, D], vt_prefix [Hkv, Lp/32, D, 32]
    (ragged prefixes: prefix p's keys are rows prefix_off[p] ..; V transposed in 32-key
    tiles, see blocked_vt); prefix_off [n_prefix] int64, prefix_len [n_prefix] int32
    (device), max_prefix_len >= every prefix_len (host); k_hist [S, Hkv, ldh, D], vt_hist
    [S, Hkv, ldh/32, D, 32] (S = n_groups*n_str); hist_base [1] int32 (device).
    prefix_len_host (per prefix) / group_prefix_host: host bounds that size the key splits
    of the work plan (default: max_prefix_len everywhere); ``plan`` overrides them.
    Returns out [n_tok, H, D] bf16.  Replaces the per-call prompt re-encoding of
    src/utils.py:249-259."""
    L = _lib.load()
    if q.dim() != 3 or q.dtype != torch.bfloat16 or not q.is_contiguous():
        raise CSError("q must be a contiguous [n_tok, H, D] bfloat16 tensor")
    n_tok, H, D = q.shape
    Hkv, Lp, Dk = k_prefix.shape
    S, Hkv2, ldh, Dh = k_hist.shape
    if Dk != D or Dh != D or Hkv2 != Hkv:
        raise CSError("head layout mismatch between q, k_prefix and k_hist")
    if hist_rows is not None:
        # the buffers may hold more rows than query streams (a token tree's earlier levels)
        if tuple(vt_hist.shape) != (S, Hkv, ldh, D):
            raise CSError("row-layout history: V [R, Hkv, ldh, D] like K expected")
        if hist_rows.dtype != torch.int32 or hist_rows.dim() != 2 or hist_rows.shape[1] != ldh or \
                hist_rows.shape[0] > S or not hist_rows.is_contiguous():
            raise CSError("hist_rows must be a contiguous int32 [S, ldh] tensor (S <= buffer rows)")
        if _DEBUG_TABLES and hist_rows.numel() and not torch.cuda.is_current_stream_capturing():
            if int(hist_rows.min()) < 0 or int(hist_rows.max()) >= S:
                raise CSError("hist_rows names a row outside the K / V buffer")
        S = hist_rows.shape[0]
    if tuple(vt_prefix.shape) != (Hkv, Lp // 32, D, 32) or \
            (hist_rows is None and tuple(vt_hist.shape) != (S, Hkv, ldh // 32, D, 32)):
        raise CSError("vt_prefix [Hkv, Lp/32, D, 32] / vt_hist [S, Hkv, ldh/32, D, 32] "
                      "(V^T in 32-key tiles) expected")
    for t in (k_prefix, vt_prefix, k_hist, vt_hist):
        if t.dtype != torch.bfloat16 or not t.is_contiguous():
            raise CSError("K/V buffers must be contiguous bfloat16")
    if n_str <= 0 or T <= 0 or S % n_str != 0 or n_tok != S * T:
        raise CSError(f"n_tok {n_tok} != streams {S} x T {T} (n_str {n_str})")
    n_groups = S // n_str
    n_prefix = prefix_len.numel()
    if group_prefix is None and n_groups != n_prefix:
        raise CSError("n_groups must equal n_prefix without group_prefix")
    if group_prefix is not None and (group_prefix.dtype != torch.int32 or group_prefix.numel() != n_groups):
        raise CSError("group_prefix must be int32 [n_groups]")
    if prefix_len.dtype != torch.int32 or prefix_off.dtype != torch.int64 or \
            prefix_off.numel() != n_prefix:
        raise CSError("prefix_len must be int32 [n_prefix] and prefix_off int64 [n_prefix]")
    if hist_base.dtype != torch.int32 or hist_base.numel() != 1:
        raise CSError("hist_base must be a one-element int32 device tensor")
    _require_cuda(q, k_prefix, vt_prefix, prefix_off, prefix_len, k_hist, vt_hist, hist_base,
                  group_prefix, out, hist_rows)
    if out is None:
        out = torch.empty_like(q)
    mpl = int(max_prefix_len)
    if plan is None:
        if prefix_len_host is None or (group_prefix is not None and group_prefix_host is None):
            # no host lengths: every group bounded by max_prefix_len
            lens_h, gp_h = [mpl], [0] * n_groups
        else:
            lens_h = [min(int(x), mpl) for x in prefix_len_host]
            gp_h = None if group_prefix is None else list(group_prefix_host)
            if len(lens_h) != n_prefix or (gp_h is not None and len(gp_h) != n_groups):
                raise CSError("prefix_len_host / group_prefix_host sizes do not match")
        plan = attention_plan(lens_h, gp_h, n_groups, n_str, T, H, Hkv, D, ldh, q.device)
    else:
        _retain(plan)
    ws = plan.workspace
    gp = group_prefix.data_ptr() if group_prefix is not None else None
    pe = plan.entries.data_ptr() if plan.entries is not None else None
    wsp, wsn = (ws.data_ptr(), ws.numel()) if ws is not None else (None, 0)
    if hist_rows is not None:
        rc = L.cs_prefix_attention_rows(q.data_ptr(), k_prefix.data_ptr(), vt_prefix.data_ptr(), Lp,
                                        prefix_off.data_ptr(), prefix_len.data_ptr(), mpl, gp,
                                        n_groups, k_hist.data_ptr(), vt_hist.data_ptr(),
                                        hist_rows.data_ptr(), ldh, hist_base.data_ptr(), n_str, T,
                                        H, Hkv, D, float(scale), float(softcap), int(window), pe,
                                        plan.n_attn, plan.n_merge, out.data_ptr(), wsp, wsn,
                                        _stream())
        _lib.check(rc, "cs_prefix_attention_rows")
        return out
    rc = L.cs_prefix_attention(q.data_ptr(), k_prefix.data_ptr(), vt_prefix.data_ptr(), Lp,
                               prefix_off.data_ptr(), prefix_len.data_ptr(), mpl, gp,
                               n_groups, k_hist.data_ptr(), vt_hist.data_ptr(), ldh,
                               hist_base.data_ptr(), n_str, T, H, Hkv, D, float(scale),
                               float(softcap), int(window), pe, plan.n_attn, plan.n_merge,
                               out.data_ptr(), wsp, wsn, _stream())
    _lib.check(rc, "cs_prefix_attention")
    return out


def rope_place(qkv: "torch.Tensor | SplitPartials", inv_freq: torch.Tensor, prefix_len: torch.Tensor,
               hist_base: torch.Tensor, n_str: int, T: int, H: int, Hkv: int, D: int,
               q_out: torch.Tensor, k_hist: torch.Tensor, vt_hist: torch.Tensor, *,
               group_prefix: Optional[torch.Tensor] = None, v_rows: bool = False) -> torch.Tensor:
    """RoPE of the fused projection + placement of q / the new K, V (cs_rope_place).  qkv
    may be a K-split GEMM's unfolded SplitPartials (T < 32): folded inside the launch
    (cs_rope_place_splitk), bitwise the folded projection.  v_rows: vt_hist is a row-layout
    V [S, Hkv, ldh, D] (cs_rope_place_rows, the cs_prefix_attention_rows history)."""
    L = _lib.load()
    vshape = (lambda S, ldh: (S, Hkv, ldh, D)) if v_rows else (lambda S, ldh: (S, Hkv, ldh // 32, D, 32))
    sfx = "_rows" if v_rows else ""
    if isinstance(qkv, SplitPartials):
        part = qkv.part
        S, Hkv2, ldh, Dk = k_hist.shape
        n_tok = part.shape[1]
        if (part.dim() != 3 or part.dtype != torch.float32 or not part.is_contiguous()
                or part.shape[2] != (H + 2 * Hkv) * D):
            raise CSError("qkv partials must be contiguous float32 [splits, n_tok, (H + 2 Hkv) D]")
        if Hkv2 != Hkv or Dk != D or tuple(vt_hist.shape) != vshape(S, ldh):
            raise CSError("k_hist [S, Hkv, ldh, D] / vt_hist [S, Hkv, ldh/32, D, 32] layout mismatch")
        if n_tok != S * T or S % n_str != 0:
            raise CSError("qkv rows must be streams x T")
        if tuple(q_out.shape) != (n_tok, H, D) or q_out.dtype != torch.bfloat16 or not q_out.is_contiguous():
            raise CSError("q_out must be a contiguous [n_tok, H, D] bfloat16 tensor")
        _require_cuda(part, inv_freq, prefix_len, hist_base, q_out, k_hist, vt_hist, group_prefix)
        rc = getattr(L, "cs_rope_place_splitk" + sfx)(part.data_ptr(), part.shape[0], inv_freq.data_ptr(),
                                    prefix_len.data_ptr(),
                                    group_prefix.data_ptr() if group_prefix is not None else None,
                                    S // n_str, hist_base.data_ptr(), n_str, T, H, Hkv, D,
                                    q_out.data_ptr(), k_hist.data_ptr(), vt_hist.data_ptr(), ldh,
                                    _stream())
        _lib.check(rc, "cs_rope_place_splitk" + sfx)
        return q_out
    if qkv.dim() != 2 or qkv.dtype != torch.bfloat16 or qkv.stride(1) != 1:
        raise CSError("qkv must be a 2-D bfloat16 tensor with unit column stride")
    n_tok = qkv.shape[0]
    S, Hkv2, ldh, Dk = k_hist.shape
    if Hkv2 != Hkv or Dk != D or tuple(vt_hist.shape) != vshape(S, ldh):
        raise CSError("k_hist [S, Hkv, ldh, D] / vt_hist [S, Hkv, ldh/32, D, 32] layout mismatch")
    if n_tok != S * T or S % n_str != 0:
        raise CSError("qkv rows must be streams x T")
    if tuple(q_out.shape) != (n_tok, H, D) or q_out.dtype != torch.bfloat16 or not q_out.is_contiguous():
        raise CSError("q_out must be a contiguous [n_tok, H, D] bfloat16 tensor")
    if inv_freq.dtype != torch.float32 or inv_freq.numel() != D // 2:
        raise CSError("inv_freq must be float32 [D/2]")
    _require_cuda(qkv, inv_freq, prefix_len, hist_base, q_out, k_hist, vt_hist, group_prefix)
    ld = qkv.stride(0) if n_tok > 1 else qkv.shape[1]
    rc = getattr(L, "cs_rope_place" + sfx)(qkv.data_ptr(), ld, inv_freq.data_ptr(), prefix_len.data_ptr(),
                         group_prefix.data_ptr() if group_prefix is not None else None,
                         S // n_str, hist_base.data_ptr(), n_str, T, H, Hkv, D, q_out.data_ptr(),
                         k_hist.data_ptr(), vt_hist.data_ptr(), ldh, _stream())
    _lib.check(rc, "cs_rope_place" + sfx)
    return q_out


def _rows2d(t: torch.Tensor, name: str):
    if t.dim() != 2 or t.dtype != torch.bfloat16 or t.stride(1) != 1:
        raise CSError(f"{name} must be a 2-D bfloat16 tensor with unit column stride")
    return t.stride(0) if t.shape[0] > 1 else t.shape[1]


class SplitPartials(NamedTuple):
    """A K-split GEMM's unfolded fp32 partials [splits, M, N] (cs_gemm_bf16 with y = NULL),
    folded by the add_rms_norm that consumes them (cs_add_rms_norm_splitk)."""
    part: torch.Tensor


def add_rms_norm(a: torch.Tensor, weight: torch.Tensor, eps: float, *,
                 b: "Optional[torch.Tensor | SplitPartials]" = None,
                 b_weight: Optional[torch.Tensor] = None, plus_one: bool = False,
                 s_out: Optional[torch.Tensor] = None,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = RMSNorm(a + b) (cs_add_rms_norm); the bf16 sum a + b is also written to s_out.
    a, b, s_out, out [rows, d] bf16; weight [d] bf16 (Gemma-2: plus_one, 1 + weight).
    b_weight: b is RMS-normalised first with that weight (Gemma-2's post norms), bitwise as
    add_rms_norm(b, b_weight) followed by this call.  b may be a SplitPartials (linear(...,
    fold=False)): folded inside this launch, bitwise as the GEMM's own fold then this call."""
    L = _lib.load()
    lda = _rows2d(a, "a")
    rows, d = a.shape
    if isinstance(b, SplitPartials):
        return _add_rms_norm_splitk(L, a, lda, weight, eps, b.part, b_weight, plus_one, s_out, out)
    ldb = _rows2d(b, "b") if b is not None else 0
    lds = _rows2d(s_out, "s_out") if s_out is not None else 0
    if (b is not None and b.shape != a.shape) or (s_out is not None and s_out.shape != a.shape):
        raise CSError("a, b and s_out must share one shape")
    if weight.dtype != torch.bfloat16 or weight.numel() != d or not weight.is_contiguous():
        raise CSError("weight must be a contiguous bfloat16 [d] tensor")
    if b_weight is not None and (b is None or b_weight.dtype != torch.bfloat16 or
                                 b_weight.numel() != d or not b_weight.is_contiguous()):
        raise CSError("b_weight must be a contiguous bfloat16 [d] tensor and needs b")
    if out is None:
        out = torch.empty_like(a, memory_format=torch.contiguous_format)
    ldy = _rows2d(out, "out")
    _require_cuda(a, b, s_out, weight, out)
    rc = L.cs_add_rms_norm(a.data_ptr(), lda, b.data_ptr() if b is not None else None, ldb,
                           b_weight.data_ptr() if b_weight is not None else None,
                           s_out.data_ptr() if s_out is not None else None, lds, weight.data_ptr(),
                           rows, d, float(eps), int(bool(plus_one)), out.data_ptr(), ldy, _stream())
    _lib.check(rc, "cs_add_rms_norm")
    return out


def _add_rms_norm_splitk(L, a, lda, weight, eps, part, b_weight, plus_one, s_out, out):
    rows, d = a.shape
    if part.dim() != 3 or part.dtype != torch.float32 or not part.is_contiguous() or \
            tuple(part.shape[1:]) != (rows, d):
        raise CSError("split partials must be a contiguous float32 [splits, rows, d] tensor")
    lds = _rows2d(s_out, "s_out") if s_out is not None else 0
    if s_out is not None and s_out.shape != a.shape:
        raise CSError("a and s_out must share one shape")
    if weight.dtype != torch.bfloat16 or weight.numel() != d or not weight.is_contiguous():
        raise CSError("weight must be a contiguous bfloat16 [d] tensor")
    if b_weight is not None and (b_weight.dtype != torch.bfloat16 or b_weight.numel() != d or
                                 not b_weight.is_contiguous()):
        raise CSError("b_weight must be a contiguous bfloat16 [d] tensor")
    if out is None:
        out = torch.empty_like(a, memory_format=torch.contiguous_format)
    ldy = _rows2d(out, "out")
    _require_cuda(a, part, s_out, weight, out)
    rc = L.cs_add_rms_norm_splitk(a.data_ptr(), lda, part.data_ptr(), int(part.shape[0]),
                                  b_weight.data_ptr() if b_weight is not None else None,
                                  s_out.data_ptr() if s_out is not None else None, lds,
                                  weight.data_ptr(), rows, d, float(eps), int(bool(plus_one)),
                                  out.data_ptr(), ldy, _stream())
    _lib.check(rc, "cs_add_rms_norm_splitk")
    return out


def gated_act(gate: torch.Tensor, up: torch.Tensor, act: str = "silu",
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(gate) * up (cs_gated_act): SiLU (Llama-3) or tanh-GeLU (Gemma-2); [rows, F] bf16."""
    L = _lib.load()
    ldg = _rows2d(gate, "gate")
    ldu = _rows2d(up, "up")
    if gate.shape != up.shape:
        raise CSError("gate and up must share one shape")
    rows, F = gate.shape
    if out is None:
        out = torch.empty(rows, F, dtype=torch.bfloat16, device=gate.device)
    ldo = _rows2d(out, "out")
    _require_cuda(gate, up, out)
    rc = L.cs_gated_act(gate.data_ptr(), ldg, up.data_ptr(), ldu, rows, F,
                        {"silu": 0, "gelu_tanh": 1}[act], out.data_ptr(), ldo, _stream())
    _lib.check(rc, "cs_gated_act")
    return out


GEMM_DISPATCH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned",
                             "gemm_dispatch_mi355x.json")
_gemm_table: Optional[dict] = None


def gemm_choice(M: int, N: int, K: int, gated: bool = False,
                packed: bool = False) -> Optional[dict]:
    """The cs_gemm_bf16 tile variant and K split measured faster than hipBLASLt for this
    exact shape on MI355X (tools/tune_gemm_dispatch.py -> tuned/gemm_dispatch_mi355x.json,
    read only), or None: the shape stays on hipBLASLt.  packed: the caller holds the weight's
    cs_gemm_pack'ed copy, so the packed form's entry counts too ({"packed": True, ...} when it
    is the fastest).  CS_GEMM_DISPATCH=0 turns the table off, CS_GEMM_DISPATCH=<file> reads
    another one."""
    global _gemm_table
    if _gemm_table is None:
        env = os.environ.get("CS_GEMM_DISPATCH", "")
        path = GEMM_DISPATCH if env in ("", "1") else env
        table = {}
        if env != "0" and os.path.exists(path):
            with open(path) as f:
                table = json.load(f).get("table", {})
        _gemm_table = table
    e = _gemm_table.get(f"{M},{N},{K},{int(bool(gated))}")
    if e is None:
        return None
    if packed and "packed" in e:
        return {"variant": int(e["packed"]["variant"]), "splits": int(e["packed"]["splits"]),
                "packed": True}
    if "variant" in e:
        return {"variant": int(e["variant"]), "splits": int(e["splits"]), "packed": False}
    return None


def gemm_pack_gain(N: int, K: int, gated: bool = False) -> float:
    """The largest time (µs) the packed form saves on an [N, K] weight at any row count the
    dispatch table measured (against the faster of hipBLASLt and the unpacked cs_gemm_bf16);
    0 when no row count runs it packed.  A model keeps cs_gemm_pack'ed copies of the weights
    with a gain, the most per byte first."""
    gemm_choice(1, N, K, gated)                 # loads the table
    if hasattr(_gemm_table, "packs"):           # a computed table (tests)
        return 1.0 if _gemm_table.packs(N, K, gated) else 0.0
    tail = f",{N},{K},{int(bool(gated))}"
    gain = 0.0
    for k, v in _gemm_table.items():
        if k.endswith(tail) and "packed" in v:
            ref = min(float(v.get("us", float("inf"))), float(v.get("torch_us", float("inf"))))
            gain = max(gain, ref - float(v["packed"]["us"]) if ref < float("inf") else 1.0)
    return gain


def gemm_packs(N: int, K: int, gated: bool = False) -> bool:
    """Whether the dispatch table runs an [N, K] weight packed at some row count."""
    return gemm_pack_gain(N, K, gated) > 0.0


def linear(x: torch.Tensor, w: torch.Tensor, *, gated: bool = False, act: str = "silu",
           out: Optional[torch.Tensor] = None, fold: bool = True,
           packed: Optional["PackedWeight"] = None):
    """y = x @ w.T (gated: act(gate) * up of the fused gate|up weight) on whichever GEMM the
    dispatch table measured faster for this shape: cs_gemm_bf16 (on the packed copy
    ``packed`` of w when given and fastest) or hipBLASLt (+ cs_gated_act).
    fold=False: a K-split cs_gemm_bf16 returns its unfolded SplitPartials (for an
    add_rms_norm to fold); every other path returns the bf16 tensor as usual."""
    if x.is_cuda and x.dim() == 2:
        ch = gemm_choice(x.shape[0], w.shape[0], w.shape[1], gated, packed=packed is not None)
        if ch is not None and ch["packed"] and gemm_ok(x, w, gated):
            if not fold and not gated and out is None and ch["splits"] > 1:
                return gemm_packed_partials(x, packed, splits=ch["splits"], variant=ch["variant"])
            return gemm_packed(x, packed, gated=gated, act=act, splits=ch["splits"],
                               variant=ch["variant"], out=out)
        if ch is not None and gemm_ok(x, w, gated):
            if not fold and not gated and out is None and int(ch["splits"]) > 1:
                return gemm_partials(x, w, splits=int(ch["splits"]), variant=int(ch["variant"]))
            return gemm(x, w, gated=gated, act=act, splits=int(ch["splits"]),
                        variant=int(ch["variant"]), out=out)
    if gated:          # the plain GEMM (on whichever form is faster) + cs_gated_act
        F = w.shape[0] // 2
        y = linear(x, w, packed=packed)
        return gated_act(y[:, :F], y[:, F:], act, out=out)
    if out is not None:
        return torch.matmul(x, w.t(), out=out)
    return x @ w.t()


def linear_into_residual(x: torch.Tensor, w: torch.Tensor, h: torch.Tensor, *,
                         packed: Optional["PackedWeight"] = None) -> bool:
    """h += x @ w.T in the GEMM's own epilogue (hipBLASLt, beta = 1: the product is added in
    fp32 and rounded once) when the dispatch table leaves this shape on hipBLASLt; returns
    False (nothing done) otherwise, and the caller takes ``linear`` + the residual add.
    For the many-row scoring forward: the residual add's launch then only normalises (one
    read and one write of the rows instead of two and two)."""
    if not (x.is_cuda and x.dim() == 2 and h.dim() == 2 and h.is_contiguous() and
            h.dtype == x.dtype == w.dtype == torch.bfloat16 and h.shape == (x.shape[0], w.shape[0])):
        return False
    if gemm_choice(x.shape[0], w.shape[0], w.shape[1], False, packed=packed is not None) is not None:
        return False
    h.addmm_(x, w.t())
    return True


def gemm_ok(x: torch.Tensor, w: torch.Tensor, gated: bool = False) -> bool:
    """Whether cs_gemm_bf16 takes y = x @ w.T: bf16 2-D operands with unit column stride,
    N a multiple of 128, K of 64, 16-byte aligned rows."""
    if x.dim() != 2 or w.dim() != 2 or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    N, K = w.shape
    if x.shape[1] != K or N % 128 or K % 64 or x.stride(1) != 1 or w.stride(1) != 1:
        return False
    if (x.stride(0) % 8 and x.shape[0] > 1) or w.stride(0) % 8:
        return False
    return x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0


def gemm(x: torch.Tensor, w: torch.Tensor, *, gated: bool = False, act: str = "silu",
         splits: int = 0, variant: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ w.T (cs_gemm_bf16): x [M, K], w [N, K] bf16, y [M, N] bf16, fp32 accumulation.
    gated: w is the fused gate|up weight [2F, K] and y [M, F] = act(gate) * up (the rounding
    of cs_gated_act).  splits: K split (0 = the library's choice); the fp32 partials are a
    per-call tensor (inside a capture it belongs to the graph's pool)."""
    L = _lib.load()
    if not gemm_ok(x, w, gated):
        raise CSError("cs_gemm_bf16 needs bf16 x [M, K], w [N, K] with N % 128 == 0, K % 64 == 0")
    M, K = x.shape
    N = w.shape[0]
    n_out = N // 2 if gated else N
    if out is None:
        out = torch.empty(M, n_out, dtype=torch.bfloat16, device=x.device)
    if out.shape != (M, n_out) or out.dtype != torch.bfloat16 or out.stride(1) != 1:
        raise CSError("out must be a bf16 [M, N] tensor with unit column stride")
    _require_cuda(x, w, out)
    if gated:
        splits = 1
    elif splits <= 0:
        splits = int(L.cs_gemm_splits(M, N, K, 0, variant))
    part = (torch.empty(splits * M * N, dtype=torch.float32, device=x.device)
            if splits > 1 else None)
    ldx = x.stride(0) if M > 1 else K
    ldy = out.stride(0) if M > 1 else n_out
    if splits > 1 and (ldy % 8 or out.data_ptr() % 16):
        # the split-K fold stores 16-byte vectors: fold into an aligned tensor, then copy
        tmp = gemm(x, w, splits=splits, variant=variant)
        out.copy_(tmp)
        return out
    rc = L.cs_gemm_bf16(x.data_ptr(), ldx, w.data_ptr(), w.stride(0), out.data_ptr(), ldy, M, N,
                        K, splits, int(bool(gated)), {"silu": 0, "gelu_tanh": 1}[act], variant,
                        part.data_ptr() if part is not None else None, _stream())
    _lib.check(rc, "cs_gemm_bf16")
    return out


class PackedWeight:
    """A [N, K] bf16 weight in cs_gemm_pack's fragment-major layout: each 16-row tile's
    64-deep K step is 2 KB of lane-ordered MFMA fragments, so cs_gemm_bf16_packed reads its
    weight stream in contiguous 1 KB pieces.  ``data`` is the packed [N * K] tensor."""

    def __init__(self, data: torch.Tensor, N: int, K: int):
        self.data, self.N, self.K = data, int(N), int(K)

    @property
    def shape(self):
        return (self.N, self.K)


def gemm_pack(w: torch.Tensor) -> PackedWeight:
    """The packed copy of w [N, K] (cs_gemm_pack; N % 16 == 0, K % 64 == 0)."""
    L = _lib.load()
    if w.dim() != 2 or w.dtype != torch.bfloat16 or w.stride(1) != 1:
        raise CSError("gemm_pack needs a bf16 [N, K] tensor with unit column stride")
    N, K = w.shape
    _require_cuda(w)
    out = torch.empty(N * K, dtype=torch.bfloat16, device=w.device)
    rc = L.cs_gemm_pack(w.data_ptr(), w.stride(0), N, K, out.data_ptr(), _stream())
    _lib.check(rc, "cs_gemm_pack")
    return PackedWeight(out, N, K)


def gemm_packed(x: torch.Tensor, pw: PackedWeight, *, gated: bool = False, act: str = "silu",
                splits: int = 0, variant: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ops.gemm on a packed weight (cs_gemm_bf16_packed, variants 0 / 2 / 3 / 4): bitwise the
    unpacked result."""
    L = _lib.load()
    M, K = x.shape
    N = pw.N
    if x.dtype != torch.bfloat16 or x.stride(1) != 1 or K != pw.K:
        raise CSError("gemm_packed needs bf16 x [M, K] matching the packed weight")
    n_out = N // 2 if gated else N
    if out is None:
        out = torch.empty(M, n_out, dtype=torch.bfloat16, device=x.device)
    if out.shape != (M, n_out) or out.dtype != torch.bfloat16 or out.stride(1) != 1:
        raise CSError("out must be a bf16 [M, N] tensor with unit column stride")
    _require_cuda(x, pw.data, out)
    if gated:
        splits = 1
    elif splits <= 0:
        splits = int(L.cs_gemm_splits(M, N, K, 0, variant))
    ldx = x.stride(0) if M > 1 else K
    ldy = out.stride(0) if M > 1 else n_out
    if splits > 1 and (ldy % 8 or out.data_ptr() % 16):
        out.copy_(gemm_packed(x, pw, splits=splits, variant=variant))
        return out
    part = (torch.empty(splits * M * N, dtype=torch.float32, device=x.device)
            if splits > 1 else None)
    rc = L.cs_gemm_bf16_packed(x.data_ptr(), ldx, pw.data.data_ptr(), out.data_ptr(), ldy, M, N,
                               K, splits, int(bool(gated)), {"silu": 0, "gelu_tanh": 1}[act],
                               variant, part.data_ptr() if part is not None else None, _stream())
    _lib.check(rc, "cs_gemm_bf16_packed")
    return out


def gemm_packed_partials(x: torch.Tensor, pw: PackedWeight, *, splits: int,
                         variant: int = 0) -> SplitPartials:
    """gemm_partials on a packed weight (cs_gemm_bf16_packed with y = NULL)."""
    L = _lib.load()
    M, K = x.shape
    N = pw.N
    if x.dtype != torch.bfloat16 or x.stride(1) != 1 or K != pw.K or splits < 2:
        raise CSError("gemm_packed_partials needs bf16 x [M, K] matching the weight, splits >= 2")
    _require_cuda(x, pw.data)
    part = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
    ldx = x.stride(0) if M > 1 else K
    rc = L.cs_gemm_bf16_packed(x.data_ptr(), ldx, pw.data.data_ptr(), None, 0, M, N, K, splits, 0,
                               0, variant, part.data_ptr(), _stream())
    _lib.check(rc, "cs_gemm_bf16_packed")
    return SplitPartials(part)


def gemm_partials(x: torch.Tensor, w: torch.Tensor, *, splits: int, variant: int = 0) -> SplitPartials:
    """The fp32 partials [splits, M, N] of cs_gemm_bf16 with a K split, unfolded (y = NULL)."""
    L = _lib.load()
    if not gemm_ok(x, w) or splits < 2:
        raise CSError("gemm_partials needs cs_gemm_bf16 operands and splits >= 2")
    M, K = x.shape
    N = w.shape[0]
    _require_cuda(x, w)
    part = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
    ldx = x.stride(0) if M > 1 else K
    rc = L.cs_gemm_bf16(x.data_ptr(), ldx, w.data_ptr(), w.stride(0), None, 0, M, N, K, splits, 0,
                        0, variant, part.data_ptr(), _stream())
    _lib.check(rc, "cs_gemm_bf16")
    return SplitPartials(part)


def hist_rows_update(src_rows: torch.Tensor, dst_rows: torch.Tensor, parent: torch.Tensor,
                     hist_base: torch.Tensor, *, n_rows: int, row_base: int = 0) -> None:
    """dst_rows[s, j] = src_rows[parent[s], j] for j < hist_base, else row_base + s
    (cs_hist_rows_update): a row-layout history's beam / tree step, no K / V moved.
    src_rows [S_src, ldh], dst_rows [S, ldh], parent [S] indexes src_rows; n_rows = the
    K / V buffer's row count (row_base + S beyond it is rejected).  With CS_DEBUG_TABLES=1
    the parents and the source table's entries are checked on the host as well."""
    L_ = _lib.load()
    if src_rows.dtype != torch.int32 or dst_rows.dtype != torch.int32 or \
            src_rows.dim() != 2 or dst_rows.dim() != 2 or src_rows.shape[1] != dst_rows.shape[1] or \
            not src_rows.is_contiguous() or not dst_rows.is_contiguous():
        raise CSError("slot tables must be contiguous int32 [S, ldh] tensors of one ldh")
    S, ldh = dst_rows.shape
    if parent.dtype != torch.int64 or parent.numel() != S or hist_base.dtype != torch.int32:
        raise CSError("parent must be int64 [S], hist_base int32 [1]")
    _require_cuda(src_rows, dst_rows, parent, hist_base)
    if _DEBUG_TABLES and S and not torch.cuda.is_current_stream_capturing():
        if int(parent.min()) < 0 or int(parent.max()) >= src_rows.shape[0]:
            raise CSError("hist_rows_update: a parent does not index the source table")
        if int(src_rows.min()) < 0 or int(src_rows.max()) >= int(n_rows):
            raise CSError("hist_rows_update: the source table names a row past n_rows")
    rc = L_.cs_hist_rows_update(src_rows.data_ptr(), dst_rows.data_ptr(), parent.data_ptr(),
                                hist_base.data_ptr(), S, ldh, int(row_base), int(n_rows),
                                _stream())
    _lib.check(rc, "cs_hist_rows_update")


def blocked_vt(v: torch.Tensor) -> torch.Tensor:
    """V rows [..., keys, D] (keys a multiple of 32) -> the kernels' V^T in 32-key tiles
    [..., keys/32, D, 32] (contiguous)."""
    *lead, n, D = v.shape
    return v.reshape(*lead, n // 32, 32, D).transpose(-1, -2).contiguous()


def rows_from_blocked(vt: torch.Tensor) -> torch.Tensor:
    """Inverse of blocked_vt: [..., nb, D, 32] -> [..., nb * 32, D]."""
    *lead, nb, D, w = vt.shape
    return vt.transpose(-1, -2).reshape(*lead, nb * w, D)
