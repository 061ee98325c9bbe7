"""Batched agent x candidate scoring engine.

The reference issues one remote call per (agent, candidate) and re-encodes the
whole ~150-800-token prompt every time (src/methods/beam_search.py:495-538,
best_of_n.py:266-321, finite_lookahead.py:464-524).  Here:

  1. ``prefill``: every agent's prompt prefix (system + template + the statement so
     far) is encoded ONCE per decode call -> per-layer K/V [A, Hkv, P, D] plus the
     hidden state at its last position.
  2. ``score``: all (agent, candidate) continuations of a step run as one batch of
     streams that attend to their agent's prefix K/V; the LM head produces one
     logits row per scored token; ``cs_logsoftmax_gather`` turns the rows into token
     log-probs and ``cs_segment_reduce`` folds them per (agent, candidate).
  3. ``BeamState``: beam search keeps per-(prefix, beam) generated K/V and advances
     every stream by one position per step (one logits row per (agent, beam),
     gathered at the K candidate tokens of that beam).

Everything after the LM head runs in the HIP kernels (ops.*).
"""
from __future__ import annotations

import os
import threading
import weakref
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from . import ops
from .model import Model


@dataclass
class PrefixCache:
    kv: list                    # per layer (k, v): [n_prefix, Hkv, Pmax, D]
    lengths: torch.Tensor       # [n_prefix] int64
    last_hidden: torch.Tensor   # [n_prefix, d] final-norm hidden at position length-1
    pos: torch.Tensor           # [n_prefix, Pmax] key positions
    valid: torch.Tensor         # [n_prefix, Pmax] bool
    hidden: torch.Tensor        # [n_prefix, Pmax, d] final-norm hidden of every position
    ids: torch.Tensor           # [n_prefix, Pmax] prefix token ids (right-padded)


def _pad(seqs: Sequence[Sequence[int]], device, fill: int = 0):
    n = len(seqs)
    T = max((len(s) for s in seqs), default=0)
    out = torch.full((n, max(T, 1)), fill, dtype=torch.long)
    lens = torch.zeros(n, dtype=torch.long)
    for i, s in enumerate(seqs):
        if len(s):
            out[i, :len(s)] = torch.as_tensor(list(s), dtype=torch.long)
        lens[i] = len(s)
    return out.to(device, non_blocking=True), lens.to(device, non_blocking=True)


def _uniform_groups(owner: Sequence[int]):
    """(prefix index of each group, streams per group) when ``owner`` is contiguous runs of
    equal length (agent-major agent x candidate batches), else None."""
    R = len(owner)
    if R == 0:
        return None
    n = 1
    while n < R and owner[n] == owner[0]:
        n += 1
    if R % n:
        return None
    groups = [int(owner[i]) for i in range(0, R, n)]
    for gi, g in enumerate(groups):
        base = gi * n
        if any(owner[base + j] != g for j in range(n)):
            return None
    return groups, n


def _id_matrix(rows) -> np.ndarray:
    """Token ids of stored rows as one [n, width] array, right-padded with -1 (never a
    token id, so it ends every common run)."""
    m = np.full((len(rows), max(r.shape[0] for r in rows)), -1, dtype=np.int64)
    for i, r in enumerate(rows):
        m[i, :r.shape[0]] = r
    return m


def _best_lcp(r: np.ndarray, smat: np.ndarray):
    """(first stored row with the longest common token prefix with r, that length): one
    vectorised compare against every stored row."""
    n = min(r.shape[0], smat.shape[1])
    if n == 0:
        return 0, 0
    mism = smat[:, :n] != r[None, :n]
    lcp = np.where(mism.any(axis=1), mism.argmax(axis=1), n)
    j = int(lcp.argmax())
    return j, int(lcp[j])


class ScoringEngine:
    """Owns a model on one device and scores continuations under many prefixes.

    Prefix reuse: the reference re-encodes every prompt from scratch on every call
    (src/utils.py:249-259).  Consecutive calls of one method mostly share their prompts'
    leading tokens (MCTS: every simulation's 2A scoring prompts and the reference
    prompt differ from the previous call's only in the statement's last tokens;
    finite lookahead: one step's agent prompts extend the previous step's), so
    ``prefill`` keeps its last ``reuse_caches`` results and runs only each new prefix's
    tokens past its longest common token prefix with a stored row through the model
    (K/V of a causal prefix depend on that prefix alone).  ``reuse_caches = 0`` (or env
    CS_PREFIX_REUSE=0) prefills every prompt in full."""

    def __init__(self, model: Model, max_rows_per_chunk: int = 32768,
                 max_streams_per_chunk: int = 1024, reuse_caches: Optional[int] = None,
                 reuse_min_tokens: int = 16, reuse_max_tokens: int = 1 << 18,
                 reuse_max_bytes: int = 8 << 30,
                 fused_scoring: bool = True, fused_max_rows: int = 1 << 17):
        self.model = model
        # bf16 models score agent x candidate batches on the stream kernels
        # (_score_fused); fused_max_rows bounds a chunk's logits block (2^17 rows of the
        # 128,256 Llama-3 vocab = 34 GB of bf16 logits, an eighth of the HBM)
        self.fused_scoring = bool(fused_scoring)
        self.fused_max_rows = int(fused_max_rows)
        self.device = model.device
        self.softcap = model.cfg.final_softcap
        self.max_rows = max_rows_per_chunk
        self.max_streams = max_streams_per_chunk
        self.ws = ops.Workspace()
        self.beam_ws = ops.Workspace(zeroed=True)   # cs_beam_step (arrival counters)
        if reuse_caches is None:
            reuse_caches = 0 if os.environ.get("CS_PREFIX_REUSE", "1") == "0" else 4
        self.reuse_caches = int(reuse_caches)
        self.reuse_min_tokens = max(1, int(reuse_min_tokens))
        self.reuse_max_tokens = int(reuse_max_tokens)   # bound on stored rows x width
        # ... and on the bytes the stored caches pin (K/V of every layer + final hidden)
        c = model.cfg
        esz = torch.finfo(model.dtype).bits // 8
        self.bytes_per_cached_token = (c.n_layers * 2 * c.n_kv_heads * c.head_dim + c.d_model) * esz
        self.reuse_max_bytes = int(reuse_max_bytes)
        self._store: List[tuple] = []     # (PrefixCache, [rows, width] ids, -1 padded), newest last
        self._store_lock = threading.Lock()
        self.reuse_stats = {"prefills": 0, "reused": 0, "tokens": 0, "tokens_run": 0}

    # --- prefixes ---------------------------------------------------------------
    @torch.no_grad()
    def prefill(self, prefixes: Sequence[Sequence[int]]) -> PrefixCache:
        if any(len(p) == 0 for p in prefixes):
            raise ValueError("every prefix needs at least one token (BOS)")
        rows = [np.asarray(list(p), dtype=np.int64) for p in prefixes]
        total = sum(r.shape[0] for r in rows)
        self.reuse_stats["prefills"] += 1
        self.reuse_stats["tokens"] += total
        with self._store_lock:
            plan = self._reuse_plan(rows) if self.reuse_caches > 0 else None
        if plan is not None:
            cache = self._prefill_extending(prefixes, rows, *plan)
            self.reuse_stats["reused"] += 1
        else:
            self.reuse_stats["tokens_run"] += len(rows) * max(r.shape[0] for r in rows)
            ids, lens = _pad(prefixes, self.device)
            kv, h, valid = self.model.prefill(ids, lens)
            last = h[torch.arange(h.shape[0], device=self.device), lens - 1]
            P = ids.shape[1]
            pos = torch.arange(P, device=self.device)[None].expand(ids.shape[0], P)
            cache = PrefixCache(kv=kv, lengths=lens, last_hidden=last, pos=pos, valid=valid,
                                hidden=h, ids=ids)
        if (self.reuse_caches > 0 and cache.ids.numel() <= self.reuse_max_tokens and
                cache.ids.numel() * self.bytes_per_cached_token <= self.reuse_max_bytes):
            with self._store_lock:
                self._store.append((cache, _id_matrix(rows)))
                del self._store[:-self.reuse_caches]
                while (sum(c.ids.numel() for c, _ in self._store) > self.reuse_max_tokens or
                       sum(c.ids.numel() for c, _ in self._store) * self.bytes_per_cached_token
                       > self.reuse_max_bytes):
                    del self._store[0]
        return cache

    @torch.no_grad()
    def prefill_streams(self, prefixes: Sequence[Sequence[int]], bucket_ratio: float = 1.25,
                        bucket_tokens: int = 1 << 16, reserve: int = 0) -> StreamPrefix:
        """Prefill for the stream decode (bf16 models): prompts of very different lengths
        (64 agent prompts of ~200 tokens and a reference prompt listing every opinion)
        are prefilled in length buckets (padding <= bucket_ratio, <= bucket_tokens padded
        tokens per forward) and their K/V written straight into the ragged FusedPrefix
        buffers — nothing is padded to the longest prompt.  ``reserve``: key slots left
        free after every prefix for tokens appended later (append_prefix_tokens)."""
        if any(len(p) == 0 for p in prefixes):
            raise ValueError("every prefix needs at least one token (BOS)")
        m = self.model
        c = m.cfg
        dev = self.device
        lens = [len(p) for p in prefixes]
        n = len(prefixes)
        off = _offsets32([x + int(reserve) for x in lens])
        Lp = off[-1]
        ks = [torch.zeros(c.n_kv_heads, Lp, c.head_dim, dtype=m.dtype, device=dev)
              for _ in range(c.n_layers)]
        vrs = [torch.zeros(c.n_kv_heads, Lp, c.head_dim, dtype=m.dtype, device=dev)
               for _ in range(c.n_layers)]            # V rows; tiled (ops.blocked_vt) at the end
        last = torch.empty(n, c.d_model, dtype=m.dtype, device=dev)
        order = sorted(range(n), key=lambda i: lens[i])
        j = 0
        while j < n:
            b = [order[j]]
            j += 1
            while (j < n and lens[order[j]] <= bucket_ratio * lens[b[0]]
                   and (len(b) + 1) * lens[order[j]] <= bucket_tokens):
                b.append(order[j])
                j += 1
            ids, lt = _pad([prefixes[i] for i in b], dev)
            nb, Pb = ids.shape
            if m.fused_ok():
                # the prompts as streams over an empty prefix: causal attention over their
                # own tokens on cs_prefix_attention (O(T) memory; no T x T score matrix
                # for a several-thousand-token reference prompt)
                ldh = _ceil32(Pb)
                hk = [torch.zeros(nb, c.n_kv_heads, ldh, c.head_dim, dtype=m.dtype, device=dev)
                      for _ in range(c.n_layers)]
                hv = [torch.zeros(nb, c.n_kv_heads, ldh // 32, c.head_dim, 32, dtype=m.dtype,
                                  device=dev) for _ in range(c.n_layers)]
                h = m.forward_streams(ids.reshape(-1), _empty_prefix(m), hk, hv,
                                      torch.zeros(1, dtype=torch.int32, device=dev), 1, Pb,
                                      group_prefix=torch.zeros(nb, dtype=torch.int32, device=dev),
                                      group_prefix_host=[0] * nb)
                h = h.view(nb, Pb, -1)
                kv = [(k, ops.rows_from_blocked(v)) for k, v in zip(hk, hv)]
            else:
                kv, h, _ = m.prefill(ids, lt)
            last[torch.as_tensor(b, device=dev)] = h[torch.arange(nb, device=dev), lt - 1]
            for li, (k, v) in enumerate(kv):
                for r, i in enumerate(b):
                    ks[li][:, off[i]:off[i] + lens[i]] = k[r, :, :lens[i]]
                    vrs[li][:, off[i]:off[i] + lens[i]] = v[r, :, :lens[i]]
            del kv, h
        vts = [ops.blocked_vt(v) for v in vrs]
        del vrs
        fp = FusedPrefix(k=ks, vt=vts, off=torch.as_tensor(off[:-1], dtype=torch.int64, device=dev),
                         lengths=torch.as_tensor(lens, dtype=torch.int32, device=dev),
                         max_len=max(lens), lens_host=list(lens),
                         cap_host=[off[i + 1] - off[i] for i in range(n)], off_host=off[:-1])
        return StreamPrefix(fused=fp, last_hidden=last,
                            lengths=torch.as_tensor(lens, dtype=torch.long, device=dev), lens=lens)

    @torch.no_grad()
    def append_prefix_tokens(self, sp: StreamPrefix, hist_k: torch.Tensor, hist_vt: torch.Tensor,
                             streams: Sequence[int], slot: int, hidden: torch.Tensor,
                             which: Optional[Sequence[int]] = None, v_rows: bool = False) -> None:
        """Append one token to prefixes of ``sp`` in place: prefix p (every prefix, or those
        in ``which``) takes the K/V that stream (buffer row) streams[i] holds in history slot
        ``slot`` of hist_k [L, S, Hkv, ldh, D] / hist_vt [L, S, Hkv, ldh/32, D, 32] (v_rows: V
        row-layout [L, S, Hkv, ldh, D], a TokenTree's buffers) as its next key, and
        hidden[i] (that stream's final-norm hidden) as its new last hidden.  The token's
        K/V were computed by the stream forward that scored it, so committing a lookahead
        token costs copies, not a forward (the reference re-encodes the grown prompt,
        src/methods/finite_lookahead.py:99-153 via src/utils.py:249-259)."""
        fp = sp.fused
        which = list(range(len(sp.lens))) if which is None else list(which)
        if len(streams) != len(which) or fp.cap_host is None:
            raise ValueError("append_prefix_tokens needs a prefill_streams prefix and one stream "
                             "per appended prefix")
        for p in which:
            if sp.lens[p] + 1 > fp.cap_host[p]:
                raise ValueError("prefix capacity exhausted (prefill_streams reserve)")
        dev = self.device
        pw = torch.as_tensor(which, dtype=torch.long, device=dev)
        rows = torch.as_tensor([fp.off_host[p] + sp.lens[p] for p in which], dtype=torch.long,
                               device=dev)
        st = torch.as_tensor(list(streams), dtype=torch.long, device=dev)
        tile, lane = rows // 32, rows % 32
        for li in range(len(fp.k)):
            # K [Hkv, Lp, D] <- hist_k[l][s, :, slot, :]; V^T [Hkv, Lp/32, D, 32] column
            fp.k[li][:, rows, :] = hist_k[li][st, :, slot, :].transpose(0, 1)
            v = hist_vt[li][st, :, slot, :] if v_rows else \
                hist_vt[li][st, :, slot // 32, :, slot % 32]                # [n, Hkv, D]
            fp.vt[li][:, tile, :, lane] = v          # (separated advanced indices: [n, Hkv, D])
        for p in which:
            sp.lens[p] += 1
            fp.lens_host[p] += 1
        fp.max_len = max(fp.max_len, max(sp.lens[p] for p in which))
        fp.lengths[pw] += 1
        sp.lengths[pw] += 1
        sp.last_hidden[pw] = hidden.to(sp.last_hidden.dtype)

    def reset_prefix_store(self) -> None:
        with self._store_lock:
            self._store = []

    def _reuse_plan(self, rows):
        """(stored cache, source row per prefix, reused length per prefix) from the stored
        cache that saves the most padded work, or None when a full prefill is as cheap."""
        best = None
        full_cost = len(rows) * max(r.shape[0] for r in rows)
        for cache, smat in self._store:
            src, lcp = [], []
            for r in rows:
                bi, bl = _best_lcp(r, smat)
                bl = min(bl, r.shape[0] - 1)          # at least one token runs
                if bl < self.reuse_min_tokens:
                    bl = 0
                src.append(bi)
                lcp.append(bl)
            cost = len(rows) * max(r.shape[0] - l for r, l in zip(rows, lcp))
            if best is None or cost < best[0]:
                best = (cost, cache, src, lcp)
        if best is None or 2 * best[0] > full_cost:
            return None
        self.reuse_stats["tokens_run"] += best[0]
        return best[1], best[2], best[3]

    def _prefill_extending(self, prefixes, rows, base: PrefixCache, src, lcp) -> PrefixCache:
        """The PrefixCache ``prefill(prefixes)`` returns, with row r's first lcp[r]
        positions (K/V, hidden) taken from ``base`` row src[r] and only the rest run
        through the model (extend over base's K/V, visible up to lcp[r])."""
        dev = self.device
        R = len(rows)
        lens_l = [r.shape[0] for r in rows]
        S = max(n - l for n, l in zip(lens_l, lcp))
        suf = torch.zeros(R, S, dtype=torch.long)
        for i, (r, l) in enumerate(zip(rows, lcp)):
            suf[i, :r.shape[0] - l] = torch.from_numpy(r[l:])
        suf = suf.to(dev, non_blocking=True)
        l_t = torch.as_tensor(lcp, dtype=torch.long).to(dev, non_blocking=True)
        s_t = torch.as_tensor(src, dtype=torch.long).to(dev, non_blocking=True)
        Pc = base.ids.shape[1]
        pos = l_t[:, None] + torch.arange(S, device=dev)[None]
        cmask = torch.arange(Pc, device=dev)[None] < l_t[:, None]
        room = (0, 0, 0, S)            # free key slots: extend writes the new keys there
        ctx = [(F.pad(k, room)[s_t], F.pad(v, room)[s_t]) for k, v in base.kv]
        h_new, _ = self.model.extend(suf, pos, ctx, cmask, base.pos[s_t])
        # contiguous layout, position j of row r: base row j (j < lcp) or new j - lcp
        ids, lens = _pad(prefixes, dev)
        P = ids.shape[1]
        j = torch.arange(P, device=dev)[None]
        idx = torch.where(j < l_t[:, None], j, Pc + (j - l_t[:, None]).clamp(max=S - 1))
        idx = idx.clamp(max=Pc + S - 1)

        def merge(both):                         # [R, H, Pc + S, D] -> [R, H, P, D]
            g = idx[:, None, :, None].expand(R, both.shape[1], P, both.shape[3])
            return torch.gather(both, 2, g)

        kv = [(merge(kb), merge(vb)) for kb, vb in ctx]
        hb = torch.cat([base.hidden[s_t], h_new], dim=1)
        h = torch.gather(hb, 1, idx[:, :, None].expand(R, P, hb.shape[2]))
        valid = j < lens[:, None]
        last = h[torch.arange(R, device=dev), lens - 1]
        return PrefixCache(kv=kv, lengths=lens, last_hidden=last,
                           pos=j.expand(R, P), valid=valid, hidden=h, ids=ids)

    @torch.no_grad()
    def prefix_tail_logprobs(self, cache: PrefixCache, m: int) -> torch.Tensor:
        """log p of the last m tokens of every prefix given what precedes them
        ([n_prefix, m], NaN where the prefix is shorter than m + 1)."""
        n = cache.lengths.shape[0]
        if m <= 0:
            return torch.empty(n, 0, dtype=torch.float32, device=self.device)
        j = cache.lengths[:, None] - m + torch.arange(m, device=self.device)[None]   # token pos
        ok = j >= 1
        jj = j.clamp(min=1)
        rows = torch.arange(n, device=self.device)[:, None]
        h = cache.hidden[rows, jj - 1].reshape(n * m, -1)
        t = cache.ids[rows, jj].reshape(n * m, 1)
        lp = self.rows_logprobs(h, t).view(n, m)
        return torch.where(ok, lp, torch.full_like(lp, float("nan")))

    @torch.no_grad()
    def next_hidden(self, cache: PrefixCache, owner: Sequence[int],
                    conts: Sequence[Sequence[int]]) -> torch.Tensor:
        """Hidden state predicting the token that follows prefix[owner[r]] + conts[r]."""
        dev = self.device
        own = torch.as_tensor(list(owner), dtype=torch.long, device=dev)
        out = cache.last_hidden[own].clone()
        if not any(len(c) for c in conts):
            return out
        toks, lens = _pad(conts, dev)
        pos = cache.lengths[own][:, None] + torch.arange(toks.shape[1], device=dev)[None]
        room = (0, 0, 0, toks.shape[1])             # free key slots (see _score_chunk)
        ctx = [(F.pad(k, room)[own], F.pad(v, room)[own]) for k, v in cache.kv]
        h, _ = self.model.extend(toks, pos, ctx, cache.valid[own], cache.pos[own])
        has = lens > 0
        idx = (lens - 1).clamp(min=0)
        hl = h[torch.arange(len(conts), device=dev), idx]
        return torch.where(has[:, None], hl, out)

    # --- one logits block -> token log-probs --------------------------------------
    def rows_logprobs(self, hidden: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        """hidden [rows, d] -> logits [rows, V] (LM head) -> log p(targets) [rows, k]."""
        logits = self.model.lm_head(hidden)
        tok, _ = ops.logsoftmax_gather(logits, targets.to(torch.int32), softcap=self.softcap,
                                       workspace=self.ws)
        return tok

    # --- continuation scoring ---------------------------------------------------
    @torch.no_grad()
    def score(self, cache: PrefixCache, owner: Sequence[int],
              conts: Sequence[Sequence[int]]) -> torch.Tensor:
        """Token log-probs of every continuation under its owner's prefix.

        Returns a flat float32 tensor: for stream r the slice
        [off[r], off[r+1]) holds log p(conts[r][t] | prefix[owner[r]], conts[r][:t]).
        Use ``offsets(conts)`` for the CSR boundaries.
        """
        R = len(conts)
        lens = [len(c) for c in conts]
        out = torch.empty(sum(lens), dtype=torch.float32, device=self.device)
        grouping = _uniform_groups(owner)
        if (grouping is not None and self.fused_scoring and R and max(lens) > 1 and
                self.model.fused_ok(int(cache.ids.shape[1]) + max(lens))):
            self._score_fused(cache, grouping, conts, lens, out)
            return out
        # chunk streams so that the logits block stays bounded
        r0, o0 = 0, 0
        while r0 < R:
            r1, rows = r0, 0
            while r1 < R and (r1 == r0 or (rows + lens[r1] <= self.max_rows and
                                           r1 - r0 < self.max_streams)):
                rows += lens[r1]
                r1 += 1
            self._score_chunk(cache, owner[r0:r1], conts[r0:r1], out[o0:o0 + rows])
            r0, o0 = r1, o0 + rows
        return out

    def _score_fused(self, cache, grouping, conts, lens, out):
        """Scoring over shared prefixes on the stream kernels: every chunk is whole groups
        (all n_str continuations of some prefixes), padded to the longest continuation;
        continuation tokens 0..T-2 run through forward_streams (each stream's own tokens
        in one reusable history buffer, the prefix K/V read once per (prefix, head) per
        layer), token 0 is scored from the prefix's last hidden, rows -> LM head ->
        cs_logsoftmax_gather.  Replaces the per-stream gathered [prefix | tokens] contexts
        of _score_chunk (one copy of each prefix per candidate per layer)."""
        dev = self.device
        m = self.model
        c = m.cfg
        groups, n_str = grouping
        pfx = fused_prefix(cache)          # once per call, shared by the chunks
        T = max(lens)
        per_group = n_str * T
        g_per_chunk = max(1, self.fused_max_rows // max(per_group, 1))
        o0 = 0
        for g0 in range(0, len(groups), g_per_chunk):
            gs = groups[g0:g0 + g_per_chunk]
            S = len(gs) * n_str
            cs = conts[g0 * n_str:g0 * n_str + S]
            ls = lens[g0 * n_str:g0 * n_str + S]
            toks, lens_t = _pad(cs, dev)
            Tc = toks.shape[1]
            own = torch.as_tensor(gs, dtype=torch.long, device=dev).repeat_interleave(n_str)
            last = cache.last_hidden[own]
            if Tc > 1:
                ldh = _ceil32(Tc - 1)
                hk = torch.zeros(S, c.n_kv_heads, ldh, c.head_dim, dtype=m.dtype, device=dev)
                hv = torch.zeros(S, c.n_kv_heads, ldh // 32, c.head_dim, 32, dtype=m.dtype,
                                 device=dev)
                hb = torch.zeros(1, dtype=torch.int32, device=dev)
                gp = torch.as_tensor(gs, dtype=torch.int32, device=dev)
                # one history buffer serves every layer: a chunk's K/V are not kept
                h = m.forward_streams(toks[:, :Tc - 1].reshape(-1), pfx, [hk] * c.n_layers,
                                      [hv] * c.n_layers, hb, n_str, Tc - 1, group_prefix=gp,
                                      group_prefix_host=list(gs))
                hpad = torch.cat([last[:, None, :], h.view(S, Tc - 1, -1)], dim=1)   # [S, Tc, d]
                del h, hk, hv
            else:
                hpad = last[:, None, :]
            rows = sum(ls)
            if all(L == Tc for L in ls):
                rows_h, rows_t = hpad.reshape(S * Tc, -1), toks.reshape(-1, 1)
            else:
                idx_r = torch.repeat_interleave(torch.arange(S, device=dev), lens_t)
                idx_t = torch.cat([torch.arange(L, device=dev) for L in ls])
                rows_h, rows_t = hpad[idx_r, idx_t], toks[idx_r, idx_t][:, None]
            out[o0:o0 + rows].copy_(self.rows_logprobs(rows_h, rows_t).view(-1))
            o0 += rows

    def _score_chunk(self, cache, owner, conts, out):
        dev = self.device
        m = self.model
        R = len(conts)
        own = torch.as_tensor(list(owner), dtype=torch.long, device=dev)
        toks, lens = _pad(conts, dev)
        T = toks.shape[1]
        # hidden state that predicts each continuation token:
        # t = 0 -> last prefix position; t > 0 -> continuation position t-1
        need_ext = T > 1
        if need_ext:
            inp = toks[:, :T - 1]
            plen = cache.lengths[own]
            pos = plen[:, None] + torch.arange(T - 1, device=dev)[None]
            # per-stream context with T - 1 free key slots: extend writes the new keys into
            # them instead of concatenating per layer (padding the n_prefix source rows is
            # cheap; the gather to R streams happens once either way)
            room = (0, 0, 0, T - 1)
            ctx = [(F.pad(k, room)[own], F.pad(v, room)[own]) for k, v in cache.kv]
            h, _ = m.extend(inp, pos, ctx, cache.valid[own], cache.pos[own])
            del ctx
        flat_h, flat_t = [], []
        lens_l = lens.tolist()
        last = cache.last_hidden[own]
        # gather rows in stream-major order
        idx_r = torch.repeat_interleave(torch.arange(R, device=dev), lens)
        idx_t = torch.cat([torch.arange(L, device=dev) for L in lens_l]) if R else \
            torch.empty(0, dtype=torch.long, device=dev)
        if need_ext:
            hpad = torch.cat([last[:, None, :], h], dim=1)   # [R, T, d]
        else:
            hpad = last[:, None, :]
        rows_h = hpad[idx_r, idx_t]
        rows_t = toks[idx_r, idx_t][:, None]
        tok = self.rows_logprobs(rows_h, rows_t)
        out.copy_(tok.view(-1))
        del flat_h, flat_t

    @torch.no_grad()
    def score_tree(self, cache: PrefixCache, owner: Sequence[int], tokens: Sequence[int],
                   parents: Sequence[int]) -> torch.Tensor:
        """Log-probs of every node of ONE token tree under each owner's prefix.

        tokens[i] is node i's token, parents[i] its parent node (< i) or -1 for a child of
        the prefix.  Node i's log-prob is log p(tokens[i] | prefix, ancestors of i): every
        node is scored once however many paths share it (a path's log-probs are its
        nodes'), in one extend over all nodes with a tree attention mask (ancestors and
        self), one logits row per node, cs_logsoftmax_gather.  Returns [len(owner), N]."""
        dev = self.device
        R, N = len(owner), len(tokens)
        if N == 0:
            return torch.empty(R, 0, dtype=torch.float32, device=dev)
        depth = [0] * N
        anc = torch.zeros(N, N, dtype=torch.bool)
        for i, p in enumerate(parents):
            if p >= i:
                raise ValueError("parents must precede their children")
            depth[i] = 0 if p < 0 else depth[p] + 1
            if p >= 0:
                anc[i] = anc[p]
            anc[i, i] = True
        own = torch.as_tensor(list(owner), dtype=torch.long, device=dev)
        toks = torch.as_tensor(list(tokens), dtype=torch.long, device=dev)[None].expand(R, N)
        last = cache.last_hidden[own]                                   # [R, d]
        # only internal nodes (some node's parent) need a forward: their outputs predict
        # their children; leaves are scored from their parent's row
        internal = sorted({p for p in parents if p >= 0})
        slot = {n: j + 1 for j, n in enumerate(internal)}               # 0 = the prefix
        par_slot = torch.as_tensor([slot.get(p, 0) for p in parents], dtype=torch.long,
                                   device=dev)
        if internal:
            ii = torch.as_tensor(internal, dtype=torch.long)
            it = toks[:, ii.to(dev)]
            pos = cache.lengths[own][:, None] + torch.as_tensor([depth[n] for n in internal],
                                                                device=dev)[None]
            room = (0, 0, 0, len(internal))         # free key slots (see _score_chunk)
            ctx = [(F.pad(k, room)[own], F.pad(v, room)[own]) for k, v in cache.kv]
            h, _ = self.model.extend(it, pos, ctx, cache.valid[own], cache.pos[own],
                                     self_mask=anc[ii][:, ii].to(dev))
            hpad = torch.cat([last[:, None, :], h], dim=1)
            rows_h = hpad[:, par_slot]                                  # [R, N, d]
        else:
            rows_h = last[:, None, :].expand(R, N, last.shape[-1])
        tgt = toks.reshape(R * N, 1).to(torch.int32)
        return self.rows_logprobs(rows_h.reshape(R * N, -1), tgt).view(R, N)

    @staticmethod
    def offsets(conts: Sequence[Sequence[int]], device) -> torch.Tensor:
        off = [0]
        for c in conts:
            off.append(off[-1] + len(c))
        return torch.as_tensor(off, dtype=torch.int32, device=device)


class BeamState:
    """Per-(prefix, beam) incremental decode state for beam search.

    Streams are laid out prefix-major: stream s = p * n_beams + b.  Each step
    appends one token to every live beam (all beams share one length), so the
    generated K/V is a dense [S, Hkv, G, D] tensor per layer.
    """

    def __init__(self, engine: ScoringEngine, cache: PrefixCache, n_prefix: int):
        self.e = engine
        self.cache = cache
        self.n_prefix = n_prefix
        self.n_beams = 1
        self.gen_kv: Optional[list] = None   # per layer (k, v) [S, Hkv, G, D]
        self.G = 0
        # hidden that predicts the next token of each stream: start = last prefix position
        self.next_hidden = cache.last_hidden.clone()          # [S, d] with n_beams = 1

    def next_logprobs(self, targets: torch.Tensor) -> torch.Tensor:
        """targets [n_prefix, n_beams, k] int -> log-probs [n_prefix, n_beams, k]."""
        P, B, K = targets.shape
        tok = self.e.rows_logprobs(self.next_hidden, targets.reshape(P * B, K))
        return tok.view(P, B, K)

    def agent_logits(self, n_prefix: int) -> torch.Tensor:
        """Logits rows [n_prefix * n_beams, V] of the first n_prefix prefixes (the agents),
        row p * n_beams + b — the layout cs_beam_step takes."""
        return self.e.model.lm_head(self.next_hidden[:n_prefix * self.n_beams])

    def next_logits(self, prefix_idx: int) -> torch.Tensor:
        """Raw logits rows [n_beams, V] of one prefix (e.g. the reference policy)."""
        B = self.n_beams
        h = self.next_hidden[prefix_idx * B:(prefix_idx + 1) * B]
        return self.e.model.lm_head(h)

    @torch.no_grad()
    def advance(self, parent: Sequence[int], tokens: Sequence[int]) -> None:
        """New beams j = (parent beam parent[j], appended token tokens[j]) for every prefix."""
        dev = self.e.device
        m = self.e.model
        P, Bo, Bn = self.n_prefix, self.n_beams, len(parent)
        par = torch.as_tensor(list(parent), dtype=torch.long, device=dev)
        src = (torch.arange(P, device=dev)[:, None] * Bo + par[None, :]).reshape(-1)   # [P*Bn]
        own = torch.arange(P, device=dev).repeat_interleave(Bn)
        tok = torch.as_tensor(list(tokens), dtype=torch.long, device=dev).repeat(P)[:, None]
        c = self.cache
        plen = c.lengths[own]
        pos = (plen + self.G)[:, None]
        pre_mask = c.valid[own]
        pre_pos = c.pos[own]
        if self.G > 0:
            gpos = plen[:, None] + torch.arange(self.G, device=dev)[None]
            cmask = torch.cat([pre_mask, torch.ones(len(own), self.G, dtype=torch.bool,
                                                    device=dev)], 1)
            cpos = torch.cat([pre_pos, gpos], 1)
        else:
            cmask, cpos = pre_mask, pre_pos
        # per stream one buffer [prefix | history | 1 free slot]: the prefix rows padded once
        # and gathered, the parents' history written in, the new key written into the slot
        # by extend; the next history is a view of the buffer (no concatenations)
        Pm = c.kv[0][0].shape[2]
        room = (0, 0, 0, self.G + 1)
        ctx = []
        for li, (pk, pv) in enumerate(c.kv):
            kb, vb = F.pad(pk, room)[own], F.pad(pv, room)[own]
            if self.G > 0:
                gk, gv = self.gen_kv[li]
                kb[:, :, Pm:Pm + self.G] = gk[src]
                vb[:, :, Pm:Pm + self.G] = gv[src]
            ctx.append((kb, vb))
        h, _ = m.extend(tok, pos, ctx, cmask, cpos)
        # compact history copies: views would keep every layer's whole [prefix | history]
        # context buffer alive until the next advance (2x the persistent K/V at peak)
        self.gen_kv = [(kb[:, :, Pm:].clone(), vb[:, :, Pm:].clone()) for kb, vb in ctx]
        del ctx
        self.G += 1
        self.n_beams = Bn
        self.next_hidden = h[:, 0, :]


def _ceil32(n: int) -> int:
    return max(32, (int(n) + 31) // 32 * 32)


@dataclass
class FusedPrefix:
    """Prefix K/V in the cs_prefix_attention layouts (include/consensus_scoring.h): all
    prefixes of one prefill in one ragged buffer per layer, prefix p's keys at rows
    off[p] .. off[p] + lengths[p] (off[p] % 32 == 0, each prefix padded to 32 keys)."""
    k: list                     # per layer [Hkv, Lp, D]
    vt: list                    # per layer [Hkv, Lp/32, D, 32] (V^T in 32-key tiles)
    off: torch.Tensor           # [n_prefix] int64 (device)
    lengths: torch.Tensor       # [n_prefix] int32 (device)
    max_len: int                # host copy of max(lengths)
    lens_host: Optional[List[int]] = None   # host copies of the lengths (or bounds), if known
    cap_host: Optional[List[int]] = None    # key slots allotted to each prefix (prefill_streams)
    off_host: Optional[List[int]] = None    # host copy of off


@dataclass
class StreamPrefix:
    """What the stream decode needs of a prefill (engine.prefill_streams): the ragged
    prefix K/V, each prefix's last final-norm hidden and its length."""
    fused: FusedPrefix
    last_hidden: torch.Tensor   # [n_prefix, d]
    lengths: torch.Tensor       # [n_prefix] int64 (device)
    lens: List[int]             # host copy


def _empty_prefix(m: Model) -> FusedPrefix:
    """One prefix of length 0 (prefill of prompts as streams of their own tokens)."""
    c = m.cfg
    dev = m.device
    return FusedPrefix(
        k=[torch.zeros(c.n_kv_heads, 32, c.head_dim, dtype=m.dtype, device=dev)] * c.n_layers,
        vt=[torch.zeros(c.n_kv_heads, 1, c.head_dim, 32, dtype=m.dtype, device=dev)] * c.n_layers,
        off=torch.zeros(1, dtype=torch.int64, device=dev),
        lengths=torch.zeros(1, dtype=torch.int32, device=dev), max_len=0, lens_host=[0])


def _offsets32(lens: Sequence[int]) -> List[int]:
    off, o = [], 0
    for n in lens:
        off.append(o)
        o += _ceil32(n)
    return off + [o]


def fused_prefix(cache: PrefixCache) -> FusedPrefix:
    """A padded prefill's K/V re-laid for the stream kernels (prefix p at rows p * ldp,
    ldp = the padded length rounded up to 32, zero-filled; V^T in 32-key tiles).  One copy."""
    n, Hkv, P, D = cache.kv[0][0].shape
    ldp = _ceil32(P)
    ks, vts = [], []
    for k, v in cache.kv:
        kp = torch.zeros(Hkv, n, ldp, D, dtype=k.dtype, device=k.device)
        kp[:, :, :P] = k.transpose(0, 1)
        vr = torch.zeros(Hkv, n, ldp, D, dtype=v.dtype, device=v.device)
        vr[:, :, :P] = v.transpose(0, 1)
        ks.append(kp.view(Hkv, n * ldp, D))
        vts.append(ops.blocked_vt(vr.view(Hkv, n * ldp, D)))
    dev = cache.lengths.device
    return FusedPrefix(k=ks, vt=vts, off=torch.arange(n, device=dev, dtype=torch.int64) * ldp,
                       lengths=cache.lengths.to(torch.int32), max_len=P)


class DecodeState:
    """Static-shape incremental decode of n_beams streams per prefix on the HIP stream
    kernels (bf16 models; BeamState is the general eager path).

    Streams are prefix-major, s = p * n_beams + b, always n_beams of them per prefix (the
    caller pads missing beams with copies and ignores their candidates).  Every stream's
    generated K/V lives in a preallocated history buffer [S, Hkv, ldh, D], slot t = the
    token of step t; the prefix K/V is shared by the stream's n_beams siblings through
    cs_prefix_attention.  ``advance`` = inherit the parents' histories, forward the new
    tokens with hist_base = t read from device memory, keep the final-norm hidden.  The
    history is row-layout (K and V [S, Hkv, ldh, D]) behind a [S, ldh] slot table: slot t of
    stream s is row rows[s, t], written once by the step that made it and never moved; a
    step's inheritance is one table update (cs_hist_rows_update, a ping-pong pair of tables)
    and the attention gathers through it (cs_prefix_attention_rows).  After the first (eager) advance each parity's step is captured once in a hipGraph and
    replayed, so a decode step costs one graph launch plus its inputs' copies; ``post``
    (optional, fixed per state) is captured with it, e.g. the LM head + the fused
    cs_beam_decode_step of the beam search.

    Restates the reference's per-step re-encoding of every agent prompt + beam text
    (src/methods/beam_search.py:491-538 through src/utils.py:249-259) as one token per
    stream per step."""

    def __init__(self, engine: "ScoringEngine", cache, n_prefix: int, n_beams: int,
                 max_steps: int, use_graphs: bool = True):
        """cache: a StreamPrefix (engine.prefill_streams) or a PrefixCache (re-laid)."""
        self.e = engine
        m = engine.model
        c = m.cfg
        self.P, self.B = int(n_prefix), int(n_beams)
        self.S = self.P * self.B
        dev = engine.device
        self.pfx = cache.fused if isinstance(cache, StreamPrefix) else fused_prefix(cache)
        self.ldh = _ceil32(max_steps)
        self.max_steps = int(max_steps)

        # K and V of every layer and stream, row-major [L, S, Hkv, ldh, D] each, written in
        # place (never copied); a ping-pong pair of slot tables [S, ldh] so a queued step can
        # be undone (rewind)
        kv = torch.zeros(2, c.n_layers, self.S, c.n_kv_heads, self.ldh, c.head_dim,
                         dtype=m.dtype, device=dev)
        self.k_hist, self.v_hist = kv[0], kv[1]
        self.rows = [torch.arange(self.S, dtype=torch.int32, device=dev)[:, None]
                     .expand(self.S, self.ldh).contiguous() for _ in range(2)]
        self.cur = 0
        self.steps = 0                                   # tokens appended so far (host copy)
        self.hist_base = torch.zeros(1, dtype=torch.int32, device=dev)
        # a step's inputs (parent stream, new token per stream): ONE pinned host buffer and
        # ONE device buffer, one asynchronous copy per step (the graphs read the device side)
        self._in_h = [torch.empty(2 * self.S, dtype=torch.long, pin_memory=True) for _ in range(2)]
        self._in_ev: List[Optional[torch.cuda.Event]] = [None, None]
        self._in_d = torch.zeros(2 * self.S, dtype=torch.long, device=dev)
        self._in_d[:self.S] = torch.arange(self.S, dtype=torch.long, device=dev)
        self.src, self.tok = self._in_d[:self.S], self._in_d[self.S:]
        self.hidden = cache.last_hidden.repeat_interleave(self.B, dim=0).contiguous()   # [S, d]
        self.use_graphs = use_graphs
        # captured step graphs keyed by (parity, weak reference to ``post``): a ``post``
        # closure usually references this state, so a strong key would make a reference
        # cycle that only the cyclic collector frees -- possibly in the middle of a later
        # capture, where destroying a graph is refused (and aborts the process)
        self._graphs: dict = {}
        self._pool = None
        # the attention work plans the captured graphs point into (ops.retain_plans)
        self._plans: dict = {}

    @property
    def n_beams(self) -> int:
        return self.B

    def _body(self, post) -> None:
        m = self.e.model
        rows = self.rows[1 - self.cur]
        ops.hist_rows_update(self.rows[self.cur], rows, self.src, self.hist_base, n_rows=self.S)
        h = m.forward_streams(self.tok, self.pfx, list(self.k_hist.unbind(0)),
                              list(self.v_hist.unbind(0)), self.hist_base, self.B, 1,
                              hist_rows=rows)
        self.hidden.copy_(h)
        self.hist_base += 1
        if post is not None:
            post()

    @torch.no_grad()
    def advance(self, parent: Sequence[int], tokens: Sequence[int], post=None) -> None:
        """New beam j of every prefix = (parent beam parent[j], token tokens[j]), j < n_beams."""
        if len(parent) != self.B or len(tokens) != self.B:
            raise ValueError(f"advance takes exactly n_beams = {self.B} (parent, token) pairs")
        if self.steps >= self.ldh:
            raise ValueError("history capacity exhausted (max_steps)")
        dev = self.e.device
        P, B, S = self.P, self.B, self.S
        # two pinned staging buffers: the one written now was last copied two steps ago;
        # wait for that copy only (back-to-back replays keep the queue full)
        k = self.steps & 1
        if self._in_ev[k] is not None:
            self._in_ev[k].synchronize()
        h = self._in_h[k].numpy()
        h[:S] = (np.arange(P)[:, None] * B + np.asarray(parent, dtype=np.int64)[None, :]).reshape(-1)
        h[S:] = np.tile(np.asarray(tokens, dtype=np.int64), P)
        self._in_d.copy_(self._in_h[k], non_blocking=True)   # stream-ordered after the last replay
        ev = self._in_ev[k] = torch.cuda.Event()
        ev.record()
        self._replay(post)

    def _replay(self, post) -> None:
        dev = self.e.device
        key = (self.cur, None if post is None else weakref.ref(post))
        if not self.use_graphs or self.steps == 0:
            with ops.retain_plans(self._plans):
                self._body(post)                  # the first step runs eagerly (warm-up)
        else:
            g = self._graphs.get(key)
            if g is None:
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream(device=dev)
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s), ops.retain_plans(self._plans):
                    with torch.cuda.graph(g, pool=self._pool, stream=s):
                        self._body(post)
                torch.cuda.current_stream().wait_stream(s)
                self._pool = g.pool()
                self._graphs[key] = g
            g.replay()
        self.cur = 1 - self.cur
        self.steps += 1

    @torch.no_grad()
    def advance_device(self, post=None) -> None:
        """advance() with the step's inputs already in device memory (``src`` / ``tok``,
        e.g. written by the previous step's ``post`` from its own candidate order): no
        host input, so the step can be queued before the host has read the last one."""
        if self.steps >= self.ldh:
            raise ValueError("history capacity exhausted (max_steps)")
        self._replay(post)

    def rewind(self) -> None:
        """Undo the last advance (queued after it on the stream): the ping-pong parity, the
        step count and the device-side history base.  The other history buffer it wrote is
        rewritten by the next advance (it reads only the buffer this one read)."""
        self.cur = 1 - self.cur
        self.steps -= 1
        self.hist_base -= 1

    def release(self) -> None:
        """Drop the captured step graphs and their memory pool now (after the work that
        replays them has finished), instead of whenever the garbage collector reaches the
        state's reference cycles (its ``post`` closures)."""
        if self._graphs:
            torch.cuda.current_stream().synchronize()
        self._graphs.clear()
        self._pool = None
        self._plans.clear()


def tree_pool(engine: "ScoringEngine", n_prefix: int, bf: int, max_depth: int) -> dict:
    """A TokenTree K / V pool sized up front for the largest tree of a lookahead statement:
    under each of n_prefix prefixes the nodes of levels 1 .. max_depth - 1 (the expanded
    ones; b + b^2 + ... + b^(d-1), at least the one committed node of a depth-1 tree).
    Allocated before the first stream forward, so the packed-weight copies made there
    (Model.pack_decode_weights) budget around it instead of leaving the tree to grow into
    the reserve (a 70B lookahead outgrew 16 GB)."""
    c = engine.model.cfg
    per = max(1, sum(bf ** t for t in range(1, max(1, max_depth))))
    rows = max(256, n_prefix * per)
    shape = (c.n_layers, rows, c.n_kv_heads, _ceil32(max(1, max_depth)), c.head_dim)
    return {"kv": (torch.zeros(shape, dtype=engine.model.dtype, device=engine.device),
                   torch.zeros(shape, dtype=engine.model.dtype, device=engine.device))}


class TokenTree:
    """One token tree decoded under every prefix of a StreamPrefix on the stream kernels
    (bf16 models), in SEGMENTS: a segment is a set of m sibling-level nodes forwarded
    together, each carrying t tokens, whose parents all lie in one earlier segment (or are
    the prefix itself, t = 1).  A node whose draw hit an end-of-sequence token carries its
    parent's tokens and is not forwarded: it shares its parent's stream (``hidden`` of the
    parent's segment and index).

    ``forward(parent_seg, parents, tokens)`` forwards m new nodes: under each of the P
    prefixes the segment's streams are s = p * m + j (one group of m streams per prefix, ONE
    forward_streams over all P * m), history slots 0 .. t-2 inherited from the parent
    streams, slot t-1 written by the forward.  Every segment's streams are rows of ONE
    row-layout K / V buffer (the segment's rows ``off`` .. off + P m - 1), and a stream reaches
    its inherited slots through its [P m, ldh] slot table (cs_hist_rows_update from the
    parent segment's table; cs_prefix_attention_rows): a node's K / V is written once by the
    forward that made it and never copied.  ``hidden(seg, idx)`` is the final-norm hidden
    predicting each listed node's children under every prefix ([P, len(idx), d]; seg = -1:
    the prefix's last position).

    Restates what the reference does per lookahead node and per (path, agent): re-encode
    the prompt plus the path (src/methods/finite_lookahead.py:297-399, 464-524 through
    src/utils.py:77-198, 201-281) -- here each node is one token of one stream per prefix,
    forwarded once."""

    def __init__(self, engine: "ScoringEngine", sp: StreamPrefix, max_depth: int,
                 pool: Optional[dict] = None):
        """pool: the reusable K / V buffer (kept by the caller across the trees of one
        statement; grown, never shrunk).  Buffers are zero-filled when allocated: the
        attention reads whole 32-slot blocks and weights the unfilled slots by 0, so they
        must hold finite values (a stale earlier tree's K/V are fine, NaN garbage is not)."""
        self.e = engine
        self.sp = sp
        self.P = len(sp.lens)
        self.ldh = _ceil32(max_depth)
        self.segs: List[dict] = []       # {t, m, off, rows, hidden}
        self.pool = {} if pool is None else pool
        self.used = 0                     # buffer rows taken by this tree's segments

    def _reserve(self, S: int) -> int:
        """S more buffer rows for a new segment: their first row.  A full buffer is replaced
        by one twice as large holding the rows already written (their K / V move once; each
        old buffer is released as soon as it is copied, so the grow holds at most one old
        and two new buffers)."""
        c = self.e.model.cfg
        need = self.used + S
        ent = self.pool.get("kv")
        cap = 0 if ent is None else ent[0].shape[1]
        layout = (c.n_kv_heads, self.ldh, c.head_dim)
        if ent is not None and self.used and tuple(ent[0].shape[2:]) != layout:
            # this tree's earlier segments live in the pool: their row tables would point
            # into a buffer of another layout
            raise ValueError("TokenTree: the pool's history layout changed under a tree "
                             "with segments in it")
        if ent is None or tuple(ent[0].shape[2:]) != layout or cap < need:
            new_cap = max(need, 2 * cap, 256)
            shape = (c.n_layers, new_cap, *layout)
            old = list(self.pool.pop("kv", None) or (None, None))
            keep = self.used if old[0] is not None else 0
            ent = None
            bufs = []
            for j in range(2):       # K, then V: each old buffer freed once it is copied
                t = torch.zeros(shape, dtype=self.e.model.dtype, device=self.e.device)
                if keep:
                    t[:, :keep] = old[j][:, :keep]
                old[j] = None
                bufs.append(t)
            self.pool["kv"] = (bufs[0], bufs[1])
        off = self.used
        self.used = need
        return off

    @property
    def k(self) -> torch.Tensor:
        """The K buffer [L, R, Hkv, ldh, D] (a segment's stream s is row off + s)."""
        return self.pool["kv"][0]

    @property
    def v(self) -> torch.Tensor:
        """The V buffer [L, R, Hkv, ldh, D], row-major like K."""
        return self.pool["kv"][1]

    def forward(self, parent_seg: int, parents: Sequence[int], tokens: Sequence[int]) -> int:
        """Forward m new nodes whose parents are nodes ``parents`` of segment parent_seg
        (-1: the prefix); returns the new segment's id."""
        m_ = self.e.model
        dev = self.e.device
        P, m = self.P, len(tokens)
        if m == 0:
            raise ValueError("a tree segment needs at least one node")
        t = 1 if parent_seg < 0 else self.segs[parent_seg]["t"] + 1
        if t > self.ldh:
            raise ValueError("tree deeper than max_depth")
        S = P * m
        off = self._reserve(S)
        hb = torch.full((1,), t - 1, dtype=torch.int32, device=dev)
        rows = torch.empty(S, self.ldh, dtype=torch.int32, device=dev)
        if t > 1:
            prev = self.segs[parent_seg]
            mp_ = prev["m"]
            par = torch.as_tensor(list(parents), dtype=torch.long)
            if par.numel() != m or int(par.min()) < 0 or int(par.max()) >= mp_:
                raise ValueError("parents must index the parent segment's nodes")
            src = (torch.arange(P)[:, None] * mp_ + par[None, :]).reshape(-1).to(dev)
            ops.hist_rows_update(prev["rows"], rows, src, hb, n_rows=self.k.shape[1],
                                 row_base=off)
        else:
            rows.copy_((off + torch.arange(S, dtype=torch.int32, device=dev))[:, None]
                       .expand(S, self.ldh))
        tok = torch.as_tensor(list(tokens), dtype=torch.long).repeat(P).to(dev)
        h = m_.forward_streams(tok, self.sp.fused, list(self.k.unbind(0)), list(self.v.unbind(0)),
                               hb, m, 1, hist_rows=rows, hist_row_base=off)
        self.segs.append({"t": t, "m": m, "off": off, "rows": rows, "hidden": h.view(P, m, -1)})
        return len(self.segs) - 1

    def append_to_prefix(self, seg: int, j: int, which: Optional[Sequence[int]] = None) -> None:
        """Commit node j of a depth-1 segment: every prefix (or those in ``which``) takes that
        node's K / V (its slot 0, in its own row) as its next key
        (engine.append_prefix_tokens)."""
        sg = self.segs[seg]
        if sg["t"] != 1:
            raise ValueError("only a depth-1 node's token extends the prefixes")
        ps = range(self.P) if which is None else which
        self.e.append_prefix_tokens(self.sp, self.k, self.v, [sg["off"] + p * sg["m"] + j for p in ps],
                                    0, sg["hidden"][list(ps), j], which=which, v_rows=True)

    def hidden(self, seg: int, idx: Sequence[int]) -> torch.Tensor:
        """[P, len(idx), d]: the hidden predicting the children of nodes idx of ``seg``."""
        if seg < 0:
            return self.sp.last_hidden[:, None, :].expand(self.P, len(idx), -1)
        ii = torch.as_tensor(list(idx), dtype=torch.long, device=self.e.device)
        return self.segs[seg]["hidden"][:, ii]
