"""Minimal Llama-3 / Gemma-2 decoder forward with an explicit KV layout.

PyTorch here is plumbing: it runs the transformer GEMMs (hipBLASLt) and attention
(SDPA).  What the scoring path needs from it is narrow and is shaped for reuse:

  * ``prefill(ids)``       one pass over a batch of prompt prefixes -> per-layer K/V
                           [n_prefix, Hkv, P, D] and the final-norm hidden state of
                           every position (the last one predicts the first
                           continuation token).
  * ``extend(...)``        T new tokens for each of R streams; stream r attends to
                           prefix ``owner[r]`` (shared, never copied per candidate
                           in HBM beyond the transient SDPA operand), to its own
                           generated history (beam search) and causally to itself.
  * ``lm_head(h)``         hidden -> logits in the weight dtype (bf16); the
                           log-softmax / gather / welfare after it are the HIP kernels.

The Gemma-2 final-logit soft-cap (30) is NOT applied here: cs_logsoftmax_gather
applies it on load (one fewer HBM pass over the logits).

Weights are random-init (seeded, architecture-exact shapes): no checkpoints are
available offline and throughput is independent of weight values.
"""
from __future__ import annotations

import math
import os
import threading
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F


@dataclass
class ModelConfig:
    name: str
    family: str            # "llama3" | "gemma2"
    vocab: int
    d_model: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    d_ff: int
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    tie_embeddings: bool = False
    rope_scaling: Optional[dict] = None      # llama3-style frequency scaling
    final_softcap: float = 0.0               # gemma2: 30.0 (applied in the HIP kernel)
    attn_softcap: float = 0.0                # gemma2: 50.0
    sliding_window: int = 0                  # gemma2: 4096 on even layers
    query_pre_attn_scalar: Optional[float] = None
    init_std: float = 0.02
    extra: Dict = field(default_factory=dict)


LLAMA31_ROPE = {"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                "original_max_position_embeddings": 8192}
LLAMA32_ROPE = {"factor": 32.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                "original_max_position_embeddings": 8192}

PRESETS = {
    "llama-3.2-1b": ModelConfig("llama-3.2-1b", "llama3", 128256, 2048, 16, 32, 8, 64, 8192,
                                tie_embeddings=True, rope_scaling=LLAMA32_ROPE),
    "llama-3.1-8b": ModelConfig("llama-3.1-8b", "llama3", 128256, 4096, 32, 32, 8, 128, 14336,
                                rope_scaling=LLAMA31_ROPE),
    "llama-3.3-70b": ModelConfig("llama-3.3-70b", "llama3", 128256, 8192, 80, 64, 8, 128, 28672,
                                 rope_scaling=LLAMA31_ROPE),
    "gemma-2-9b": ModelConfig("gemma-2-9b", "gemma2", 256000, 3584, 42, 16, 8, 256, 14336,
                              rope_theta=10000.0, rms_eps=1e-6, tie_embeddings=True,
                              final_softcap=30.0, attn_softcap=50.0, sliding_window=4096,
                              query_pre_attn_scalar=256.0),
    # small architecture-faithful models for parity fixtures
    "tiny-llama": ModelConfig("tiny-llama", "llama3", 384, 64, 2, 4, 2, 16, 128,
                              rope_scaling=LLAMA31_ROPE, init_std=0.15),
    "tiny-gemma": ModelConfig("tiny-gemma", "gemma2", 384, 64, 2, 4, 2, 16, 128,
                              rope_theta=10000.0, rms_eps=1e-6, tie_embeddings=True,
                              final_softcap=30.0, attn_softcap=50.0, sliding_window=8,
                              query_pre_attn_scalar=16.0, init_std=0.15),
}


def preset(name: str, **overrides) -> ModelConfig:
    return replace(PRESETS[name], **overrides)


def rope_inv_freq(cfg: ModelConfig, device) -> torch.Tensor:
    D = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, D, 2, dtype=torch.float64, device=device) / D))
    rs = cfg.rope_scaling
    if rs:
        factor, lo, hi = rs["factor"], rs["low_freq_factor"], rs["high_freq_factor"]
        old = rs["original_max_position_embeddings"]
        wavelen = 2 * math.pi / inv
        scaled = torch.where(wavelen > old / lo, inv / factor, inv)
        smooth = (old / wavelen - lo) / (hi - lo)
        smoothed = (1 - smooth) * scaled / factor + smooth * scaled
        medium = (wavelen >= old / hi) & (wavelen <= old / lo)
        inv = torch.where(medium, smoothed, scaled)
    return inv.to(torch.float32)


# where a K-split projection's partials are folded in the stream forward: q|k|v inside
# cs_rope_place_splitk (CS_FOLD_IN_ROPE=0: in cs_gemm_bf16's own launch); the output
# projection inside the residual add's cs_add_rms_norm (CS_FOLD_IN_NORM=0: in its own
# launch).  Round 4 measured the norm fold 0.4 ms slower at C5 (profiles/r04s_fold_ab.jsonl);
# since round 5 it loads only its splits' partials, and round 6 measured it faster or equal
# on every decode step: per-rank C3 5.76 -> 5.67 ms (with the per-rank output projection on
# the packed K-split GEMM), per-rank C5 27.10 -> 26.94, one-GPU C5 76.4 -> 76.0, C1 / one-GPU
# C3 within noise (profiles/r06v_fold_ab/)
_FOLD_IN_ROPE = os.environ.get("CS_FOLD_IN_ROPE", "1") != "0"
_PACK_LOCK = threading.Lock()
_FOLD_IN_NORM = os.environ.get("CS_FOLD_IN_NORM", "1") != "0"
# models without branch norms (Llama): an output or down projection that runs on hipBLASLt
# (the scoring chunks, prompt prefill, C4's largest tree segments) adds into the residual in
# hipBLASLt's epilogue (ops.linear_into_residual), and the residual add's launch only
# normalises; the cs_gemm shapes keep their K-split fold in the residual add
_RESID_IN_GEMM = os.environ.get("CS_RESID_IN_GEMM", "1") != "0"


class Model:
    """Decoder weights + forward.  ``dtype`` is the weight/activation dtype."""

    # fp32 scores the soft-capped eager attention materialises at once (_attend_grouped)
    softcap_chunk_scores = 1 << 27

    def __init__(self, cfg: ModelConfig, device, dtype=torch.bfloat16, seed: int = 0,
                 weights: Optional[Dict[str, torch.Tensor]] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.w = weights if weights is not None else self._init(seed)
        self.inv_freq = rope_inv_freq(cfg, self.device)
        self._fuse()
        # cs_gemm_pack'ed copies of the decode-step weights the dispatch table runs packed
        # (pack_decode_weights; None until the first stream forward)
        self.wp: Optional[Dict[str, object]] = None

    def _fuse(self) -> None:
        """Per layer one [q; k; v] and one [gate; up] weight, so each is ONE GEMM; the
        separate weights in ``w`` become views of them (nothing is stored twice)."""
        c = self.cfg
        self.wf: Dict[str, torch.Tensor] = {}
        for i in range(c.n_layers):
            p = f"l{i}."
            for fused, parts in (("qkv", ("wq", "wk", "wv")), ("gate_up", ("w_gate", "w_up"))):
                full = torch.cat([self.w[p + n] for n in parts])
                sizes = [self.w[p + n].shape[0] for n in parts]
                for n, view in zip(parts, full.split(sizes)):
                    self.w[p + n] = view
                self.wf[p + fused] = full

    # --- weights ----------------------------------------------------------------
    def shapes(self) -> Dict[str, tuple]:
        c = self.cfg
        s = {"embed": (c.vocab, c.d_model), "norm": (c.d_model,)}
        if not c.tie_embeddings:
            s["lm_head"] = (c.vocab, c.d_model)
        for i in range(c.n_layers):
            p = f"l{i}."
            s[p + "attn_norm"] = (c.d_model,)
            s[p + "wq"] = (c.n_heads * c.head_dim, c.d_model)
            s[p + "wk"] = (c.n_kv_heads * c.head_dim, c.d_model)
            s[p + "wv"] = (c.n_kv_heads * c.head_dim, c.d_model)
            s[p + "wo"] = (c.d_model, c.n_heads * c.head_dim)
            s[p + "mlp_norm"] = (c.d_model,)
            s[p + "w_gate"] = (c.d_ff, c.d_model)
            s[p + "w_up"] = (c.d_ff, c.d_model)
            s[p + "w_down"] = (c.d_model, c.d_ff)
            if c.family == "gemma2":
                s[p + "post_attn_norm"] = (c.d_model,)
                s[p + "post_mlp_norm"] = (c.d_model,)
        return s

    def _init(self, seed: int) -> Dict[str, torch.Tensor]:
        c = self.cfg
        gen_dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        g = torch.Generator(device=gen_dev).manual_seed(seed)
        w = {}
        for name, shp in self.shapes().items():
            if "norm" in name:
                # llama: weight ~ 1; gemma: (1 + weight) with weight ~ 0
                base = 0.0 if c.family == "gemma2" else 1.0
                t = base + 0.1 * torch.randn(shp, generator=g, device=gen_dev)
            elif name == "embed":
                t = torch.randn(shp, generator=g, device=gen_dev) * (1.0 if c.family == "llama3" else
                                                                    1.0 / math.sqrt(c.d_model))
            else:
                t = torch.randn(shp, generator=g, device=gen_dev) * c.init_std
            w[name] = t.to(self.device, self.dtype)
        return w

    def num_params(self) -> int:
        return sum(t.numel() for t in self.w.values())

    # --- building blocks --------------------------------------------------------
    def _rms(self, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        if c.family != "gemma2":
            # one fused launch (fp32 statistics, one rounding to x.dtype) instead of the
            # 7-kernel chain: 54 vs 439 us on [16384, 4096] bf16 (profiles/r01l_rms_ab.jsonl)
            return F.rms_norm(x, (x.shape[-1],), w.to(x.dtype), c.rms_eps)
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + c.rms_eps)
        return (y * (1.0 + w.float())).to(x.dtype)

    def _rope_tables(self, pos: torch.Tensor, dtype) -> tuple:
        """(cos, signed sin) [B, 1, T, D] of positions pos [B, T]: [cos, cos] and
        [-sin, sin]; computed once per forward and shared by every layer's q and k."""
        ang = pos.to(torch.float32)[:, None, :, None] * self.inv_freq[None, None, None, :]
        c, s = ang.cos(), ang.sin()
        return torch.cat([c, c], dim=-1).to(dtype), torch.cat([-s, s], dim=-1).to(dtype)

    def _rope(self, x: torch.Tensor, pos: torch.Tensor, tables: Optional[tuple] = None) -> torch.Tensor:
        """x [B, H, T, D], pos [B, T] (half-rotation convention):
        x * cos + [-x2, x1] * sin, with [x2, x1] = roll(x, D/2) and the sign in the table
        (3 launches instead of 5)."""
        cos, ssin = tables if tables is not None else self._rope_tables(pos, x.dtype)
        return torch.addcmul(x * cos, x.roll(x.shape[-1] // 2, dims=-1), ssin)

    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        h = self.w["embed"][ids]
        if self.cfg.family == "gemma2":
            # the normalizer in the activation dtype, made once (no host copy inside a
            # captured decode step)
            sc = getattr(self, "_emb_scale", None)
            if sc is None or sc.dtype != h.dtype:
                sc = self._emb_scale = torch.tensor(self.cfg.d_model ** 0.5, dtype=h.dtype,
                                                    device=h.device)
            h = h * sc
        return h

    def _mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        p = f"l{i}."
        if x.numel() // x.shape[-1] <= 4096:
            # few tokens (decode / prefill): one launch for both
            g, u = (x @ self.wf[p + "gate_up"].t()).split(self.cfg.d_ff, dim=-1)
        else:
            # score chunks: two GEMMs keep g and u contiguous, so SiLU·up runs vectorised
            # (3.0 vs 3.1 ms at 16k tokens of the 8B MLP; profiles/r01l_fuse_ab.jsonl)
            g = x @ self.w[p + "w_gate"].t()
            u = x @ self.w[p + "w_up"].t()
        act = F.gelu(g, approximate="tanh") if self.cfg.family == "gemma2" else F.silu(g)
        return (act * u) @ self.w[p + "w_down"].t()

    def _attend(self, i: int, q, k, v, mask, q_pos, k_pos):
        """q [B,H,T,D]; k,v [B,Hkv,S,D]; mask [B,1,rep*T,S] bool (True = attend; row r*T+t
        is query t, see _prepare).  The rep query heads that share a K/V head ride along the
        query axis ([B,Hkv,rep*T,D]), so K/V are attended in place, never repeated."""
        c = self.cfg
        B, D = q.shape[0], q.shape[-1]
        rep = c.n_heads // c.n_kv_heads
        if rep > 1 and q.shape[1] == c.n_heads:       # [B,H,T,D] -> grouped (else already)
            q = q.reshape(B, c.n_kv_heads, rep * q.shape[2], D)
        T = q.shape[2] // rep
        H = c.n_heads
        if rep > 1:
            q_pos = q_pos.repeat(1, rep)
        if c.sliding_window and i % 2 == 0:
            # q - k < W  <=>  k > q - W on integer positions: the comparison broadcasts
            # straight to bool, never materialising an int64 [B, 1, rep*T, S] difference
            mask = mask & (k_pos[:, None, None, :] > (q_pos - c.sliding_window)[:, None, :, None])
        return self._attend_grouped(q, k, v, mask).reshape(B, H, T, D)

    def _attend_grouped(self, q, k, v, mask):
        c = self.cfg
        scale = (c.query_pre_attn_scalar ** -0.5) if c.query_pre_attn_scalar else c.head_dim ** -0.5
        if c.attn_softcap > 0:
            # the soft-capped scores are materialised in fp32: in query-row chunks of at most
            # softcap_chunk_scores of them, so a batched prefill of long prompts stays
            # bounded (each row's softmax is independent of the others)
            B, G, R, _ = q.shape
            rows = max(1, self.softcap_chunk_scores // max(1, B * G * k.shape[2]))
            if rows >= R or mask.shape[2] != R:
                return self._softcap_attend(q, k, v, mask, scale)
            return torch.cat([self._softcap_attend(q[:, :, r:r + rows], k, v,
                                                   mask[:, :, r:r + rows], scale)
                              for r in range(0, R, rows)], dim=2)
        return F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=scale)

    def _softcap_attend(self, q, k, v, mask, scale):
        cap = self.cfg.attn_softcap
        s = (q.float() @ k.float().transpose(-1, -2)) * scale
        s = cap * torch.tanh(s / cap)
        s = s.masked_fill(~mask, float("-inf"))
        p = torch.softmax(s, dim=-1).to(v.dtype)
        return p @ v

    def _layer(self, i, h, pos, ctx_k, ctx_v, ctx_mask, ctx_pos, self_mask=None, pre=None):
        """One decoder layer over new tokens h [B,T,d] at positions pos [B,T].

        ctx_k/ctx_v [B,Hkv,S,D] is the earlier context (prefix + history), visible
        where ctx_mask [B,S] is True.  The new tokens see each other causally, or through
        self_mask [T,T] (True = attend; e.g. a token tree: ancestors and self).
        ``pre`` = _prepare(...) of this forward (rope tables, mask, key positions), shared
        by the layers.  Returns (h, k_new, v_new)."""
        c = self.cfg
        p = f"l{i}."
        B, T, _ = h.shape
        if pre is None:
            pre = self._prepare(pos, h.dtype, ctx_mask if ctx_k is not None else None, ctx_pos,
                                self_mask)
        tables, tables_q, m, kp = pre
        rep = c.n_heads // c.n_kv_heads
        x = self._rms(h, self.w[p + "attn_norm"])
        kvd = c.n_kv_heads * c.head_dim
        q, k, v = (x @ self.wf[p + "qkv"].t()).split([c.n_heads * c.head_dim, kvd, kvd], dim=-1)
        # q straight into the grouped layout [B, Hkv, rep*T, D] (one copy), so RoPE runs on
        # contiguous rows with the grouped tables and _attend needs no further reshape
        q = q.view(B, T, c.n_heads, c.head_dim).transpose(1, 2).reshape(
            B, c.n_kv_heads, rep * T, c.head_dim)
        k = k.view(B, T, c.n_kv_heads, c.head_dim).transpose(1, 2)
        # own storage: the cached V must not keep the whole q/k/v GEMM output alive
        v = v.contiguous().view(B, T, c.n_kv_heads, c.head_dim).transpose(1, 2)
        q = self._rope(q, pos, tables_q)
        k = self._rope(k, pos, tables)
        if ctx_k is not None and ctx_k.shape[2] == ctx_mask.shape[1] + T:
            # the caller left T free key slots after the context: write the new keys there
            # instead of concatenating (one copy of the context per layer saved)
            S = ctx_mask.shape[1]
            ctx_k[:, :, S:] = k
            ctx_v[:, :, S:] = v
            K, V = ctx_k, ctx_v
        elif ctx_k is not None:
            K = torch.cat([ctx_k, k], dim=2)
            V = torch.cat([ctx_v, v], dim=2)
        else:
            K, V = k, v
        o = self._attend(i, q, K, V, m, pos, kp)
        o = o.transpose(1, 2).reshape(B, T, c.n_heads * c.head_dim) @ self.w[p + "wo"].t()
        if c.family == "gemma2":
            o = self._rms(o, self.w[p + "post_attn_norm"])
        h = h + o
        x = self._rms(h, self.w[p + "mlp_norm"])
        y = self._mlp(i, x)
        if c.family == "gemma2":
            y = self._rms(y, self.w[p + "post_mlp_norm"])
        return h + y, k, v

    def _prepare(self, pos, dtype, ctx_mask=None, ctx_pos=None, self_mask=None):
        """Per-forward inputs every layer shares: rope tables, the attention mask
        [B, 1, T, S+T] (context where ctx_mask, the new tokens causally or by self_mask)
        and the key positions."""
        B, T = pos.shape
        causal = (torch.ones(T, T, dtype=torch.bool, device=pos.device).tril()
                  if self_mask is None else self_mask)
        if ctx_mask is not None:
            S = ctx_mask.shape[1]
            m = torch.cat([ctx_mask[:, None, :].expand(B, T, S), causal[None].expand(B, T, T)], -1)
            kp = torch.cat([ctx_pos, pos], dim=1)
        else:
            m, kp = causal[None].expand(B, T, T), pos
        m = m[:, None]
        rep = self.cfg.n_heads // self.cfg.n_kv_heads
        tables = self._rope_tables(pos, dtype)
        tables_q = tables
        if rep > 1:                       # rows r*T + t: query t of group member r (_attend)
            m = m.repeat(1, 1, rep, 1)
            tables_q = tuple(t.repeat(1, 1, rep, 1) for t in tables)
        return tables, tables_q, m, kp

    # --- public forward ----------------------------------------------------------
    @torch.no_grad()
    def prefill(self, ids: torch.Tensor, lengths: torch.Tensor):
        """ids [B, P] right-padded, lengths [B].  Returns (kv list of (k, v) per layer,
        final-norm hidden [B, P, d])."""
        B, P = ids.shape
        pos = torch.arange(P, device=ids.device)[None].expand(B, P)
        valid = pos < lengths[:, None]
        h = self._embed(ids)
        kv = []
        pre = self._prepare(pos, h.dtype)
        for i in range(self.cfg.n_layers):
            # padding keys sit after every valid key, so the causal mask already hides them
            h, k, v = self._layer(i, h, pos, None, None, None, None, pre=pre)
            kv.append((k, v))
        h = self._rms(h, self.w["norm"])
        return kv, h, valid

    @torch.no_grad()
    def extend(self, tokens: torch.Tensor, pos: torch.Tensor, ctx_kv, ctx_mask: torch.Tensor,
               ctx_pos: torch.Tensor, self_mask: torch.Tensor = None):
        """tokens [R, T], pos [R, T]; ctx_kv per layer (k, v) [R, Hkv, S, D] with
        ctx_mask [R, S] (or [R, Hkv, S + T, D] buffers whose last T slots are free: the new
        keys are written there, the buffers are modified); self_mask [T, T] (optional,
        default causal).  Returns
        (final-norm hidden [R, T, d], new kv per layer)."""
        h = self._embed(tokens)
        new = []
        pre = self._prepare(pos, h.dtype, ctx_mask if ctx_kv is not None else None, ctx_pos,
                            self_mask)
        for i in range(self.cfg.n_layers):
            ck, cv = ctx_kv[i] if ctx_kv is not None else (None, None)
            h, k, v = self._layer(i, h, pos, ck, cv, ctx_mask, ctx_pos, self_mask, pre=pre)
            new.append((k, v))
        return self._rms(h, self.w["norm"]), new

    def lm_head(self, h: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        W = self.w["embed"] if self.cfg.tie_embeddings else self.w["lm_head"]
        if h.is_cuda and h.dim() == 2 and h.dtype == W.dtype == torch.bfloat16:
            from . import ops   # local: model.py stays importable without the library
            pw = (self.wp or {}).get("lm_head")
            if ops.gemm_choice(h.shape[0], W.shape[0], W.shape[1], packed=pw is not None) is not None:
                return ops.linear(h, W, out=out, packed=pw)
        if out is not None:
            return torch.matmul(h.to(W.dtype), W.t(), out=out)
        return h.to(W.dtype) @ W.t()

    # --- packed decode weights ----------------------------------------------------
    def decode_weights(self) -> Dict[str, tuple]:
        """name -> (weight, gated) of every GEMM weight a stream forward runs."""
        out = {"lm_head": (self.w["embed"] if self.cfg.tie_embeddings else self.w["lm_head"], False)}
        for i in range(self.cfg.n_layers):
            p = f"l{i}."
            out[p + "qkv"] = (self.wf[p + "qkv"], False)
            out[p + "wo"] = (self.w[p + "wo"], False)
            out[p + "gate_up"] = (self.wf[p + "gate_up"], True)
            out[p + "w_down"] = (self.w[p + "w_down"], False)
        return out

    @torch.no_grad()
    def pack_decode_weights(self, reserve_bytes: Optional[int] = None) -> int:
        """Keep a cs_gemm_pack'ed copy (ops.gemm_pack: fragment-major, every weight load one
        contiguous 1 KB) of each decode weight the dispatch table runs packed at some row
        count, while the device keeps ``reserve_bytes`` free (default 16 GB: the first stream
        forward runs after its prefix caches and K/V histories exist, and the reserve leaves
        room for a second decode state of the same shape, e.g. the re-tokenized text path's,
        plus activations, logits and graph pools -- measured enough at C5, the largest state:
        a 70B replica with 64 agents and its text path, profiles/r05ab_bench_res16.jsonl;
        the former 48 GB left the 70B down projection unpacked).  The weights whose
        packed form saves the most time per byte (ops.gemm_pack_gain) go first, so a partial
        budget (a 70B replica) packs where it pays most.  CS_GEMM_PACK=0 turns packing off;
        CS_GEMM_PACK_RESERVE_GB sets the reserve.
        The copies are snapshots: code that changes a weight in place after the first stream
        forward must call this again (or set ``wp = None``).  Returns the bytes packed."""
        from . import ops
        if (os.environ.get("CS_GEMM_PACK", "1") == "0" or self.device.type != "cuda"
                or self.dtype != torch.bfloat16):
            self.wp = {}
            return 0
        free, total = torch.cuda.mem_get_info(self.device)
        if reserve_bytes is None:
            gb = os.environ.get("CS_GEMM_PACK_RESERVE_GB")
            reserve_bytes = int(float(gb) * (1 << 30)) if gb else 16 << 30
        budget = free - reserve_bytes
        cands = []
        for name, (w, gated) in self.decode_weights().items():
            if w.shape[0] % 16 or w.shape[1] % 64:
                continue
            # a gate|up weight runs packed fused (gated key) or as the plain packed GEMM +
            # cs_gated_act (plain key), whichever the table kept
            gain = ops.gemm_pack_gain(w.shape[0], w.shape[1], gated)
            if gated:
                gain = max(gain, ops.gemm_pack_gain(w.shape[0], w.shape[1], False))
            if gain > 0.0:
                cands.append((gain / (w.numel() * w.element_size()), name, w))
        cands.sort(key=lambda c: -c[0])
        used = 0
        wp = {}
        for _, name, w in cands:
            nbytes = w.numel() * w.element_size()
            if nbytes <= budget - used:
                wp[name] = ops.gemm_pack(w)
                used += nbytes
        # the copies are written on this thread's stream: finish them before publishing, so a
        # forward or capture on another stream never reads a copy the GPU is still writing
        if wp:
            torch.cuda.current_stream(self.device).synchronize()
        self.wp = wp          # published whole: a concurrent forward sees all or nothing
        return used

    # --- stream forward over shared prefixes (HIP attention) ----------------------
    def attn_scale(self) -> float:
        c = self.cfg
        return (c.query_pre_attn_scalar ** -0.5) if c.query_pre_attn_scalar else c.head_dim ** -0.5

    def fused_ok(self, max_ctx: int = 0) -> bool:
        """Whether forward_streams (cs_rope_place + cs_prefix_attention) serves this model:
        bf16 weights on a HIP device, head_dim in {64, 128, 256} (Gemma-2's sliding window
        and attention soft-cap are applied in the kernel).  ``max_ctx`` is kept for callers
        that size contexts; every length is served."""
        c = self.cfg
        return (self.device.type == "cuda" and self.dtype == torch.bfloat16
                and c.head_dim in (64, 128, 256) and c.n_heads % c.n_kv_heads == 0
                and c.n_heads // c.n_kv_heads <= 64)

    @torch.no_grad()
    def forward_streams(self, tokens: torch.Tensor, pfx, hist_k: List[torch.Tensor],
                        hist_vt: List[torch.Tensor], hist_base: torch.Tensor, n_str: int, T: int,
                        group_prefix: Optional[torch.Tensor] = None,
                        group_prefix_host: Optional[Sequence[int]] = None,
                        hist_rows: Optional[torch.Tensor] = None,
                        hist_row_base: int = 0) -> torch.Tensor:
        """T new tokens for each of S = n_groups * n_str streams (tokens [S*T], stream-major):
        stream s = i * n_str + b attends to its group's prefix (pfx: engine.FusedPrefix, the
        ragged layouts of include/consensus_scoring.h cs_prefix_attention; group i uses
        prefix group_prefix[i] or i) and to its own history slots [0, hist_base + t] in
        hist_k[layer] [S, Hkv, ldh, D] / hist_vt[layer] [S, Hkv, D, ldh]; the new tokens'
        K / V are written to slots hist_base + t.  Per layer: one fused q|k|v GEMM,
        cs_rope_place, cs_prefix_attention, output GEMM, MLP.  No host synchronisation and
        no shape depends on hist_base: a decode step is graph-capturable.  Returns the
        final-norm hidden [S*T, d].  pfx.lens_host (+ group_prefix_host) size the key splits
        of the attention work plan.  hist_rows [S, ldh] int32: a row-layout history
        (hist_vt[layer] is V [S, Hkv, ldh, D] like K; slot j of stream s in row hist_rows[s, j]:
        cs_prefix_attention_rows / cs_rope_place_rows); the buffers may hold more rows than
        the S streams (a token tree's levels), the streams' own rows then start at
        hist_row_base."""
        from . import ops   # local: model.py stays importable without the library
        c = self.cfg
        H, Hkv, D = c.n_heads, c.n_kv_heads, c.head_dim
        n_tok = tokens.shape[0]
        scale = self.attn_scale()
        g2 = c.family == "gemma2"
        act = "gelu_tanh" if g2 else "silu"
        eps = c.rms_eps
        if self.wp is None and not torch.cuda.is_current_stream_capturing():
            # once per model; a concurrent first forward waits here, so every forward (and
            # every graph captured after its thread's first eager forward) uses the same copies
            with _PACK_LOCK:
                if self.wp is None:
                    self.pack_decode_weights()
        wp = self.wp or {}
        h = self._embed(tokens).contiguous()                 # the residual stream [n_tok, d]
        # every residual add + RMSNorm is one cs_add_rms_norm launch; h is updated in place
        x = ops.add_rms_norm(h, self.w["l0.attn_norm"], eps, plus_one=g2)
        for i in range(c.n_layers):
            p = f"l{i}."
            # a K-split q|k|v (decode steps, T < 32) hands its partials to cs_rope_place, a
            # K-split output projection to the residual add: no fold launches
            qkv = ops.linear(x, self.wf[p + "qkv"], packed=wp.get(p + "qkv"),
                             fold=T >= 32 or c.head_dim % 16 != 0 or not _FOLD_IN_ROPE)
            q = torch.empty(n_tok, H, D, dtype=h.dtype, device=h.device)
            kpl, vpl = hist_k[i], hist_vt[i]
            if hist_rows is not None and (hist_row_base or kpl.shape[0] != n_tok // T):
                kpl = kpl[hist_row_base:hist_row_base + n_tok // T]
                vpl = vpl[hist_row_base:hist_row_base + n_tok // T]
            ops.rope_place(qkv, self.inv_freq, pfx.lengths, hist_base, n_str, T, H, Hkv, D, q,
                           kpl, vpl, group_prefix=group_prefix, v_rows=hist_rows is not None)
            o = ops.prefix_attention(q, pfx.k[i], pfx.vt[i], pfx.off, pfx.lengths, pfx.max_len,
                                     hist_k[i], hist_vt[i], hist_base, n_str, T, scale=scale,
                                     softcap=c.attn_softcap,
                                     window=c.sliding_window if i % 2 == 0 else 0,
                                     group_prefix=group_prefix,
                                     prefix_len_host=getattr(pfx, "lens_host", None),
                                     group_prefix_host=group_prefix_host, hist_rows=hist_rows)
            resid = not g2 and _RESID_IN_GEMM
            if resid and ops.linear_into_residual(o.view(n_tok, H * D), self.w[p + "wo"], h,
                                                  packed=wp.get(p + "wo")):
                x = ops.add_rms_norm(h, self.w[p + "mlp_norm"], eps)
            else:
                o = ops.linear(o.view(n_tok, H * D), self.w[p + "wo"], packed=wp.get(p + "wo"),
                               fold=not _FOLD_IN_NORM)
                # Gemma-2's post-attention / post-MLP norms of the branch ride in the residual
                # add's launch (b_weight): one cs_add_rms_norm per residual add
                x = ops.add_rms_norm(h, self.w[p + "mlp_norm"], eps, b=o, s_out=h, plus_one=g2,
                                     b_weight=self.w[p + "post_attn_norm"] if g2 else None)
            act_x = ops.linear(x, self.wf[p + "gate_up"], gated=True, act=act,
                               packed=wp.get(p + "gate_up"))
            nxt = self.w[f"l{i + 1}.attn_norm"] if i + 1 < c.n_layers else self.w["norm"]
            if resid and ops.linear_into_residual(act_x, self.w[p + "w_down"], h,
                                                  packed=wp.get(p + "w_down")):
                x = ops.add_rms_norm(h, nxt, eps)
            else:
                # a K-split down projection hands its partials to the residual add's launch
                y = ops.linear(act_x, self.w[p + "w_down"], fold=False, packed=wp.get(p + "w_down"))
                x = ops.add_rms_norm(h, nxt, eps, b=y, s_out=h, plus_one=g2,
                                     b_weight=self.w[p + "post_mlp_norm"] if g2 else None)
        return x


def hf_state_dict(model: Model) -> Dict[str, torch.Tensor]:
    """Map weights to Hugging Face Llama/Gemma2 names (for the independent CPU oracle)."""
    c = model.cfg
    w = model.w
    sd = {"model.embed_tokens.weight": w["embed"], "model.norm.weight": w["norm"]}
    sd["lm_head.weight"] = w["embed"] if c.tie_embeddings else w["lm_head"]
    for i in range(c.n_layers):
        p, q = f"l{i}.", f"model.layers.{i}."
        sd[q + "self_attn.q_proj.weight"] = w[p + "wq"]
        sd[q + "self_attn.k_proj.weight"] = w[p + "wk"]
        sd[q + "self_attn.v_proj.weight"] = w[p + "wv"]
        sd[q + "self_attn.o_proj.weight"] = w[p + "wo"]
        sd[q + "mlp.gate_proj.weight"] = w[p + "w_gate"]
        sd[q + "mlp.up_proj.weight"] = w[p + "w_up"]
        sd[q + "mlp.down_proj.weight"] = w[p + "w_down"]
        sd[q + "input_layernorm.weight"] = w[p + "attn_norm"]
        if c.family == "gemma2":
            sd[q + "post_attention_layernorm.weight"] = w[p + "post_attn_norm"]
            sd[q + "pre_feedforward_layernorm.weight"] = w[p + "mlp_norm"]
            sd[q + "post_feedforward_layernorm.weight"] = w[p + "post_mlp_norm"]
        else:
            sd[q + "post_attention_layernorm.weight"] = w[p + "mlp_norm"]
    return sd
