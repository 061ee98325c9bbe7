"""Drop-in for the utility / welfare entry points of the reference's ``core.py``.

Same names, arguments and return types (NumPy in, NumPy out), but the per-step
log-softmax + gather and the per-leaf folding run on the GPU through the C-ABI
kernels (``ops.logsoftmax_gather`` -> ``ops.segment_reduce``), and the point-mass
welfare / selection through ``ops.welfare`` / ``ops.topk``.

Reference (core.py):
  generate_params      49-56    (host RNG: parameters are inputs, not the hot path)
  enumerate_leaves     59-61
  log_softmax_rows     64-68    -> cs_logsoftmax_gather (k = vocab: full rows)
  compute_utilities    71-100   -> one batched launch over every (agent, leaf, step) row
  F_val                108-113  (general lottery: host; point mass: point_mass_welfare)
  utilitarian argmax   374-376  -> point_mass_select(U, "utilitarian")

The lottery solvers (FW_nash_welfare, egalitarian_lottery) and the coalition LPs
are outside the decode hot path and are not provided here.
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from . import ops


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise ops.CSError("core: the GPU path needs a HIP device (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def generate_params(B, L, d, n_agents, seed=123):
    """Random unit token vectors v[t, a] and agent vectors w[i] (core.py:49-56 contract)."""
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(L, B, d))
    v /= np.linalg.norm(v, axis=2, keepdims=True) + 1e-12
    w = rng.normal(size=(n_agents, d))
    w /= np.linalg.norm(w, axis=1, keepdims=True) + 1e-12
    return v, w


def enumerate_leaves(B, L):
    """All length-L action tuples in lexicographic order (core.py:59-61 contract)."""
    return list(itertools.product(range(B), repeat=L))


def log_softmax_rows(M):
    """Row-wise log-softmax of a 2-D array on the GPU (core.py:64-68 contract)."""
    M = np.asarray(M)
    dev = _device()
    X = torch.as_tensor(np.ascontiguousarray(M, dtype=np.float32), device=dev)
    n, B = X.shape
    tgt = torch.arange(B, dtype=torch.int32, device=dev).repeat(n, 1)
    out, _ = ops.logsoftmax_gather(X, tgt)
    return out.double().cpu().numpy()


def compute_utilities(v, w, rho):
    """Agent-by-leaf utilities U[i, j] (core.py:71-100 contract), returns (U, leaves).

    Every (agent i, leaf j, step t) logits row rho * w_i . (z_t(j) + v[t, b]) is
    built in one batched GEMM, the whole [n * B^L * L, B] block goes through one
    cs_logsoftmax_gather launch (target = a_t), and cs_segment_reduce folds the L
    steps of each (agent, leaf) — the sum of core.py:90.
    """
    v = np.asarray(v, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64)
    L, B, d = v.shape
    n = w.shape[0]
    leaves = enumerate_leaves(B, L)
    m = len(leaves)
    dev = _device()
    A = torch.as_tensor(np.array(leaves, dtype=np.int64), device=dev)          # [m, L]
    vt = torch.as_tensor(v, device=dev)                                         # [L, B, d]
    wt = torch.as_tensor(w, device=dev)                                         # [n, d]
    chosen = vt[torch.arange(L, device=dev)[None, :], A]                        # [m, L, d]
    z = torch.cumsum(chosen, dim=1) - chosen                                    # state before step t
    X = z[:, :, None, :] + vt[None, :, :, :]                                    # [m, L, B, d]
    logits = float(rho) * torch.einsum("id,mtbd->imtb", wt, X)                  # [n, m, L, B]
    logits = logits.reshape(n * m * L, B).to(torch.float32).contiguous()
    tgt = A[None, :, :].expand(n, m, L).reshape(-1, 1).to(torch.int32).contiguous()
    tok, _ = ops.logsoftmax_gather(logits, tgt)
    offs = torch.arange(0, n * m * L + 1, L, dtype=torch.int32, device=dev)
    seg = ops.segment_reduce(tok, offs)
    # fp32 segment sums carry fp64-accumulated values; finish the stabilisation in fp64
    logu = seg["sum_lp"].double().reshape(n, m)
    U = torch.exp(logu - logu.max(dim=1, keepdim=True).values) + 1e-300        # core.py:94-99
    return U.cpu().numpy(), leaves


def F_val(U, p):
    """Nash welfare of a lottery: sum_i log(U_i . p) (core.py:108-113 contract, host)."""
    a = np.asarray(U) @ np.asarray(p)
    if np.any(a <= 0):
        return -np.inf
    return float(np.sum(np.log(a)))


_KIND = {"nash": "sumlog", "utilitarian": "sum", "egalitarian": "min"}


def point_mass_welfare(U, kind="nash", eps=0.0):
    """Welfare of every point-mass lottery e_j, i.e. per column of U [n, m], on the GPU.

    nash        -> sum_i log(U[i, j])   (= F_val(U, e_j), core.py:108-113)
    utilitarian -> sum_i U[i, j]        (core.py:374)
    egalitarian -> min_i U[i, j]
    """
    dev = _device()
    Ut = torch.as_tensor(np.ascontiguousarray(U, dtype=np.float32), device=dev)
    tiny = float(np.finfo(np.float32).tiny) if eps == 0.0 else float(eps)
    return ops.welfare(Ut, _KIND.get(kind, kind), eps=tiny).double().cpu().numpy()


def point_mass_select(U, kind="utilitarian"):
    """argmax_j of the point-mass welfare, first index on ties (np.argmax, core.py:374)."""
    dev = _device()
    Ut = torch.as_tensor(np.ascontiguousarray(U, dtype=np.float32), device=dev)
    W = ops.welfare(Ut, _KIND.get(kind, kind), eps=float(np.finfo(np.float32).tiny))
    idx, _ = ops.topk(W, 1)
    return int(idx.item())
