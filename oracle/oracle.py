"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker (or the timed CPU baseline).
The product path never imports it: the package's ops fail loudly when the HIP
library is missing instead of falling back here.

Two layers:

* ``libcs_oracle.so`` (``cs_oracle.c``) — fp64 C restatement of the reference's
  scoring arithmetic (core.py:64-68 log-softmax + gather, best_of_n.py:303-305 /
  finite_lookahead.py:520 / evaluation.py:203-213 folds, evaluation.py:337-381
  welfare, beam_search.py:558-560 stable ordering).  OpenMP row-parallel.
* small NumPy restatements used to cross-check the C layer on tiny inputs.

Pinning: the C layer is checked against golden vectors produced by the
reference itself (``tests/golden/``, made by ``tests/golden/make_golden.py``
importing ``/root/reference`` in the build container) and against the
reference's committed ``results/`` CSVs (welfare identities).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libcs_oracle.so")
_lib = None

F32, BF16, F16 = 0, 1, 2
MIN, SUM, SUMLOG, MAX = 0, 1, 2, 3

_dbl_p = ctypes.POINTER(ctypes.c_double)
_i32_p = ctypes.POINTER(ctypes.c_int32)


def build() -> str:
    """Compile libcs_oracle.so in place (gcc + OpenMP)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_logsoftmax_gather.argtypes = [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
            _i32_p, ctypes.c_int32, ctypes.c_double, _dbl_p, _dbl_p]
        L.oracle_logsoftmax_gather.restype = None
        L.oracle_segment_reduce.argtypes = [_dbl_p, _i32_p, ctypes.c_int64, _dbl_p, _dbl_p,
                                            _i32_p, _dbl_p]
        L.oracle_segment_reduce.restype = None
        L.oracle_welfare.argtypes = [_dbl_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                     ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, _dbl_p]
        L.oracle_welfare.restype = None
        L.oracle_topk.argtypes = [_dbl_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                  ctypes.c_int32, _i32_p]
        L.oracle_topk.restype = None
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_num_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def dtype_code(arr: np.ndarray, bf16: bool = False) -> int:
    if bf16:
        assert arr.dtype == np.uint16, "bf16 logits are passed as their uint16 bit patterns"
        return BF16
    if arr.dtype == np.float32:
        return F32
    if arr.dtype == np.float16:
        return F16
    raise TypeError(f"unsupported logits dtype {arr.dtype}")


def logsoftmax_gather(logits: np.ndarray, targets: np.ndarray, softcap: float = 0.0,
                      bf16: bool = False, vocab: int | None = None):
    """fp64 (tok_lp[rows, k], lse[rows]) for a 2-D logits array (row stride = shape[1])."""
    assert logits.ndim == 2 and logits.flags.c_contiguous
    rows, ld = logits.shape
    vocab = ld if vocab is None else vocab
    targets = np.ascontiguousarray(targets, dtype=np.int32).reshape(rows, -1)
    k = targets.shape[1]
    tok = np.empty((rows, k), dtype=np.float64)
    lse = np.empty(rows, dtype=np.float64)
    lib().oracle_logsoftmax_gather(logits.ctypes.data, dtype_code(logits, bf16), rows, vocab, ld,
                                   _p(targets, _i32_p), k, float(softcap), _p(tok, _dbl_p),
                                   _p(lse, _dbl_p))
    return tok, lse


def segment_reduce(tok_lp: np.ndarray, offsets: np.ndarray):
    tok = np.ascontiguousarray(tok_lp, dtype=np.float64).reshape(-1)
    off = np.ascontiguousarray(offsets, dtype=np.int32)
    n = off.shape[0] - 1
    out = {k: np.empty(n, dtype=np.float64) for k in ("sum_lp", "sum_p", "last")}
    cnt = np.empty(n, dtype=np.int32)
    lib().oracle_segment_reduce(_p(tok, _dbl_p), _p(off, _i32_p), n, _p(out["sum_lp"], _dbl_p),
                                _p(out["sum_p"], _dbl_p), _p(cnt, _i32_p), _p(out["last"], _dbl_p))
    out["count"] = cnt
    return out


def welfare(U: np.ndarray, kind: int, eps: float = 1e-9, nonfinite: int = 0,
            nan_val: float = -10.0, posinf_val: float = 20.0, neginf_val: float = -20.0):
    U = np.ascontiguousarray(U, dtype=np.float64)
    A, C = U.shape
    W = np.empty(C, dtype=np.float64)
    lib().oracle_welfare(_p(U, _dbl_p), A, C, C, kind, eps, nonfinite, nan_val, posinf_val,
                         neginf_val, _p(W, _dbl_p))
    return W


def topk(W: np.ndarray, k: int):
    W = np.ascontiguousarray(np.atleast_2d(W), dtype=np.float64)
    n_seg, seg_len = W.shape
    idx = np.empty((n_seg, k), dtype=np.int32)
    lib().oracle_topk(_p(W, _dbl_p), n_seg, seg_len, seg_len, k, _p(idx, _i32_p))
    return idx


def set_threads(n: int) -> int:
    lib().oracle_set_num_threads(int(n))
    return lib().oracle_num_threads()


# --- NumPy restatements for tiny cross-checks -------------------------------------
def log_softmax_rows_np(M: np.ndarray) -> np.ndarray:
    """Row-wise log-softmax, the formula of core.py:64-68 (max-shifted, fp64)."""
    M = np.asarray(M, dtype=np.float64)
    shifted = M - M.max(axis=1, keepdims=True)
    return shifted - np.log(np.exp(shifted).sum(axis=1, keepdims=True))


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16 bit patterns (uint16), NaN kept NaN."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(x)
    r[nan] = 0x7FC0
    return r


def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


# --- candidate proposer (restates the product's counter-based RNG bit for bit) -----
_M64 = (1 << 64) - 1


def cs_uniform(seed: int, v: np.ndarray) -> np.ndarray:
    """u(seed, v) in (0, 1): splitmix64 finaliser of (seed, v), top 23 bits + 0.5 over 2^23.
    Exactly the device function cs_uniform in csrc/proposer.hip."""
    with np.errstate(over="ignore"):
        x = (np.uint64(seed & _M64) * np.uint64(0x9E3779B97F4A7C15)
             + (np.asarray(v, dtype=np.uint64) + np.uint64(1)) * np.uint64(0xD1B54A32D192ED03))
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return ((x >> np.uint64(41)).astype(np.float32) + np.float32(0.5)) * np.float32(2.0 ** -23)


def gumbel_sample(logits_row: np.ndarray, seed: int, temperature: float = 1.0):
    """argmax_v x[v]/T + g(seed, v), first index on ties; returns (id, log-prob of id)."""
    x = np.asarray(logits_row, dtype=np.float64) / temperature
    u = cs_uniform(seed, np.arange(x.shape[0])).astype(np.float64)
    s = x - np.log(-np.log(u))
    i = int(np.argmax(s))
    mx = x.max()
    lse = mx + np.log(np.exp(x - mx).sum())
    return i, float(x[i] - lse)


def vocab_topk(logits: np.ndarray, k: int):
    """Top-k ids per row ordered by (value desc, id asc) -> (ids, values)."""
    x = np.asarray(logits, dtype=np.float64)
    ids = topk(x, k)
    return ids, np.take_along_axis(x, ids, 1)
