"""ctypes binding of ``libconsensus_scoring.so`` — the C-ABI declared in
``include/consensus_scoring.h``.

The library is built in-tree by ``build.py`` (``hipcc --offload-arch=gfx950``).
There is no fallback: if the library is missing or fails to load, every op raises
``CSError``.  ``torch`` is imported before the library is opened so that the
library's ``libamdhip64.so.7`` dependency binds to the HIP runtime torch already
loaded (same SONAME) — one runtime, so torch stream handles are valid here.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libconsensus_scoring.so"

# enum values from include/consensus_scoring.h
CS_F32, CS_BF16, CS_F16 = 0, 1, 2
WELFARE_MIN, WELFARE_SUM, WELFARE_SUMLOG, WELFARE_MAX = 0, 1, 2, 3
NONFINITE_SKIP, NONFINITE_REPLACE = 0, 1

EXPORTED = (
    "cs_version", "cs_last_error", "cs_workspace_size", "cs_logsoftmax_gather",
    "cs_segment_reduce", "cs_welfare_reduce", "cs_segmented_topk", "cs_vocab_topk_workspace_size",
    "cs_vocab_topk", "cs_vocab_sample_workspace_size", "cs_vocab_sample",
    "cs_beam_step_workspace_size", "cs_beam_step", "cs_beam_decode_workspace_size",
    "cs_beam_decode_step", "cs_beam_select", "cs_prefix_attention_plan",
    "cs_prefix_attention", "cs_rope_place", "cs_add_rms_norm", "cs_gated_act",
    "cs_gemm_bf16", "cs_gemm_splits",
    "cs_gemm_bf16_packed", "cs_gemm_pack", "cs_rope_place_splitk",
    "cs_add_rms_norm_splitk", "cs_prefix_attention_rows", "cs_rope_place_rows",
    "cs_rope_place_splitk_rows", "cs_hist_rows_update",
)


class CSError(RuntimeError):
    """Raised when the native library is missing or a C-ABI call fails."""


_lib = None


def lib_path() -> str:
    return os.path.join(_HERE, LIB_NAME)


def load():
    """Open the native library once (idempotent)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (binds libamdhip64.so.7 to torch's copy first)

    path = lib_path()
    if not os.path.exists(path):
        raise CSError(
            f"{LIB_NAME} is not built ({path} missing). Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` from the repo root.")
    from . import build as _build
    if _build.built_hash() != _build.source_hash():
        # a library older than its sources would be called with the new signatures
        raise CSError(f"{LIB_NAME} is stale (built from other sources than csrc/ and "
                      "include/ now hold). Rebuild it with "
                      "`python -c 'import __graft_entry__ as g; g.build()'`.")
    try:
        L = ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover - environment dependent
        raise CSError(f"failed to load {path}: {e}") from e
    vp, i64, i32, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    L.cs_version.restype = ctypes.c_char_p
    L.cs_last_error.restype = ctypes.c_char_p
    L.cs_workspace_size.argtypes = [i64, i64, i32]
    L.cs_workspace_size.restype = ctypes.c_size_t
    L.cs_logsoftmax_gather.argtypes = [vp, ctypes.c_int, i64, i64, i64, vp, i32, f32, vp, vp, vp,
                                       ctypes.c_size_t, vp]
    L.cs_logsoftmax_gather.restype = ctypes.c_int
    L.cs_segment_reduce.argtypes = [vp, i64, vp, i64, vp, vp, vp, vp, vp]
    L.cs_segment_reduce.restype = ctypes.c_int
    L.cs_welfare_reduce.argtypes = [vp, i32, i32, i64, ctypes.c_int, f32, ctypes.c_int, f32, f32,
                                    f32, vp, vp]
    L.cs_welfare_reduce.restype = ctypes.c_int
    L.cs_segmented_topk.argtypes = [vp, i32, i32, i64, i32, vp, vp, vp]
    L.cs_segmented_topk.restype = ctypes.c_int
    L.cs_vocab_topk_workspace_size.argtypes = [i64, i64, i32]
    L.cs_vocab_topk_workspace_size.restype = ctypes.c_size_t
    L.cs_vocab_topk.argtypes = [vp, ctypes.c_int, i64, i64, i64, i32, f32, vp, vp, vp,
                                ctypes.c_size_t, vp]
    L.cs_vocab_topk.restype = ctypes.c_int
    L.cs_vocab_sample_workspace_size.argtypes = [i64, i64, i32]
    L.cs_vocab_sample_workspace_size.restype = ctypes.c_size_t
    L.cs_vocab_sample.argtypes = [vp, ctypes.c_int, i64, i64, i64, f32, f32, vp, i32, vp, vp, vp,
                                  ctypes.c_size_t, vp]
    L.cs_vocab_sample.restype = ctypes.c_int
    L.cs_beam_step_workspace_size.argtypes = [i64, i64]
    L.cs_beam_step_workspace_size.restype = ctypes.c_size_t
    L.cs_beam_step.argtypes = [vp, ctypes.c_int, i32, i32, i64, i64, vp, i32, vp, f32, ctypes.c_int,
                               f32, vp, vp, i32, vp, vp, vp, vp, ctypes.c_size_t, vp]
    L.cs_beam_step.restype = ctypes.c_int
    L.cs_beam_decode_workspace_size.argtypes = [i32, i32, i64, i32]
    L.cs_beam_decode_workspace_size.restype = ctypes.c_size_t
    L.cs_beam_decode_step.argtypes = [vp, i64, vp, i64, ctypes.c_int, i32, i32, i64, i32, f32, vp,
                                      ctypes.c_int, f32, vp, vp, vp, i32, vp, vp, vp, vp,
                                      ctypes.c_size_t, vp]
    L.cs_beam_decode_step.restype = ctypes.c_int
    L.cs_beam_select.argtypes = [vp, i32, ctypes.c_int, vp, i32, i32, vp, vp, vp, vp, vp]
    L.cs_beam_select.restype = ctypes.c_int
    L.cs_prefix_attention_plan.argtypes = [vp, i32, vp, i32, i32, i32, i32, i32, i32, i64, vp, i64,
                                           vp, vp, vp]
    L.cs_prefix_attention_plan.restype = i64
    L.cs_prefix_attention.argtypes = [vp, vp, vp, i64, vp, vp, i32, vp, i32, vp, vp, i64, vp, i32,
                                      i32, i32, i32, i32, f32, f32, i32, vp, i32, i32, vp, vp,
                                      ctypes.c_size_t, vp]
    L.cs_prefix_attention.restype = ctypes.c_int
    L.cs_rope_place.argtypes = [vp, i64, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, vp, vp, vp,
                                i64, vp]
    L.cs_rope_place.restype = ctypes.c_int
    L.cs_add_rms_norm.argtypes = [vp, i64, vp, i64, vp, vp, i64, vp, i64, i64, f32, ctypes.c_int,
                                  vp, i64, vp]
    L.cs_add_rms_norm.restype = ctypes.c_int
    L.cs_add_rms_norm_splitk.argtypes = [vp, i64, vp, i32, vp, vp, i64, vp, i64, i64, f32,
                                         ctypes.c_int, vp, i64, vp]
    L.cs_add_rms_norm_splitk.restype = ctypes.c_int
    L.cs_gated_act.argtypes = [vp, i64, vp, i64, i64, i64, ctypes.c_int, vp, i64, vp]
    L.cs_gated_act.restype = ctypes.c_int
    L.cs_gemm_bf16.argtypes = [vp, i64, vp, i64, vp, i64, i64, i64, i64, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_int, vp, vp]
    L.cs_gemm_bf16.restype = ctypes.c_int
    L.cs_gemm_splits.argtypes = [i64, i64, i64, ctypes.c_int, ctypes.c_int]
    L.cs_gemm_splits.restype = i64
    L.cs_gemm_bf16_packed.argtypes = [vp, i64, vp, vp, i64, i64, i64, i64, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]
    L.cs_gemm_bf16_packed.restype = ctypes.c_int
    L.cs_gemm_pack.argtypes = [vp, i64, i64, i64, vp, vp]
    L.cs_gemm_pack.restype = ctypes.c_int
    i32 = ctypes.c_int32
    L.cs_rope_place_splitk.argtypes = [vp, i32, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, vp,
                                       vp, vp, i64, vp]
    L.cs_rope_place_splitk.restype = ctypes.c_int
    L.cs_prefix_attention_rows.argtypes = [vp, vp, vp, i64, vp, vp, i32, vp, i32, vp, vp, vp, i64,
                                           vp, i32, i32, i32, i32, i32, f32, f32, i32, vp, i32, i32,
                                           vp, vp, ctypes.c_size_t, vp]
    L.cs_prefix_attention_rows.restype = ctypes.c_int
    L.cs_rope_place_rows.argtypes = L.cs_rope_place.argtypes
    L.cs_rope_place_rows.restype = ctypes.c_int
    L.cs_rope_place_splitk_rows.argtypes = L.cs_rope_place_splitk.argtypes
    L.cs_rope_place_splitk_rows.restype = ctypes.c_int
    L.cs_hist_rows_update.argtypes = [vp, vp, vp, vp, i64, i32, i64, i64, vp]
    L.cs_hist_rows_update.restype = ctypes.c_int
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().cs_last_error().decode(errors="replace")
        raise CSError(f"{what} failed (status {rc}): {msg}")


def version() -> str:
    return load().cs_version().decode()
