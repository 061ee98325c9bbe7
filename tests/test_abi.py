"""CPU tests of the C-ABI boundary: the library loads, exports every symbol the
header declares, and rejects bad arguments with a status + message (no launch)."""
import ctypes
import glob
import os
import re

import pytest

from conftest import REPO


def _declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(cs_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    return syms


def test_header_declares_the_boundary():
    syms = _declared_symbols()
    for s in ("cs_logsoftmax_gather", "cs_segment_reduce", "cs_welfare_reduce",
              "cs_segmented_topk", "cs_workspace_size", "cs_last_error", "cs_version"):
        assert s in syms


def test_library_exports_every_declared_symbol(pkg):
    from importlib import import_module
    lib = import_module(pkg.__name__ + "._lib")
    L = lib.load()
    missing = [s for s in _declared_symbols() if not hasattr(L, s)]
    assert not missing, f"symbols declared in include/*.h but not exported: {missing}"
    assert set(lib.EXPORTED) == _declared_symbols()


def test_library_is_gfx950_code_object(pkg):
    from importlib import import_module
    path = import_module(pkg.__name__ + "._lib").lib_path()
    blob = open(path, "rb").read()
    assert b"gfx950" in blob, "the HIP library must carry a gfx950 code object"


def test_version_and_workspace_size(pkg):
    from importlib import import_module
    L = import_module(pkg.__name__ + "._lib").load()
    assert b"gfx950" in L.cs_version()
    # many rows: single pass, no workspace
    assert L.cs_workspace_size(76800, 128256, 1) == 0
    # few rows: split-V partials, 8 bytes per (row, split)
    ws = L.cs_workspace_size(16, 128256, 10)
    assert ws > 0 and ws % (16 * 8) == 0


@pytest.mark.parametrize("call", ["neg_rows", "bad_dtype", "ld_lt_vocab", "k_without_targets",
                                  "bad_softcap"])
def test_invalid_arguments_return_status(pkg, call):
    from importlib import import_module
    lib = import_module(pkg.__name__ + "._lib")
    L = lib.load()
    dummy = ctypes.c_void_p(16)
    args = dict(logits=dummy, dtype=1, rows=4, vocab=16, ld=16, tgt=dummy, k=1, cap=0.0,
                out=dummy)
    if call == "neg_rows":
        args["rows"] = -1
    elif call == "bad_dtype":
        args["dtype"] = 9
    elif call == "ld_lt_vocab":
        args["ld"] = 8
    elif call == "k_without_targets":
        args["tgt"] = None
    elif call == "bad_softcap":
        args["cap"] = -1.0
    rc = L.cs_logsoftmax_gather(args["logits"], args["dtype"], args["rows"], args["vocab"],
                                args["ld"], args["tgt"], args["k"], args["cap"], args["out"],
                                None, None, 0, None)
    assert rc == -1
    assert L.cs_last_error().decode()


def test_invalid_welfare_and_topk(pkg):
    from importlib import import_module
    L = import_module(pkg.__name__ + "._lib").load()
    d = ctypes.c_void_p(16)
    assert L.cs_welfare_reduce(d, 2, 4, 4, 7, 1e-9, 0, 0.0, 0.0, 0.0, d, None) == -1
    assert L.cs_welfare_reduce(d, 2, 4, 2, 0, 1e-9, 0, 0.0, 0.0, 0.0, d, None) == -1
    assert L.cs_segmented_topk(d, 1, 20000, 20000, 1, d, None, None) == -1
    assert L.cs_segmented_topk(d, 1, 8, 8, 9, d, None, None) == -1
    assert L.cs_segment_reduce(d, -1, d, 1, None, None, None, None, None) == -1


def test_round4_entry_points_validate_before_launching(pkg):
    """The packed-weight GEMM, the thin variants and the split-K RoPE fold reject bad
    arguments with a status code (no device needed: checked before any launch)."""
    from importlib import import_module
    L = import_module(pkg.__name__ + "._lib").load()
    d = ctypes.c_void_p(256)
    odd = ctypes.c_void_p(260)
    # cs_gemm_pack: N % 16, K % 64, alignment
    assert L.cs_gemm_pack(d, 64, 24, 64, d, None) == -1
    assert L.cs_gemm_pack(d, 96, 32, 96, d, None) == -1
    assert L.cs_gemm_pack(odd, 64, 32, 64, d, None) == -1
    # cs_gemm_bf16_packed: ws2 variants only
    assert L.cs_gemm_bf16_packed(d, 64, d, d, 128, 4, 128, 64, 1, 0, 0, 5, None, None) == -1
    assert L.cs_gemm_bf16_packed(d, 64, d, d, 128, 4, 128, 64, 1, 0, 0, 1, None, None) == -1
    # thin variants: at most 80 rows, no K split
    assert L.cs_gemm_bf16(d, 64, d, 64, d, 128, 81, 128, 64, 1, 0, 0, 5, None, None) == -1
    assert L.cs_gemm_bf16(d, 128, d, 128, d, 128, 8, 128, 128, 2, 0, 0, 6, d, None) == -1
    assert L.cs_gemm_bf16(d, 64, d, 64, d, 128, 8, 128, 64, 1, 0, 0, 8, None, None) == -1
    # cs_rope_place_splitk: T < 32, head_dim % 16, partials aligned
    assert L.cs_rope_place_splitk(d, 2, d, d, None, 1, d, 1, 32, 4, 2, 64, d, d, d, 64, None) == -1
    assert L.cs_rope_place_splitk(d, 2, d, d, None, 1, d, 1, 1, 4, 2, 40, d, d, d, 32, None) == -1
    assert L.cs_rope_place_splitk(None, 2, d, d, None, 1, d, 1, 1, 4, 2, 64, d, d, d, 32, None) == -1
    assert L.cs_last_error().decode()


def test_missing_library_raises(pkg, monkeypatch, tmp_path):
    from importlib import import_module
    lib = import_module(pkg.__name__ + "._lib")
    monkeypatch.setattr(lib, "_lib", None)
    monkeypatch.setattr(lib, "_HERE", str(tmp_path))
    with pytest.raises(lib.CSError):
        lib.load()


def test_ops_refuse_cpu_tensors(ops):
    import torch
    x = torch.zeros(4, 16)
    t = torch.zeros(4, 1, dtype=torch.int32)
    with pytest.raises(ops.CSError):
        ops.logsoftmax_gather(x, t)


def _plan(L, lens, gmap, n_str, T, H, Hkv, D, ldh):
    import numpy as np
    lens = np.asarray(lens, dtype=np.int32)
    gp = None if gmap is None else np.asarray(gmap, dtype=np.int32)
    n_groups = len(lens) if gmap is None else len(gmap)
    na, nm, ws = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_size_t()
    args = (lens.ctypes.data, lens.size, None if gp is None else gp.ctypes.data, n_groups, n_str,
            T, H, Hkv, D, ldh)
    total = L.cs_prefix_attention_plan(*args, None, 0, ctypes.byref(na), ctypes.byref(nm),
                                       ctypes.byref(ws))
    if total <= 0:
        return total, None, 0, 0, 0
    out = np.zeros((total, 4), dtype=np.int32)
    assert L.cs_prefix_attention_plan(*args, out.ctypes.data, total, ctypes.byref(na),
                                      ctypes.byref(nm), ctypes.byref(ws)) == total
    return total, out, na.value, nm.value, ws.value


@pytest.mark.parametrize("shape", [
    # lens, group map, n_str, T, H, Hkv, D, ldh
    ([5500] + [210] * 64, None, 8, 1, 64, 8, 128, 32),      # C5 decode: one long reference prompt
    ([1700] + [210] * 16, None, 16, 1, 16, 8, 256, 32),     # C3 decode
    ([600] + [210] * 4, None, 4, 1, 32, 8, 64, 64),         # C1 decode
    ([3000, 700], [1, 0, 1], 4, 1, 32, 8, 64, 96),          # group -> prefix map
    ([0], [0, 0], 1, 300, 32, 8, 128, 320),                 # prompts as streams: no prefix
    ([4100] + [250] * 32, None, 64, 1, 32, 8, 128, 32),     # C4 tree level 3: >= 1024 cells,
                                                            # the reference cells 16x longer
])
def test_prefix_attention_plan_covers_every_cell(pkg, shape):
    """cs_prefix_attention_plan (host): every (group, head, query group) cell is covered by
    exactly n_used attention entries with splits 0 .. n_used-1; split cells own distinct
    partial slots inside the workspace and are merged row chunk by row chunk."""
    from importlib import import_module
    L = import_module(pkg.__name__ + "._lib").load()
    lens, gmap, n_str, T, H, Hkv, D, ldh = shape
    total, plan, na, nm, ws = _plan(L, lens, gmap, n_str, T, H, Hkv, D, ldh)
    n_groups = len(lens) if gmap is None else len(gmap)
    M = n_str * T * (H // Hkv)
    n_qg = -(-M // 64)
    if plan is None:                      # enough cells without splits
        assert total == 0 and n_groups * Hkv * n_qg >= 1024 or total == 0
        assert lens[0] <= 4 * max(lens[-1], 1) or T > 1, "imbalanced cells need a plan"
        return
    assert total == na + nm and nm > 0
    att, mer = plan[:na], plan[na:]
    cells = {}
    slots = set()
    for pg, qg, z, slot in att.tolist():
        sp, nu = z & 255, z >> 8
        assert 0 <= pg < n_groups * Hkv and 0 <= qg < n_qg and 1 <= nu <= 32 and sp < nu
        cells.setdefault((pg, qg), set()).add((sp, nu))
        if nu > 1:
            assert slot not in slots
            slots.add(slot)
    assert len(cells) == n_groups * Hkv * n_qg
    for key, ss in cells.items():
        nu = next(iter(ss))[1]
        assert ss == {(s, nu) for s in range(nu)}, key
    assert ws == len(slots) * 64 * (D + 2) * 4
    merged = {}
    for pg, qg, slot0, z in mer.tolist():
        ch, nu = z & 255, z >> 8
        assert nu > 1 and 0 <= slot0 and slot0 + nu <= len(slots)
        merged.setdefault((pg, qg), []).append(ch)
    for key, ss in cells.items():
        nu = next(iter(ss))[1]
        if nu > 1:
            rows = min(64, M - key[1] * 64)
            assert sorted(merged[key]) == list(range(-(-rows // 8))), key
        else:
            assert key not in merged
    # the long reference prompt's cells split further than the agents' short ones
    if gmap is None and lens[0] > 4 * lens[-1]:
        nu_of = {pg // Hkv: z >> 8 for pg, qg, z, _ in att.tolist()}
        assert nu_of[0] > nu_of[len(lens) - 1]


def test_prefix_attention_plan_rejects_bad_arguments(pkg):
    from importlib import import_module
    L = import_module(pkg.__name__ + "._lib").load()
    assert _plan(L, [100, 100], [0, 5], 4, 1, 32, 8, 128, 32)[0] == -1     # prefix index range
    assert _plan(L, [100], None, 4, 1, 30, 8, 128, 32)[0] == -1            # H % Hkv
    assert _plan(L, [100], None, 4, 1, 32, 8, 96, 32)[0] == -1             # head_dim
    assert _plan(L, [100], None, 4, 1, 32, 8, 128, 40)[0] == -1            # ld_hist % 32


def test_handoff_primitives_lower_to_sc1(pkg, tmp_path):
    """The beam kernels' cross-workgroup hand-offs (cs_kernels.cuh st_sc1 / ld_sc1 / arrive)
    are relaxed agent-scope atomics whose ORDERING rests on their gfx950 lowering: the
    store and the load must be sc1 (write-through past / read past the per-XCD L2) and
    the arrival counter a device atomic.  Compile a probe with the library's own flags
    and check the disassembly, so a toolchain that lowers them otherwise fails here."""
    import shutil
    import subprocess
    from importlib import import_module
    build = import_module(pkg.__name__ + ".build")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = tmp_path / "probe.hip"
    src.write_text('#include "cs_kernels.cuh"\n'
                   '__global__ void probe(uint32_t* data, uint32_t* cnt, uint32_t* out) {\n'
                   '  st_sc1(data + threadIdx.x, threadIdx.x);\n'
                   '  wait_stores();\n'
                   '  __syncthreads();\n'
                   '  if (threadIdx.x == 0 && arrive(cnt) == gridDim.x - 1)\n'
                   '    st_sc1(out + blockIdx.x, ld_sc1(data + 7));\n'
                   '}\n')
    asm = tmp_path / "probe.s"
    flags = [f for f in build._flags() if f != "-fPIC"]
    subprocess.run([hipcc] + flags + ["--cuda-device-only", "-S", str(src), "-o", str(asm)],
                   check=True, capture_output=True)
    text = asm.read_text()
    body = text[text.index("probe"):]
    stores = [l for l in body.splitlines() if l.strip().startswith("global_store_dword")]
    loads = [l for l in body.splitlines() if l.strip().startswith("global_load_dword")]
    atomics = [l for l in body.splitlines() if l.strip().startswith("global_atomic_add")]
    assert stores and all("sc1" in l for l in stores), stores
    assert loads and all("sc1" in l for l in loads), loads
    assert atomics, "the arrival counter must be one device atomic"
    assert "s_waitcnt vmcnt(0)" in body
    shutil.rmtree(tmp_path, ignore_errors=True)


def _hipcc_or_skip():
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    return hipcc


def test_gemm_fragment_reads_are_hand_counted(pkg, tmp_path):
    """cs_gemm_bf16's 2-waves-per-SIMD kernels at 17 row tiles (C3's 272 rows, C5's 2 x 272)
    keep their LDS fragment reads in flight with counted waits (inline-asm ds_read_b128 +
    s_waitcnt lgkmcnt(5), csrc/gemm.hip) and do not spill: the compiler's own schedule drains
    every read with lgkmcnt(0) before its use (decode-step GEMMs)."""
    import re
    import subprocess
    from importlib import import_module
    build = import_module(pkg.__name__ + ".build")
    hipcc = _hipcc_or_skip()
    asm = tmp_path / "gemm.s"
    flags = [f for f in build._flags() if f != "-fPIC"]
    gemm = [s for s in build.SOURCES if s.endswith("gemm.hip")][0]
    subprocess.run([hipcc] + flags + ["--cuda-device-only", "-S", gemm, "-o", str(asm)],
                   check=True, capture_output=True)
    text = asm.read_text()
    names = re.findall(r"^(_Z\w*ws2_gemm_kernelILi17E\w+):", text, re.M)
    assert names, "no 17-row-tile instantiation"
    for n in names:
        i = text.index(n + ":")
        body = text[i:text.index(".Lfunc_end", i)]
        meta = text[text.index(".Lfunc_end", i):]
        assert "lgkmcnt(5)" in body, n
        assert re.search(r"ScratchSize: (\d+)", meta).group(1) == "0", n
