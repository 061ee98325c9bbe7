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
