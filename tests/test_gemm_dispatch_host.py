"""Host logic of the GEMM selection (no GPU): the dispatch table's unpacked / packed entries
as ops.gemm_choice reads them, the per-weight packing gain, and the merge of per-config
tuner outputs (tools/merge_gemm_dispatch.py)."""
import importlib
import types
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"


@pytest.fixture
def ops_table():
    ops = importlib.import_module(PKG + ".ops")
    saved = ops._gemm_table
    table = {
        "48,1024,512,0": {"variant": 3, "splits": 2, "us": 20.0, "torch_us": 25.0,
                          "packed": {"variant": 3, "splits": 4, "us": 15.0}},
        "272,1024,512,0": {"variant": 2, "splits": 1, "us": 30.0, "torch_us": 31.0},
        "48,2048,512,1": {"packed": {"variant": 2, "splits": 1, "us": 40.0}, "torch_us": 50.0},
    }
    ops._gemm_table = table
    yield ops
    ops._gemm_table = saved


def test_gemm_choice_normalises_unpacked_and_packed_entries(ops_table):
    ops = ops_table
    assert ops.gemm_choice(48, 1024, 512) == {"variant": 3, "splits": 2, "packed": False}
    assert ops.gemm_choice(48, 1024, 512, packed=True) == {"variant": 3, "splits": 4, "packed": True}
    assert ops.gemm_choice(272, 1024, 512, packed=True) == {"variant": 2, "splits": 1, "packed": False}
    # a packed-only entry: hipBLASLt without the packed copy, the packed form with it
    assert ops.gemm_choice(48, 2048, 512, True) is None
    assert ops.gemm_choice(48, 2048, 512, True, packed=True)["packed"] is True
    assert ops.gemm_choice(8, 1024, 512) is None


def test_pack_gain_is_the_best_saving_over_row_counts(ops_table):
    ops = ops_table
    assert ops.gemm_pack_gain(1024, 512) == pytest.approx(5.0)       # min(20, 25) - 15
    assert ops.gemm_pack_gain(2048, 512, True) == pytest.approx(10.0)  # torch 50 - 40
    assert ops.gemm_pack_gain(4096, 512) == 0.0
    assert ops.gemm_packs(1024, 512) and not ops.gemm_packs(1024, 512, True)


def test_merge_replaces_the_measured_shapes_only(tmp_path, monkeypatch):
    sys.path.insert(0, REPO)
    merge = importlib.import_module("tools.merge_gemm_dispatch")
    base = {"table": {"1,128,64,0": {"variant": 2, "splits": 1, "us": 1.0},
                      "2,128,64,0": {"variant": 3, "splits": 1, "us": 2.0}},
            "measured": [{"M": 1, "N": 128, "K": 64, "gated": 0, "torch_us": 3.0},
                         {"M": 2, "N": 128, "K": 64, "gated": 0, "torch_us": 4.0}]}
    new = {"table": {"3,128,64,0": {"packed": {"variant": 2, "splits": 1, "us": 0.5}}},
           "measured": [{"M": 2, "N": 128, "K": 64, "gated": 0, "torch_us": 1.0},
                        {"M": 3, "N": 128, "K": 64, "gated": 0, "torch_us": 1.0}],
           "device": "x", "torch": "t", "hip": "h", "library": "l"}
    inst = tmp_path / "installed.json"
    inst.write_text(json.dumps(base))
    f = tmp_path / "new.json"
    f.write_text(json.dumps(new))
    out = tmp_path / "merged.json"
    monkeypatch.setattr(merge, "INSTALLED", str(inst))
    monkeypatch.setattr(sys, "argv", ["merge", str(f), "--out", str(out)])
    assert merge.main() == 0
    m = json.loads(out.read_text())
    # shape 2 was re-measured and lost its cs_gemm entry; 1 kept; 3 added
    assert set(m["table"]) == {"1,128,64,0", "3,128,64,0"}
    assert sorted(r["M"] for r in m["measured"]) == [1, 2, 3]
    assert [r["torch_us"] for r in m["measured"] if r["M"] == 2] == [1.0]


def test_pack_decode_weights_orders_by_gain_per_byte_within_the_budget(monkeypatch):
    """Model.pack_decode_weights keeps packed copies of the weights with a packed gain, the
    most time saved per byte first, while the device keeps its reserve free (host logic:
    the device memory query and the pack launch are stubbed)."""
    import torch
    M = importlib.import_module(PKG + ".model")
    ops = importlib.import_module(PKG + ".ops")
    cfg = M.preset("tiny-llama")
    m = M.Model(cfg, "cpu", dtype=torch.bfloat16)
    m.device = torch.device("cuda", 0)                 # the packing path, with stubs below
    sizes = {n: w.numel() * 2 for n, (w, _) in m.decode_weights().items()}
    # gains (us) by weight kind: gate|up saves the most per byte, then q|k|v; down none
    gains = {"gate_up": 4.0, "qkv": 1.5, "wo": 0.1, "w_down": 0.0, "lm_head": 0.2}

    def gain(N, K, gated=False):
        if gated:
            return gains["gate_up"] * N * K
        for name, (w, g) in m.decode_weights().items():
            if not g and tuple(w.shape) == (N, K):
                return gains[name.split(".")[-1]] * N * K
        return 0.0

    packed = []
    monkeypatch.setattr(ops, "gemm_pack_gain", gain)
    monkeypatch.setattr(ops, "gemm_pack", lambda w: packed.append(tuple(w.shape)) or ("packed", w.shape))
    gu = sum(v for n, v in sizes.items() if n.endswith("gate_up"))
    qkv = sum(v for n, v in sizes.items() if n.endswith("qkv"))
    budget = gu + qkv // 2                             # every gate|up, half the q|k|v
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (budget + (1 << 30), 8 << 30))
    # the packed copies are finished on their stream before they are published (no device here)
    synced = []
    monkeypatch.setattr(torch.cuda, "current_stream",
                        lambda dev=None: types.SimpleNamespace(synchronize=lambda: synced.append(1)))
    used = m.pack_decode_weights(reserve_bytes=1 << 30)
    assert synced, "the packed copies were published without finishing their stream"
    names = set(m.wp)
    assert all(n in names for n in sizes if n.endswith("gate_up"))
    assert not any(n.endswith("w_down") for n in names)          # no gain: never packed
    assert used <= budget and used == sum(sizes[n] for n in names)
    n_qkv = sum(1 for n in names if n.endswith("qkv"))
    assert 0 < n_qkv < cfg.n_layers                     # the budget ran out inside q|k|v
    monkeypatch.setenv("CS_GEMM_PACK", "0")
    assert m.pack_decode_weights() == 0 and m.wp == {}


def test_prune_drops_fused_gated_entries_that_lose_to_plain_plus_act():
    sys.path.insert(0, REPO)
    merge = importlib.import_module("tools.merge_gemm_dispatch")
    table = {"48,256,64,1": {"packed": {"variant": 3, "splits": 1, "us": 50.0}},
             "80,256,64,1": {"variant": 2, "splits": 1, "us": 40.0},
             "48,256,64,0": {"packed": {"variant": 3, "splits": 1, "us": 38.0}}}
    measured = [
        {"M": 48, "N": 256, "K": 64, "gated": 1, "torch_us": 60.0, "cs_gemm": []},
        {"M": 48, "N": 256, "K": 64, "gated": 0, "torch_us": 55.0, "cs_gemm": [{"us": 45.0}],
         "cs_gemm_packed": [{"us": 38.0}]},
        {"M": 80, "N": 256, "K": 64, "gated": 1, "torch_us": 70.0, "cs_gemm": []},
        {"M": 80, "N": 256, "K": 64, "gated": 0, "torch_us": 64.0, "cs_gemm": [{"us": 50.0}]},
    ]
    # 48: plain packed 38 + act (60 - 55) = 43 < fused 50 -> dropped
    # 80: plain 50 + act 6 = 56 > fused 40 -> kept
    assert merge.prune_gated(table, measured) == ["48,256,64,1"]
    assert "80,256,64,1" in table and "48,256,64,0" in table
