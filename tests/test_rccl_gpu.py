"""The direct RCCL communicator (parallel.RcclComm) on the one GPU of the box: unique-id
exchange over the ProcessGroup, ncclCommInitRank, and an in-place ncclAllReduce(MIN) on
the caller's stream.  With one rank the reduction is the identity, so this pins the
binding (argument types, the 128-byte id, the stream handle), not the xGMI transport;
the multi-rank combine semantics are covered by tests/test_parallel_gloo.py."""
import importlib
import socket

import pytest
import torch

from conftest import PKG_DIR

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_comm_single_rank_all_reduce(pkg):
    import torch.distributed as dist
    par = importlib.import_module(PKG_DIR + ".parallel")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}",
                            world_size=1, rank=0, device_id=dev)
    try:
        comm = par.RcclComm()
        assert (comm.rank, comm.world) == (0, 1)
        x = torch.tensor([3.0, -1.5, float("inf"), -7.25], device=dev)
        ref = x.clone()
        st = torch.cuda.Stream(device=dev)
        st.wait_stream(torch.cuda.current_stream())
        comm.all_reduce(x, comm.MIN, stream=st)
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
        y = torch.arange(10, dtype=torch.int64, device=dev)
        comm.all_reduce(y, comm.SUM)
        torch.cuda.synchronize()
        assert torch.equal(y, torch.arange(10, dtype=torch.int64, device=dev))
        with pytest.raises(ValueError):
            comm.all_reduce(torch.zeros(4, 4, device=dev).t(), comm.MIN)   # not contiguous
        comm.close()
    finally:
        dist.destroy_process_group()


def test_sharded_step_graph_records_the_rccl_exchange(pkg, monkeypatch):
    """with the direct RCCL communicator the sharded fast beam loop
    captures its broadcast + MIN all-reduce INSIDE the step graph (one replay per step,
    decode_path "fused-topk-sharded-graph").  On the box's one GPU: a one-rank nccl group,
    the agents sharded as rank 0 of 2 (as bench.py --emulate-ranks does), the captured loop
    against the uncaptured sharded loop (CS_RCCL_IN_GRAPH=0) and the host loop -- identical
    candidates, min-rewards, kept beams and statements, speculation hits and misses
    included (beam_search.py:439-667 on an agent shard).  The 2-3-rank semantics of the
    exchange itself are pinned by tests/test_methods_sharded_gloo.py; this is unmeasured on
    more than one GPU."""
    import sys
    import os
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import test_lookahead_stream_gpu as tl
    par = importlib.import_module(PKG_DIR + ".parallel")
    R = importlib.import_module(PKG_DIR + ".runtime")
    T = importlib.import_module(PKG_DIR + ".tokenizer")
    methods = importlib.import_module(PKG_DIR + ".methods")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}",
                            world_size=1, rank=0, device_id=dev)
    try:
        monkeypatch.setattr(par, "method_shard",
                            lambda n_agents, config=None: par.AgentShard(n_agents, 0, 2))
        assert par.StepComm(par.AgentShard(4, 0, 2)).capturable
        opinions = {f"Agent {i}": t for i, t in enumerate(
            ["Fund public transit first.", "Lower taxes before anything else.",
             "Protect parks above all.", "Build housing near the center."], 1)}
        issue = "How should the city spend its budget?"
        for family in ("llama3", "gemma2"):
            eng = tl._tiny(family, dev, seed=7)
            tok = T.CharTokenizer(family, vocab_size=eng.model.cfg.vocab)
            R.register_engine("test/rccl-graph", eng, tok)
            cfg = {"beam_width": 3, "max_tokens": 9, "proposer": "topk", "top_k": 6}
            runs = {}
            for name, extra, env in (("graph", {"speculative_force_miss": 2}, "1"),
                                     ("nograph", {"speculative_force_miss": 2}, "0"),
                                     ("host", {"fast_topk": False}, "1")):
                monkeypatch.setenv("CS_RCCL_IN_GRAPH", env)
                g = methods.get_method_generator("beam_search", dict(cfg, **extra),
                                                 "test/rccl-graph")
                runs[name] = (g, g.generate_statement(issue, opinions))
            assert runs["graph"][0].decode_path == "fused-topk-sharded-graph"
            assert runs["nograph"][0].decode_path == "fused-topk-sharded"
            common = ("candidates", "min_rewards", "kept")
            logs = {k: [{c: s_[c] for c in common} for s_ in g.step_log]
                    for k, (g, _) in runs.items()}
            assert logs["graph"] == logs["nograph"] == logs["host"], family
            assert runs["graph"][1] == runs["nograph"][1] == runs["host"][1]
            gg = runs["graph"][0]
            assert gg.spec_hits > 0 and gg.spec_misses > 0, (gg.spec_hits, gg.spec_misses)
            R.clear_engines()
    finally:
        dist.destroy_process_group()
