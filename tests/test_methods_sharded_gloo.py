"""Agent-sharded methods on CPU (gloo, 2 and 3 ranks): beam search, Best-of-N, finite
lookahead and MCTS split the agents over the ranks (parallel.method_shard), combine the welfare
across them, and must still replay the reference's own traces — the same statements,
BoN candidates, rewards and welfare as one process — on every rank.  The kernels are
emulated by the oracle (tests/cpu_emulation.py); the collectives are real
torch.distributed.  3 ranks over the fixture's agents leave ragged shards."""
import os
import socket

import pytest
import torch.multiprocessing as mp

METHODS = ("beam_search", "best_of_n", "finite_lookahead", "mcts")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, gpu=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here, os.path.join(os.path.dirname(here), "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import cpu_emulation
    import method_parity as mpar
    torch.set_num_threads(2)
    if gpu:   # the real HIP library on the box's one GPU, every rank on cuda:0
        torch.cuda.set_device(0)
    else:
        cpu_emulation.install()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    traces = mpar.load_traces("method_traces.json")
    traces = dict(traces, runs=[r for r in traces["runs"] if r["method"] in METHODS])
    mpar.register_fixture_engine(traces, torch.device("cuda:0" if gpu else "cpu"))
    import importlib
    par = importlib.import_module(cpu_emulation.PKG + ".parallel")
    A = len(traces["agent_opinions"])
    shard = par.method_shard(A)
    assert shard.world == world and len(shard.local) < A   # the agents really are split
    failures = mpar.check_methods(traces)
    stmts = [stmt for _run, _gen, stmt in mpar.run_methods(dict(traces, runs=traces["runs"][:2]))]
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, failures, stmts, len(traces["runs"])))


def _run(world, gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, gpu)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, failures, stmts, n_runs = q.get(timeout=600)
        res[rank] = (failures, stmts, n_runs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, (failures, stmts, n_runs) in res.items():
        assert n_runs > 0
        assert not failures, f"rank {rank}:\n" + "\n".join(failures)
        assert stmts == res[0][1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_methods_replay_reference_traces(world):
    _run(world, gpu=False)


@pytest.mark.gpu
def test_sharded_methods_on_gpu_gloo_rehearsal():
    """The same replay through the real HIP library: 2 ranks on the one GPU of the box,
    gloo collectives on device tensors (RCCL needs one GPU per rank)."""
    _run(2, gpu=True)
