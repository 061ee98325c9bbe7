"""Multi-rank agent sharding on CPU (gloo, world size 2): the welfare combination of
parallel.combine_welfare equals the single-process fold over all agents, for every
welfare kind, with ragged shards and non-finite utilities.  The kernels are emulated
by the oracle (tests/cpu_emulation.py); the collectives are real torch.distributed."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, A, C, q):
    import importlib
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here, os.path.join(os.path.dirname(here), "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import cpu_emulation
    cpu_emulation.install()
    par = importlib.import_module(cpu_emulation.PKG + ".parallel")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rng = np.random.default_rng(0)
    U = rng.uniform(-6, -0.1, size=(A, C)).astype(np.float32)
    U[1, 3] = np.nan
    U[:, 5] = np.nan          # no usable utility anywhere
    U[0, 7] = -np.inf
    shard = par.AgentShard(A, rank, world)
    local = torch.as_tensor(U[shard.local])
    out = {}
    for kind in ("min", "max", "sum", "sumlog"):
        for nf in ("skip", "replace"):
            W = par.combine_welfare(local, kind, shard, eps=1e-9, nonfinite=nf)
            out[(kind, nf)] = W.numpy().copy()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("A", [5, 8])
def test_sharded_welfare_equals_single_rank(A, orc):
    world, C = 2, 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, A, C, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(0)
    U = rng.uniform(-6, -0.1, size=(A, C)).astype(np.float32)
    U[1, 3] = np.nan
    U[:, 5] = np.nan
    U[0, 7] = -np.inf
    codes = {"min": orc.MIN, "max": orc.MAX, "sum": orc.SUM, "sumlog": orc.SUMLOG}
    for (kind, nf), W0 in res[0].items():
        ref = orc.welfare(U.astype(np.float64), codes[kind], eps=1e-9,
                          nonfinite=0 if nf == "skip" else 1).astype(np.float32)
        for r in range(world):
            W = res[r][(kind, nf)]
            assert np.array_equal(np.isnan(W), np.isnan(ref)), (kind, nf, W, ref)
            m = ~np.isnan(ref)
            np.testing.assert_array_equal(W[m], ref[m])  # bit-identical to one rank
        np.testing.assert_array_equal(res[0][(kind, nf)], res[1][(kind, nf)])


def test_agent_shard_layout():
    import importlib
    import cpu_emulation  # noqa: F401  (path setup)
    par = importlib.import_module(cpu_emulation.PKG + ".parallel")
    s0, s1 = par.AgentShard(5, 0, 2), par.AgentShard(5, 1, 2)
    assert s0.local == [0, 2, 4] and s1.local == [1, 3]
    assert s0.global_order() == [0, 3, 1, 4, 2]


def _agree_worker(rank, world, port, case, q):
    import importlib
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here, os.path.join(os.path.dirname(here), "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import cpu_emulation
    cpu_emulation.install()
    par = importlib.import_module(cpu_emulation.PKG + ".parallel")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    replayed = []

    def capture():
        if case == "capture_fails_on_rank1" and rank == 1:
            raise RuntimeError("capture refused")

        def replay_ok():
            replayed.append(rank)
            return not (case == "replay_wrong_on_rank0" and rank == 0)
        return replay_ok

    verdict = par.agree_capture(capture, torch.device("cpu"))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, verdict, replayed))


@pytest.mark.parametrize("case", ["all_capture", "capture_fails_on_rank1",
                                  "replay_wrong_on_rank0"])
def test_capture_probe_agrees_over_ranks(case):
    """parallel.agree_capture (the RCCL-in-graph probe's protocol): a rank whose capture is
    refused makes EVERY rank skip the replay (a replayed collective would wait for it
    forever) and take the uncaptured path; one rank's wrong replay turns every rank's
    verdict off; all ranks agree in every case."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, case, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (v, rep) for r, v, rep in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    verdicts = {v for v, _ in res.values()}
    assert len(verdicts) == 1
    if case == "all_capture":
        assert verdicts == {True} and all(rep == [r] for r, (_, rep) in res.items())
    elif case == "capture_fails_on_rank1":
        assert verdicts == {False} and all(rep == [] for _, rep in res.values())
    else:
        assert verdicts == {False} and all(rep == [r] for r, (_, rep) in res.items())
