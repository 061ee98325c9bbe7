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
