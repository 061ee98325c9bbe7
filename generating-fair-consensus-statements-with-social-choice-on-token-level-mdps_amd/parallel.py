"""Agent sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Scorings are independent per (agent, candidate); agents share nothing but the
per-candidate welfare reduction.  Each rank owns a subset of the
agents (round-robin by agent index), holds their prefix K/V and a full model
replica, scores its agents x ALL candidates, and then:

  egalitarian (MIN) / MAX   local cs_welfare_reduce over its agents, then one
                            all_reduce(MIN|MAX) of C floats — order-free, so the
                            result is bit-identical to the single-GPU fold;
  utilitarian / Nash        all_gather of the local [A_local, C] utilities, then every
                            rank folds ALL agents in the global agent order with
                            cs_welfare_reduce — bit-identical to 1 GPU (a float SUM
                            all-reduce would depend on the ring order).

Every rank then runs the same deterministic selection (cs_segmented_topk), so no
second exchange is needed.  Messages are C (or A x C) floats: latency-bound, far
below a link's bandwidth.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from . import ops


class AgentShard:
    """Round-robin ownership: agent a belongs to rank a % world."""

    def __init__(self, n_agents: int, rank: int = 0, world: int = 1):
        self.n_agents, self.rank, self.world = n_agents, rank, world
        self.local: List[int] = [a for a in range(n_agents) if a % world == rank]

    def owner(self, a: int) -> int:
        return a % self.world

    def max_local(self) -> int:
        return (self.n_agents + self.world - 1) // self.world

    def global_order(self) -> List[int]:
        """Position of each gathered row (rank-major, padded to max_local) in agent order."""
        m = self.max_local()
        pos = []
        for a in range(self.n_agents):
            r = a % self.world
            pos.append(r * m + a // self.world)
        return pos


def method_shard(n_agents: int, config: Optional[dict] = None) -> AgentShard:
    """The agent shard of this process for one generate_statement call.

    Launched one process per GPU (torchrun) with the default process group initialized
    over more than one rank, the methods split the agents round-robin over the ranks:
    each rank prefills and scores only its agents (their prefix K/V live on its GPU) and
    the per-candidate welfare is combined with combine_welfare; every rank reaches the
    same statement.  config ``shard_agents: false`` keeps every agent on every rank."""
    cfg = config or {}
    if (cfg.get("shard_agents", True) and dist.is_available() and dist.is_initialized()
            and dist.get_world_size() > 1):
        return AgentShard(n_agents, dist.get_rank(), dist.get_world_size())
    return AgentShard(n_agents, 0, 1)


def same_on_all_ranks(obj, shard: AgentShard, group: Optional[dist.ProcessGroup] = None):
    """Rank 0's value of ``obj`` on every rank (candidate sets drawn with seed=None, or any
    host decision that must not diverge between ranks); identity on one rank."""
    if shard.world == 1:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=0, group=group)
    return box[0]


def broadcast_from_rank0(t: torch.Tensor, shard: AgentShard,
                         group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Rank 0's tensor on every rank, in place (e.g. the token ids rank 0 drew for a
    lookahead level: the replicated reference-policy rows of different ranks are computed
    in GEMMs of different shapes, so their bf16 roundings -- and draws -- may differ)."""
    if shard.world > 1:
        dist.broadcast(t, src=0, group=group)
    return t


def any_rank(flags: torch.Tensor, shard: AgentShard,
             group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Element-wise OR of a bool tensor over the ranks (all_reduce MAX); identity on one rank."""
    if shard.world == 1:
        return flags
    t = flags.to(torch.float32)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t > 0


def gather_agents(U_local: torch.Tensor, shard: AgentShard,
                  group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Every agent's rows [A, C] in agent order on every rank, from each rank's
    [A_local, C] (all_gather of rank-major padded blocks, then the global order)."""
    if shard.world == 1:
        return U_local
    C = U_local.shape[1]
    m = shard.max_local()
    pad = torch.full((m, C), float("nan"), dtype=U_local.dtype, device=U_local.device)
    pad[:U_local.shape[0]] = U_local
    bufs = [torch.empty_like(pad) for _ in range(shard.world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat(bufs, 0)[torch.as_tensor(shard.global_order(), device=U_local.device)]


def combine_welfare(U_local: torch.Tensor, kind: str, shard: AgentShard,
                    group: Optional[dist.ProcessGroup] = None, eps: float = 1e-9,
                    nonfinite: str = "skip", nan_val: float = -10.0, posinf_val: float = 20.0,
                    neginf_val: float = -20.0) -> torch.Tensor:
    """Welfare over ALL agents from each rank's [A_local, C] utilities (every rank gets W [C])."""
    kind = {"egalitarian": "min", "utilitarian": "sum", "nash": "sumlog"}.get(kind, kind)
    kw = dict(eps=eps, nonfinite=nonfinite, nan_val=nan_val, posinf_val=posinf_val,
              neginf_val=neginf_val)
    if shard.world == 1:
        return ops.welfare(U_local.contiguous(), kind, **kw)
    C = U_local.shape[1]
    if kind in ("min", "max"):
        if U_local.shape[0] > 0:
            W = ops.welfare(U_local.contiguous(), kind, **kw)
            # a column with no usable utility on this rank must not win the reduction
            fill = float("inf") if kind == "min" else float("-inf")
            W = torch.where(torch.isnan(W), torch.full_like(W, fill), W)
        else:
            W = torch.full((C,), float("inf") if kind == "min" else float("-inf"),
                           dtype=torch.float32, device=U_local.device)
        dist.all_reduce(W, op=dist.ReduceOp.MIN if kind == "min" else dist.ReduceOp.MAX,
                        group=group)
        return torch.where(torch.isinf(W) & (W > 0 if kind == "min" else W < 0),
                           torch.full_like(W, float("nan")), W)
    # sum / sumlog: gather every agent's utilities, fold in global agent order
    allU = gather_agents(U_local.to(torch.float32), shard, group)
    return ops.welfare(allU.contiguous(), kind, **kw)


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]   # ncclUniqueId (rccl.h, 128 bytes)


class RcclComm:
    """A direct RCCL communicator over the ranks of ``group`` (ctypes over the librccl.so
    torch ships, so it is the same RCCL the ProcessGroup uses).

    For collectives issued once per decode step: one ``ncclAllReduce`` on the caller's HIP
    stream costs a few microseconds of host time, against tens for the ProcessGroup call's
    work / event bookkeeping — with a ~40 us GPU step the latter makes the sharded step
    host-bound.  The unique id travels over ``group`` (broadcast_object_list); every rank
    must construct the communicator in the same order.  Raises on any RCCL error.
    """

    MIN, MAX, SUM = 3, 2, 0                  # ncclRedOp_t
    _DTYPES = {torch.float32: 7, torch.float64: 8, torch.int32: 2, torch.int64: 4}

    def __init__(self, group: Optional[dist.ProcessGroup] = None):
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "librccl.so"
        L = ctypes.CDLL(path)
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId,
                                       ctypes.c_int]
        L.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.ncclBroadcast.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        L.ncclGetErrorString.argtypes = [ctypes.c_int]
        self._L = L
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        uid = _UniqueId()
        if self.rank == 0:
            self._check(L.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        box = [bytes(uid) if self.rank == 0 else None]   # all 128 bytes (.internal stops at NUL)
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group else 0,
                                   group=group)
        uid = _UniqueId.from_buffer_copy(box[0])
        self._comm = ctypes.c_void_p()
        self._check(L.ncclCommInitRank(ctypes.byref(self._comm), self.world, uid, self.rank),
                    "ncclCommInitRank")

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: {self._L.ncclGetErrorString(rc).decode()}")

    def all_reduce(self, t: torch.Tensor, op: int, stream: Optional[torch.cuda.Stream] = None):
        """In-place all-reduce of the contiguous device tensor ``t`` on ``stream``
        (default: the current stream), stream-ordered like a kernel launch."""
        if not t.is_contiguous() or t.dtype not in self._DTYPES:
            raise ValueError("RcclComm.all_reduce: need a contiguous f32/f64/i32/i64 tensor")
        st = (stream or torch.cuda.current_stream(t.device)).cuda_stream
        self._check(self._L.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(),
                                          self._DTYPES[t.dtype], op, self._comm, st),
                    "ncclAllReduce")

    def broadcast(self, t: torch.Tensor, root: int = 0, stream: Optional[torch.cuda.Stream] = None):
        """In-place broadcast of the contiguous device tensor ``t`` from ``root``."""
        if not t.is_contiguous() or t.dtype not in self._DTYPES:
            raise ValueError("RcclComm.broadcast: need a contiguous f32/f64/i32/i64 tensor")
        st = (stream or torch.cuda.current_stream(t.device)).cuda_stream
        self._check(self._L.ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(),
                                          self._DTYPES[t.dtype], root, self._comm, st),
                    "ncclBroadcast")

    def close(self):
        if self._comm:
            self._L.ncclCommDestroy(self._comm)
            self._comm = ctypes.c_void_p()


class StepComm:
    """The two per-step exchanges of an agent-sharded decode loop, on the current stream:
    ``min_(W)`` (all-reduce MIN of the per-candidate welfare) and ``bcast0(ids)`` (rank 0's
    proposals).  Over RCCL (the default process group's backend is nccl) they go through
    one process-wide direct communicator (RcclComm: a few us of host time per call; built
    once, CS_DIRECT_RCCL=0 disables), otherwise through the ProcessGroup (gloo rehearsals).

    ``capturable``: the direct communicator's collectives can be recorded in a hipGraph, so
    a sharded decode step (forward, LM head, proposer, broadcast, scoring, MIN all-reduce,
    selection) is ONE graph replay.  Decided once per communicator by a probe -- a captured
    broadcast + all-reduce replayed and checked on every rank, the verdict agreed over the
    process group (every rank takes the same path) -- and CS_RCCL_IN_GRAPH=0 turns it off."""

    _direct: Optional[RcclComm] = None
    _capturable: Optional[bool] = None

    def __init__(self, shard: AgentShard):
        self.shard = shard
        self.comm = None
        if (shard.world > 1 and dist.get_backend() == "nccl"
                and os.environ.get("CS_DIRECT_RCCL", "1") != "0"):
            if StepComm._direct is None or StepComm._direct.world != dist.get_world_size():
                StepComm._direct = RcclComm()
                StepComm._capturable = None
            self.comm = StepComm._direct

    @property
    def capturable(self) -> bool:
        if self.comm is None or os.environ.get("CS_RCCL_IN_GRAPH", "1") == "0":
            return False
        if StepComm._capturable is None:
            StepComm._capturable = _probe_capture(self.comm)
        return StepComm._capturable

    def min_(self, t: torch.Tensor) -> None:
        if self.shard.world == 1:
            return
        if self.comm is not None:
            self.comm.all_reduce(t, RcclComm.MIN)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MIN)

    def bcast0(self, t: torch.Tensor) -> None:
        if self.shard.world == 1:
            return
        if self.comm is not None:
            self.comm.broadcast(t, 0)
        else:
            dist.broadcast(t, src=0)


def _probe_capture(comm: RcclComm) -> bool:
    """Whether ``comm``'s collectives record into and replay from a hipGraph on this
    system: a graph of (broadcast from rank 0, kernel, all-reduce MIN) captured, replayed
    twice with new inputs and checked, every rank agreeing (agree_capture)."""
    dev = torch.device("cuda", torch.cuda.current_device())

    def capture():
        x = torch.zeros(64, dtype=torch.float32, device=dev)
        ids = torch.zeros(16, dtype=torch.int32, device=dev)
        # warm the communicator's channels outside the capture
        comm.broadcast(ids, 0)
        comm.all_reduce(x, RcclComm.MIN)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                comm.broadcast(ids, 0)
                x.copy_(ids[:1].float().expand(64) + torch.arange(64, device=dev) * 0
                        + float(comm.rank))
                comm.all_reduce(x, RcclComm.MIN)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)

        def replay_ok() -> bool:
            ok = True
            for v in (5, 9):
                ids.fill_(v if comm.rank == 0 else -1)
                g.replay()
                torch.cuda.synchronize(dev)
                # every rank: rank 0's ids, then the MIN over ranks of ids + rank = v
                if int(ids[0]) != v or float(x.min()) != v or float(x.max()) != v:
                    ok = False
            return ok
        return replay_ok

    return agree_capture(capture, dev, on_fail=lambda: torch.cuda.synchronize(dev))


def agree_capture(capture, dev: torch.device, on_fail=None) -> bool:
    """The probe's protocol over the default process group (torch.distributed, not the
    communicator under test): ``capture()`` records the collectives and returns a callable
    that replays and checks them (or raises: the runtime refused the capture).  Two
    verdicts, each MIN-reduced over the ranks: whether every rank captured -- a rank
    replays only when all did, since a replayed collective waits for every rank's -- and
    whether every rank's replays were right, so all ranks take the same path."""
    def agreed(ok: bool) -> bool:
        v = torch.tensor([int(ok)], dtype=torch.int64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MIN)
        return bool(int(v.item()))

    try:
        replay_ok = capture()
    except Exception:          # capture refused by the runtime: take the uncaptured path
        replay_ok = None
        if on_fail is not None:
            on_fail()
    if not agreed(replay_ok is not None):
        return False
    return agreed(bool(replay_ok()))
