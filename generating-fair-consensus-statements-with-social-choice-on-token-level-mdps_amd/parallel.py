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
    m = shard.max_local()
    pad = torch.full((m, C), float("nan"), dtype=torch.float32, device=U_local.device)
    pad[:U_local.shape[0]] = U_local
    bufs = [torch.empty_like(pad) for _ in range(shard.world)]
    dist.all_gather(bufs, pad, group=group)
    allU = torch.cat(bufs, 0)[torch.as_tensor(shard.global_order(), device=U_local.device)]
    return ops.welfare(allU.contiguous(), kind, **kw)
