#!/usr/bin/env python3
"""Benchmark of the agent x candidate scoring + welfare hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): Best-of-N, N = 64 candidates x A = 8
agents per GPU, T = 150 scored tokens per candidate, Llama-3.1-8B vocabulary
(128,256) in bf16, egalitarian welfare.  One step = one full N x A scoring pass:

    logits [A*N*T, V] (resident in HBM)  --cs_logsoftmax_gather-->  token log-probs
      --cs_segment_reduce--> per-(agent, candidate) mean log-prob utility
      --cs_welfare_reduce(MIN)--> [RCCL MIN all-reduce across ranks]
      --cs_segmented_topk(k=1)--> selected candidate

Multi-GPU: agents shard across ranks (8 per GPU, weak scaling); the only exchange
is the MIN all-reduce of the N per-candidate welfare values.

Prints ONE JSON line (rank 0).  `value` = agent x candidate scorings per second of
the whole job; `roofline` prices the dominant kernel (cs_logsoftmax_gather)
against the 8 TB/s HBM peak from HIP-event timing on its own stream;
`cpu_baseline` times the CPU oracle (a port of the reference's fp64 scoring
arithmetic) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG_DIR = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    # name: (agents per GPU, candidates, scored tokens per candidate, vocab, welfare, description)
    "c2": (8, 64, 150, 128_256, "min",
           "C2 best_of_n: N=64 candidates x A=8 agents per GPU, T=150 tokens, "
           "Llama-3.1-8B vocab 128256 bf16 logits, egalitarian welfare"),
    "c4": (32, 256, 4, 128_256, "sumlog",
           "C4 finite_lookahead depth 4: R=256 paths x A=32 agents per GPU, "
           "Llama-3.1-8B vocab 128256 bf16 logits, Nash welfare"),
    # the same C4 scorings with the paths' shared prefixes scored once (the method's
    # engine.score_tree): a full 4-ary depth-4 tree has 4+16+64+256 = 340 nodes per
    # agent instead of 256 x 4 path rows
    "c4tree": (32, 256, 4, 128_256, "sumlog",
               "C4 finite_lookahead depth 4, tree-shared rows: R=256 paths (4-ary, depth 4, "
               "340 nodes) x A=32 agents per GPU, Llama-3.1-8B vocab 128256 bf16 logits, "
               "Nash welfare"),
}


def tree_layout(bf, depth, A, dev):
    """Full bf-ary tree of the given depth, nodes in level order: (nodes per agent, flat
    row index [A * leaves * depth] of every path's nodes, agent-major, path-major)."""
    levels = [bf ** (d + 1) for d in range(depth)]
    start = [sum(levels[:d]) for d in range(depth)]
    n_nodes = sum(levels)
    leaves = levels[-1]
    idx = []
    for p in range(leaves):
        for d in range(depth):
            idx.append(start[d] + p // (bf ** (depth - 1 - d)))
    per_agent = torch.as_tensor(idx, dtype=torch.long, device=dev)
    flat = (torch.arange(A, device=dev)[:, None] * n_nodes + per_agent[None]).reshape(-1)
    return n_nodes, flat


# Beam-search decode steps (BASELINE configs C1, C3, C5).  Total agents are fixed per
# config and sharded over the ranks (strong scaling); every rank proposes the same
# candidates from the replicated reference-policy rows.
BEAM_CONFIGS = {
    # name: (agents total, beams, top-k, vocab, softcap, logits dtype, description)
    "c1": (4, 4, 10, 128_256, 0.0, torch.float32,
           "C1 beam search: B=4 beams x top-10 x A=4 agents, Llama-3.2-1B vocab 128256 fp32 "
           "logits, egalitarian welfare"),
    "c3": (16, 16, 50, 256_000, 30.0, torch.bfloat16,
           "C3 beam search: B=16 beams x top-50 x A=16 agents sharded over the ranks, "
           "Gemma-2-9B vocab 256000 bf16 logits (soft-cap 30), egalitarian welfare, "
           "RCCL MIN all-reduce"),
    "c5": (64, 8, 32, 128_256, 0.0, torch.bfloat16,
           "C5 beam search: B=8 beams x top-32 x A=64 agents sharded over the ranks, "
           "Llama-3.3-70B vocab 128256 bf16 logits, egalitarian welfare, RCCL MIN all-reduce"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--beam", default="c1,c3,c5",
                    help="beam-search decode-step configs reported under 'beam' ('' disables)")
    ap.add_argument("--beam-steps", type=int, default=200)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU time for the oracle baseline sample (0 disables)")
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse "
                         "the multi-rank path with several ranks on one GPU)")
    ap.add_argument("--e2e", action="store_true",
                    help="also time the full scoring pass INCLUDING the transformer forward "
                         "(random-init Llama-3.1-8B bf16, per-agent prefix K/V) and report it "
                         "under 'end_to_end'")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                    help="rocprofv3 PMC summary giving HBM bytes per launch (optional)")
    return ap.parse_args()


def init_dist(n_gpus, backend="nccl"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or os.environ.get("CS_BENCH_FORCE_SHARDED") == "1":
        if backend == "gloo":   # rehearsal: every rank on the one visible GPU
            torch.cuda.set_device(0)
            torch.distributed.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def make_inputs(A, N, T, V, seed, dev):
    rows = A * N * T
    g = torch.Generator(device=dev).manual_seed(seed)
    logits = torch.empty(rows, V, dtype=torch.bfloat16, device=dev)
    chunk = 4096
    for r0 in range(0, rows, chunk):
        r1 = min(rows, r0 + chunk)
        logits[r0:r1] = torch.randn(r1 - r0, V, generator=g, device=dev) * 3.0
    tgt = torch.randint(0, V, (rows, 1), generator=g, device=dev, dtype=torch.int32)
    offsets = torch.arange(0, rows + 1, T, dtype=torch.int32, device=dev)
    return logits, tgt, offsets


def cpu_baseline(A, N, T, V, welfare_kind, seconds):
    """Time the CPU oracle on a bounded sample: 2 agents x 8 candidates of the workload."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    threads = max(1, min(threads, os.cpu_count() or 1))
    orc.set_threads(threads)
    a_s, n_s = 2, 8
    rows = a_s * n_s * T
    rng = np.random.default_rng(99)
    logits = orc.bf16_bits((rng.standard_normal((rows, V), dtype=np.float32) * 3.0))
    tgt = rng.integers(0, V, size=(rows, 1)).astype(np.int32)
    off = np.arange(0, rows + 1, T, dtype=np.int32)
    kind = {"min": orc.MIN, "sumlog": orc.SUMLOG}[welfare_kind]
    iters, t0 = 0, time.perf_counter()
    while True:
        tok, _ = orc.logsoftmax_gather(logits, tgt, bf16=True)
        seg = orc.segment_reduce(tok, off)
        U = (seg["sum_lp"] / seg["count"]).reshape(a_s, n_s)
        W = orc.welfare(U, kind)
        orc.topk(W, 1)
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": a_s * n_s * iters / el, "unit": "scorings/s", "cores": threads, "kind": "port",
            "sample": f"{a_s} agents x {n_s} candidates x T={T} rows of V={V} bf16 "
                      f"(oracle/cs_oracle.c fp64, OpenMP {threads} threads), {iters} passes "
                      f"in {el:.1f} s"}


def end_to_end(A, N, T, V, wkind, dev, steps=2, prefix_len=200, seed=0):
    """Full C2 scoring pass incl. the transformer forward: Llama-3.1-8B (random init, bf16)
    prefills A agent prefixes of `prefix_len` tokens once, then scores N candidates x T
    tokens under every agent (prefix K/V reused by all candidates), LM head, HIP kernels,
    welfare, selection."""
    M = importlib.import_module(PKG_DIR + ".model")
    E = importlib.import_module(PKG_DIR + ".engine")
    ops = importlib.import_module(PKG_DIR + ".ops")
    cfg = M.preset("llama-3.1-8b")
    t0 = time.perf_counter()
    model = M.Model(cfg, dev, torch.bfloat16, seed=seed)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    # every pass re-encodes the prefixes in full (no reuse of the previous pass's K/V)
    eng = E.ScoringEngine(model, max_rows_per_chunk=16384, reuse_caches=0)
    g = torch.Generator().manual_seed(11)
    prefixes = [torch.randint(300, V, (prefix_len,), generator=g).tolist() for _ in range(A)]
    cands = [torch.randint(300, V, (T,), generator=g).tolist() for _ in range(N)]
    owner = [a for a in range(A) for _ in range(N)]
    conts = [cands[c] for _ in range(A) for c in range(N)]
    offs = eng.offsets(conts, dev)

    def one_pass():
        cache = eng.prefill(prefixes)
        lp = eng.score(cache, owner, conts)
        seg = ops.segment_reduce(lp, offs)
        U = (seg["sum_lp"] / seg["count"].to(torch.float32)).view(A, N).contiguous()
        W = ops.welfare(U, wkind)
        return ops.topk(W, 1)[0]

    one_pass()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"model": "llama-3.1-8b (random init, bf16)", "prefix_tokens": prefix_len,
            "scored_tokens": A * N * T, "s_per_pass": dt, "scorings_per_s": A * N / dt,
            "tokens_per_s": A * N * T / dt, "model_init_s": init_s, "passes": steps,
            "note": "forward = PyTorch/hipBLASLt (plumbing); logits -> HIP C-ABI kernels"}


def gpu_busy(stream, ms=20.0):
    """Keep the GPU busy for ~ms so that the launches queued behind are timed by their
    events without host launch gaps (small kernels would otherwise be host-bound)."""
    with torch.cuda.stream(stream):
        try:
            torch.cuda._sleep(int(ms * 2.0e6))   # ~2 GHz shader clock
        except (AttributeError, RuntimeError):
            a = torch.randn(4096, 4096, device=stream.device)
            for _ in range(int(ms)):
                a = a @ a.T * 1e-3


def run_beam(name, world, rank, dev, steps, warmup, comm=None, pmc_json=None):
    """Beam-search decode steps on resident logits (BASELINE C1 / C3 / C5).

    One decode step, per rank:
      reference-policy rows [B, V] --cs_vocab_topk(K)--> candidate tokens [B, K]
      agent rows [A_local*B, V]   --cs_beam_step-->     U = R + lp, W = min over agents
      [RCCL MIN all-reduce of W when the agents are sharded] --> stable order (top-k)
      cumulative rewards of the B kept beams  R <- U[:, order[:B]]
    (the reference's walk over the sorted candidates, beam_search.py:562-600, keeps the
    first beam_width; synthetic candidates have no duplicates / EOS, so the B best are
    exactly what it keeps, and the launch selects just those)
    At N = 1 two whole steps are one captured hipGraph; with agents sharded a step is the
    all-reduce (one ncclAllReduce on the stream through parallel.RcclComm) followed by
    one graph holding this step's selection (cs_beam_select) and the next step's scoring.
    """
    ops = importlib.import_module(PKG_DIR + ".ops")
    par = importlib.import_module(PKG_DIR + ".parallel")
    A, B, K, V, cap, dt, desc = BEAM_CONFIGS[name]
    shard = par.AgentShard(A, rank, world)
    A_loc = len(shard.local)
    C = B * K
    g = torch.Generator(device=dev).manual_seed(4321 + rank)
    ref = (torch.randn(B, V, generator=g, device=dev) * 3.0).to(dt)
    ag = (torch.randn(A_loc * B, V, generator=g, device=dev) * 3.0).to(dt)
    # cumulative rewards, ping-pong: step i reads Rs[i % 2] and the launch writes the kept
    # beams' rewards into Rs[(i + 1) % 2] (cs_beam_step out_kept)
    Rs = [torch.zeros(A_loc, B, dtype=torch.float32, device=dev) for _ in range(2)]
    R = Rs[0]
    ws_p, ws_b, ws_d = ops.Workspace(), ops.Workspace(zeroed=True), ops.Workspace(zeroed=True)
    # CS_BENCH_FORCE_SHARDED=1 (diagnostics): the sharded step on one rank, under torchrun
    sharded = world > 1 or os.environ.get("CS_BENCH_FORCE_SHARDED") == "1"

    # sharded: persistent U / W buffers so that one captured graph can run the select of
    # step i and the scoring of step i + 1 back to back; W is all-reduced in place
    U_buf = torch.empty(A_loc, C, dtype=torch.float32, device=dev)
    Wx = torch.full((C,), float("inf"), dtype=torch.float32, device=dev)

    def score(i=0):
        if A_loc == 0:   # more ranks than agents: this rank only proposes (W stays +inf)
            ops.vocab_topk(ref, K, softcap=cap, workspace=ws_p)
            return
        if not sharded:
            # propose + score + keep the B best in ONE launch (cs_beam_decode_step): the
            # proposer runs beside the agent-row stream; the launch selects the B best
            # (radix select, no full sort) and writes their cumulative rewards
            ops.beam_decode_step(ref, ag, Rs[i % 2], K, "min", n_order=B, softcap=cap,
                                 workspace=ws_d, kept_out=Rs[(i + 1) % 2])
            return
        # sharded: every rank proposes the same candidates (same launch, no order); a
        # column with no usable utility on this rank must not win the MIN all-reduce
        ops.beam_decode_step(ref, ag, R, K, "min", n_order=0, softcap=cap, workspace=ws_d,
                             out_U=U_buf, out_W=Wx)
        Wx.nan_to_num_(nan=float("inf"), posinf=float("inf"), neginf=float("-inf"))

    def select():
        # one launch: +inf -> NaN, stable top-B, the kept beams' rewards (cs_beam_select)
        ops.beam_select(Wx, B, U=U_buf, unfill="min", kept_out=R)

    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(4):   # warm the workspaces / allocator before capture
            score(i)
            if sharded:
                select()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        if not sharded:      # two decode steps per replay (the reward buffers ping-pong)
            score(0)
            score(1)
        else:                # prologue: the first step's scoring
            score()
    if sharded:
        with torch.cuda.graph(g2):   # select of step i, scoring of step i + 1
            select()
            score()
    per_replay = 1 if sharded else 2
    steps = max(per_replay, steps - steps % per_replay)

    def all_reduce_min():
        # the direct RCCL communicator (parallel.RcclComm: one ncclAllReduce on the stream,
        # a few us of host time) when there is one, else the ProcessGroup call
        if comm is not None:
            comm.all_reduce(Wx, comm.MIN)
        else:
            torch.distributed.all_reduce(Wx, op=torch.distributed.ReduceOp.MIN)

    def step():
        if sharded:          # one step = the exchange + select + the next scoring
            all_reduce_min()
            g2.replay()
        else:
            g1.replay()

    if sharded:
        g1.replay()
    for _ in range(max(1, warmup // per_replay)):
        step()
    torch.cuda.synchronize()
    if sharded:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // per_replay):
        step()
    torch.cuda.synchronize()
    if sharded:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    coll_ms, split_us = None, None
    if sharded:   # the exchange alone, HIP events around it (outside the timed steps)
        coll_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(20)]
        for e0, e1 in coll_ev:
            e0.record()
            all_reduce_min()
            e1.record()
        torch.cuda.synchronize()
        coll_ms = float(np.median([a.elapsed_time(b) for a, b in coll_ev]))
        # GPU-side split of a sharded step (queue kept full, so host gaps do not count)
        parts = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(20)]
        gpu_busy(torch.cuda.current_stream())
        for e in parts:
            e[0].record()
            all_reduce_min()
            e[1].record()
            g2.replay()
            e[2].record()
        torch.cuda.synchronize()
        split_us = {n: float(np.median([e[i].elapsed_time(e[i + 1]) for e in parts])) * 1e3
                    for i, n in enumerate(("all_reduce", "select_and_next_scoring_graph"))}
    if sharded:
        tt = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = float(tt.item())

    # kernel-level timing (HIP events on the launch stream), eager: the one launch of a
    # step (cs_beam_decode_step; no order when sharded)
    st = torch.cuda.current_stream()
    n_ev = 50
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(n_ev)]
    gpu_busy(st)   # the host enqueues every launch before the GPU reaches the first event
    for e0, e1 in ev:
        e0.record(st)
        if A_loc:
            ops.beam_decode_step(ref, ag, Rs[0], K, "min", n_order=0 if sharded else B,
                                 softcap=cap, workspace=ws_d,
                                 kept_out=None if sharded else Rs[1])
        e1.record(st)
    torch.cuda.synchronize()
    k_ms = max(float(np.median([a.elapsed_time(b) for a, b in ev])), 1e-6)
    esz = torch.finfo(dt).bits // 8
    alg = (A_loc * B + B) * V * esz   # agent rows + proposer rows
    ms = el * 1000.0 / steps
    return {"workload": desc, "agents": A, "agents_per_gpu": A_loc, "beams": B, "top_k": K,
            "vocab": V, "dtype": str(dt).replace("torch.", ""),
            "decode_steps_per_s": 1000.0 / ms, "ms_per_step": ms,
            "scorings_per_s": A * C / (ms * 1e-3), "steps": steps,
            "timing": "hipGraph replay" + (" + eager RCCL all-reduce" if sharded else ""),
            "roofline": {"bound": "hbm", "kernel": ("cs_beam_decode_step (beam_decode_kernel: proposer + "
                                    "vocab stream + gather + welfare" +
                                    ("" if sharded else " + top-B") + ")"),
                         "kernel_ms": k_ms, "alg_bytes_per_launch": alg,
                         "traffic": (read_traffic(pmc_json, "beam_" + name, A_loc * B + B, V)
                                     if pmc_json else None),
                         "achieved": alg / (k_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "collective": {"op": ("all_reduce(MIN) of W" + (" (direct RCCL communicator)" if comm
                                                             else " (ProcessGroup)")
                                  if sharded else "none (1 GPU)"),
                           "bytes": C * 4 if sharded else 0, "ms_per_step": coll_ms},
            "gpu_split_us": split_us,
            "step_bytes": (A_loc * B + B) * V * esz,
            "step_frac_of_hbm": (A_loc * B + B) * V * esz / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def read_traffic(path, config, rows, V):
    try:
        with open(path) as f:
            d = json.load(f)
        ent = d.get(config)
        if ent and ent.get("rows") == rows and ent.get("vocab") == V:
            return ent.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    world, rank, local = init_dist(args.gpus, args.backend)
    dev = torch.device("cuda", torch.cuda.current_device())
    ops = importlib.import_module(PKG_DIR + ".ops")
    par = importlib.import_module(PKG_DIR + ".parallel")

    A, N, T, V, wkind, desc = CONFIGS[args.config]
    tree = args.config.endswith("tree")
    flat = None
    if tree:   # rows = tree nodes; each path's log-probs are gathered from its nodes
        n_nodes, flat = tree_layout(4, T, A, dev)
        rows = A * n_nodes
        logits, tgt, _ = make_inputs(A, n_nodes, 1, V, 1234 + rank, dev)
        offsets = torch.arange(0, A * N * T + 1, T, dtype=torch.int32, device=dev)
    else:
        rows = A * N * T
        logits, tgt, offsets = make_inputs(A, N, T, V, 1234 + rank, dev)
    ws = ops.Workspace()
    stream = torch.cuda.current_stream()
    shard = par.AgentShard(A * world, rank, world)   # A agents per GPU, round-robin

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        tok, _ = ops.logsoftmax_gather(logits, tgt, workspace=ws)
        if ev is not None:
            ev[1].record(stream)
        if flat is not None:
            tok = tok.view(-1).index_select(0, flat)
        seg = ops.segment_reduce(tok, offsets)
        U = (seg["sum_lp"] / seg["count"].to(torch.float32)).view(A, N)
        if wkind == "sumlog":
            U = torch.exp(U)  # Nash over geometric-mean token probability
        # agents sharded over ranks: MIN all-reduce (egalitarian) or gather + ordered fold
        if ev is not None:
            ev[2].record(stream)
        W = par.combine_welfare(U, wkind, shard, eps=1e-30)
        if ev is not None:
            ev[3].record(stream)
        idx, _ = ops.topk(W, 1)
        return idx

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4))
              for _ in range(args.steps)]
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())
    kern_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    # the welfare exchange (RCCL MIN all-reduce, or all-gather + ordered fold) broken out
    coll_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in events]))
    ms_per_step = elapsed * 1000.0 / args.steps

    line = None
    if rank == 0:
        scorings = A * N * world
        alg_bytes = rows * V * 2 + rows * 4 * 2  # logits read once + targets in + lp out
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        cpu = None
        if world == 1 and args.cpu_seconds > 0 and not tree:
            cpu = cpu_baseline(A, N, T, V, wkind, args.cpu_seconds)
        e2e = None
        if args.e2e and world == 1 and not tree:
            del logits
            torch.cuda.empty_cache()
            e2e = end_to_end(A, N, T, V, wkind, dev)
        line = {
            "metric": "agent×candidate scorings/sec + decode steps/sec at 1/2/4/8 MI355X; % HBM roofline",
            "value": scorings * args.steps / elapsed,
            "unit": "scorings/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "decode_steps_per_s": 1000.0 / ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"workload": desc, "agents_per_gpu": A, "candidates": N,
                       "tokens_per_candidate": T, "vocab": V, "rows_per_gpu": rows,
                       "welfare": wkind, "parallelism": f"agents sharded over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": read_traffic(args.pmc_json, args.config, rows, V),
                         "kernel": "lsg_stream_kernel (cs_logsoftmax_gather)",
                         "kernel_ms": kern_ms, "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "collective": {"op": ("all_reduce(MIN) of W" if wkind == "min" else
                                  "all_gather of [A_local, C] + ordered fold") if world > 1
                           else "none (1 GPU: local fold)",
                           "bytes": N * 4 if wkind == "min" else A * world * N * 4,
                           "ms_per_step": coll_ms},
        }
        if e2e is not None:
            line["end_to_end"] = e2e
    beam = {}
    beams = [b for b in args.beam.split(",") if b]
    comm = None
    if beams and torch.distributed.is_initialized() and args.backend == "nccl":
        try:
            comm = par.RcclComm()
        except Exception as e:   # every rank fails alike (library / symbol): ProcessGroup path
            print(f"bench: direct RCCL communicator unavailable ({e}); using the ProcessGroup",
                  file=sys.stderr, flush=True)
    for name in beams:
        beam[name] = run_beam(name, world, rank, dev, args.beam_steps, 20, comm, args.pmc_json)
    if comm is not None:
        comm.close()
    if rank == 0:
        if beam:
            line["beam"] = beam
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
