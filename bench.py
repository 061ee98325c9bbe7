#!/usr/bin/env python3
"""Benchmark of the agent x candidate scoring + welfare hot path on MI355X.

Headline (`value`, BASELINE.json configs[1], "C2"): Best-of-N scoring, N = 64 candidates x
A = 8 agents per GPU, T = 150 scored tokens per candidate, Llama-3.1-8B (random-init,
bf16), egalitarian welfare, END TO END: one step = one full N x A scoring pass,

    prefill the A agent prompts (prefix K/V) -> forward of every (agent, candidate) stream
    over its agent's shared prefix (cs_rope_place + cs_prefix_attention per layer,
    hipBLASLt GEMMs) -> LM head -> cs_logsoftmax_gather -> cs_segment_reduce -> mean
    log-prob utilities -> cs_welfare_reduce(MIN) [-> RCCL MIN all-reduce] ->
    cs_segmented_topk(k=1)

i.e. what one reference `_calculate_candidate_rewards` + `_calculate_egalitarian_welfare`
(src/methods/best_of_n.py:240-418) costs with every get_prompt_logprobs call
(src/utils.py:201-281) served locally.  `value` = agent x candidate scorings/s of the
whole job.  The same line carries:
  kernel_only     the post-LM-head path alone on resident logits (76,800 x 128,256 bf16 =
                  19.7 GB per pass); `roofline` prices its dominant kernel
                  (lsg_stream_kernel of cs_logsoftmax_gather) against 8 TB/s from HIP
                  events on its launch stream, `traffic` from rocprofv3 PMC counters;
  method_decode   BASELINE C1 / C3 / C5 as beam_search generator runs (proposer "topk",
                  random-init Llama-3.2-1B / Gemma-2-9B / Llama-3.3-70B bf16): decode steps/s
                  WITH the forward (one graph replay + one host walk per step);
  beam_kernel     the same decode steps' post-LM-head launch alone on resident logits;
  cpu_baseline    the reference's per-call scoring restated on the host cores (a full
                  forward of prompt + candidate per (agent, candidate), as
                  get_prompt_logprobs re-encodes the prompt every call), plus the fp64 C
                  oracle and torch.log_softmax + gather on a C2 logits sample.

Multi-GPU: `--gpus N` without a torchrun environment relaunches itself under
torch.distributed.run with N ranks (before touching the GPU) and every rank checks the
world size.  Agents shard across ranks (C2: 8 per GPU, weak scaling; C3 / C5: the
config's agents split over the ranks); the only exchange is the MIN all-reduce of the
per-candidate welfare.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG_DIR = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"

# byte-level BPE trained on the reference's texts (tests/golden/make_bpe_fixture.py): real
# prompt token counts (~4 characters per token) for the method-level runs
BPE_FIXTURE = os.path.join(REPO, "tests", "golden", "bpe_fixture")
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_DENSE_TFLOPS = 2500.0   # MI355X dense bf16 MFMA peak (no sparsity)
METRIC = "agent×candidate scorings/sec + decode steps/sec at 1/2/4/8 MI355X; % HBM roofline"

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

# method-level beam search runs (BASELINE configs[0], [2], [4]); agents are the config's
# total, split over the ranks by the generator itself (parallel.method_shard)
METHOD_CONFIGS = {
    "c1": dict(preset="llama-3.2-1b", agents=4, beam_width=4, top_k=10, max_tokens=50,
               desc="C1 beam_search: scenario 1, 4 agents, beam 4, top-10, 50 tokens, "
                    "Llama-3.2-1B (random init, bf16)"),
    "c3": dict(preset="gemma-2-9b", agents=16, beam_width=16, top_k=50, max_tokens=50,
               desc="C3 beam_search: 16 agents, beam 16 x top-50, 50 tokens, Gemma-2-9B "
                    "(random init, bf16; soft-caps 50 / 30)"),
    "c5": dict(preset="llama-3.3-70b", agents=64, beam_width=8, top_k=32, max_tokens=50,
               desc="C5 beam_search: 64 agents, beam 8 x top-32, 50 tokens, Llama-3.3-70B "
                    "(random init, bf16, full replica per GPU)"),
    # BASELINE configs[3]: finite lookahead, 4-ary depth-4 trees (256 paths per step)
    "c4": dict(preset="llama-3.1-8b", agents=32, method="finite_lookahead", branching_factor=4,
               max_depth=4, max_tokens=24, welfare="nash",
               desc="C4 finite_lookahead: depth 4, branching 4 (256 paths per step) x 32 agents, "
                    "Nash welfare, Llama-3.1-8B (random init, bf16)"),
}

# scenario 1 of the reference's appendix configs (configs/appendix/llama/scenario_1/
# beam_search.yaml:20-25): the prompt texts of the synthetic agents
SCENARIO_ISSUE = "Should a person's genetic code be considered private information?"
SCENARIO_OPINIONS = [
    "I'd like to think it should be considered private information and for the persons privacy "
    "to be respected. However, it may be important for research or for the biological family. If "
    "the person is open for it, then their opinion should be respected",
    "A persons genetic code should be considered private information for the sole reason it "
    "belongs to them. I can only think of medical case use scenarios when it may be useful to "
    "someone else in the case of faulty genes etc being eradicated by using someone else's stem "
    "cells or dna to help in this.",
    "The majority of all the genetic code is identical between people. I am undecided on the "
    "matter, the differences make us different. But by sharing all the genetic code, this may "
    "help prevent and cure illnesses so I would be slightly in favour if used appropriately.",
    "I believe that a person's genetic code should be considered private information, the same "
    "way you wouldn't give out your address or personal information to strangers, it should "
    "cover your genetic makeup as well as it could be used to screen out people with specific "
    "genetic markers and for discrimination in the future. Having access to your genetic "
    "information also has the added risk of being potentially harmful to any offspring in the "
    "future and I believe that precaution should be taken to ensure that your genetic code is "
    "safe from abuse by others.",
]


def synthetic_opinions(n):
    """n agent opinions: the scenario's 4 texts cycled, each tagged with its participant
    number so that every agent prompt is distinct (SURVEY.md §8(d) synthetic inputs)."""
    return {f"Agent {i + 1}": f"{SCENARIO_OPINIONS[i % 4]} (participant {i + 1})" for i in range(n)}


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
    # the decode launch at the shape ONE GPU of the 8-GPU C3 / C5 runs holds: its agents'
    # rows (C3 16 / 8 = 2 agents, C5 64 / 8 = 8) beside the replicated proposer rows
    "r8c3": (2, 16, 50, 256_000, 30.0, torch.bfloat16,
             "C3 per GPU at 8 ranks: B=16 beams x top-50 x A=2 local agents (of 16), Gemma-2-9B "
             "vocab 256000 bf16 logits (soft-cap 30), the launch one rank runs per step"),
    "r8c5": (8, 8, 32, 128_256, 0.0, torch.bfloat16,
             "C5 per GPU at 8 ranks: B=8 beams x top-32 x A=8 local agents (of 64), "
             "Llama-3.3-70B vocab 128256 bf16 logits, the launch one rank runs per step"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="workload of the kernel-only leg")
    ap.add_argument("--e2e", default=1, type=int,
                    help="1: the headline value is the forward-included C2 pass (default); "
                         "0: kernel-only (the headline then reports the kernel leg, labelled)")
    ap.add_argument("--method", default="c1,c3,c4,c5",
                    help="method-level decode configs: beam_search c1/c3/c5, finite_lookahead c4 "
                         "('' disables)")
    ap.add_argument("--method-bon", type=int, default=1,
                    help="1: time BASELINE C2 through BestOfNGenerator.score_candidates too")
    ap.add_argument("--method-text-steps", type=int, default=8,
                    help="steps of a short statement timed with the re-tokenized text semantics")
    ap.add_argument("--method-statements", type=int, default=1,
                    help="timed generate_statement calls per method config")
    ap.add_argument("--beam", default="c1,c3,c5,r8c3,r8c5",
                    help="kernel-level beam decode configs on resident logits ('' disables)")
    ap.add_argument("--beam-steps", type=int, default=200)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU time per CPU-baseline sample (0 disables)")
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse "
                         "the multi-rank path)")
    ap.add_argument("--selftest-launch", action="store_true",
                    help="only launch the ranks, check the world size and print the agent split "
                         "(no GPU work; CPU-testable with --backend gloo)")
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="diagnostics, one GPU: run the method legs as rank 0 of an N-rank job "
                         "(its agent shard, the sharded fast loop over a one-rank RCCL "
                         "communicator): the per-GPU shapes of BASELINE's 8-GPU configs")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                    help="rocprofv3 PMC summary giving HBM bytes per launch (optional)")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args) -> int:
    """--gpus N outside torchrun: run N ranks under torch.distributed.run as a CHILD
    process (this process never touches the GPU) and exit with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ))


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and os.environ.get("CS_BENCH_FORCE_SHARDED") != "1":
        sys.exit(f"bench: world size {world} != --gpus {args.gpus}; run under torchrun with "
                 f"--nproc-per-node {args.gpus} or let bench.py launch the ranks itself")
    if args.selftest_launch:
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo" if args.backend == "gloo" else args.backend)
        return world, rank, local
    if world == 1 and args.emulate_ranks > 1:
        # rank 0 of an emulated N-rank job: a one-rank process group (collectives are the
        # identity over it) and every method's agent shard as rank 0 of N would hold it
        torch.cuda.set_device(0)
        torch.distributed.init_process_group(
            "nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
            device_id=torch.device("cuda", 0))
        par = importlib.import_module(PKG_DIR + ".parallel")
        n_emu = args.emulate_ranks
        par.method_shard = lambda n_agents, config=None: par.AgentShard(n_agents, 0, n_emu)

        def gather_emulated(U_local, shard, group=None):
            # the other ranks' agents stand in as copies of this rank's rows (same shape
            # and device work as the all-gather's result; values are not compared)
            if shard.world == 1:
                return U_local
            pad = torch.full((shard.max_local(), U_local.shape[1]), float("nan"),
                             dtype=U_local.dtype, device=U_local.device)
            pad[:U_local.shape[0]] = U_local
            return torch.cat([pad] * shard.world, 0)[
                torch.as_tensor(shard.global_order(), device=U_local.device)]

        par.gather_agents = gather_emulated
        return world, rank, local
    if world > 1 or os.environ.get("CS_BENCH_FORCE_SHARDED") == "1":
        if args.backend == "gloo":   # rehearsal: every rank on the one visible GPU
            torch.cuda.set_device(0)
            torch.distributed.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def selftest_launch(world, rank, local):
    """The launch contract without GPU work: every rank reports itself and its agent share."""
    par = importlib.import_module(PKG_DIR + ".parallel")
    me = {"rank": rank, "local_rank": local,
          "c2_agents": par.AgentShard(8 * world, rank, world).local,
          "c3_agents": par.AgentShard(16, rank, world).local,
          "c5_agents": par.AgentShard(64, rank, world).local}
    if world > 1:
        allm = [None] * world
        torch.distributed.all_gather_object(allm, me)
        torch.distributed.barrier()
    else:
        allm = [me]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "selftest_launch": True, "n_gpus": world,
                          "ranks": allm}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def _barrier_sync(world):
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def _max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def _free(*_objs):
    R = importlib.import_module(PKG_DIR + ".runtime")
    R.clear_engines()
    import gc
    gc.collect()
    torch.cuda.empty_cache()


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


def c2_kernel_leg(args, world, rank, dev):
    """The post-LM-head path alone on resident logits (BASELINE C2 / C4 shapes):
    cs_logsoftmax_gather -> cs_segment_reduce -> mean -> welfare -> [all-reduce] -> top-1."""
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
        if ev is not None:
            ev[2].record(stream)
        W = par.combine_welfare(U, wkind, shard, eps=1e-30)
        if ev is not None:
            ev[3].record(stream)
        idx, _ = ops.topk(W, 1)
        return idx

    for _ in range(args.warmup):
        step()
    events = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4))
              for _ in range(args.steps)]
    _barrier_sync(world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    _barrier_sync(world)
    elapsed = _max_over_ranks(time.perf_counter() - t0, world, dev)
    kern_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    coll_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in events]))
    ms = elapsed * 1000.0 / args.steps
    alg_bytes = rows * V * 2 + rows * 4 * 2  # logits read once + targets in + lp out
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    del logits
    return {
        "workload": desc, "timing": "eager launches, resident bf16 logits",
        "scorings_per_s": A * N * world * args.steps / elapsed, "ms_per_step": ms,
        "passes_per_s": 1000.0 / ms, "rows_per_gpu": rows, "steps": args.steps,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": read_traffic(args.pmc_json, args.config, rows, V),
                     "kernel": "lsg_stream_kernel (cs_logsoftmax_gather)",
                     "kernel_ms": kern_ms, "alg_bytes_per_launch": alg_bytes},
        "collective": {"op": ("all_reduce(MIN) of W" if wkind == "min" else
                              "all_gather of [A_local, C] + ordered fold") if world > 1
                       else "none (1 GPU: local fold)",
                       "bytes": N * 4 if wkind == "min" else A * world * N * 4,
                       "ms_per_step": coll_ms},
    }


def _model_flops_per_token(cfg):
    """2 x the parameters one token multiplies (projections, MLP, LM head)."""
    d, L = cfg.d_model, cfg.n_layers
    per_layer = d * (cfg.n_heads + 2 * cfg.n_kv_heads) * cfg.head_dim + cfg.n_heads * cfg.head_dim * d \
        + 3 * d * cfg.d_ff
    return 2.0 * (L * per_layer + cfg.vocab * d)


def c2_e2e_leg(args, world, rank, dev, prefix_len=200, seed=0):
    """BASELINE C2 end to end: Llama-3.1-8B (random init, bf16) prefills the A agent prefixes,
    scores N candidates x T tokens under every agent (shared prefix K/V on the stream
    kernels), LM head, HIP kernels, welfare (+ RCCL MIN all-reduce), selection."""
    M = importlib.import_module(PKG_DIR + ".model")
    E = importlib.import_module(PKG_DIR + ".engine")
    ops = importlib.import_module(PKG_DIR + ".ops")
    par = importlib.import_module(PKG_DIR + ".parallel")
    A, N, T, V, wkind, desc = CONFIGS["c2"]
    cfg = M.preset("llama-3.1-8b")
    t0 = time.perf_counter()
    model = M.Model(cfg, dev, torch.bfloat16, seed=seed)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    # every pass re-encodes its prefixes (no reuse of the previous pass's K/V)
    eng = E.ScoringEngine(model, reuse_caches=0)
    g = torch.Generator().manual_seed(11 + rank)
    prefixes = [torch.randint(300, V, (prefix_len,), generator=g).tolist() for _ in range(A)]
    cands = [torch.randint(300, V, (T,), generator=g).tolist() for _ in range(N)]
    owner = [a for a in range(A) for _ in range(N)]
    conts = [cands[c] for _ in range(A) for c in range(N)]
    offs = eng.offsets(conts, dev)
    shard = par.AgentShard(A * world, rank, world)

    def one_pass():
        cache = eng.prefill(prefixes)
        lp = eng.score(cache, owner, conts)
        seg = ops.segment_reduce(lp, offs)
        U = (seg["sum_lp"] / seg["count"].to(torch.float32)).view(A, N).contiguous()
        W = par.combine_welfare(U, wkind, shard, nonfinite="replace")
        return ops.topk(W, 1)[0]

    for _ in range(args.warmup):
        one_pass()
    _barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_pass()
    _barrier_sync(world)
    el = _max_over_ranks(time.perf_counter() - t0, world, dev)
    dt = el / args.steps
    tokens = A * N * T + A * prefix_len
    flops = _model_flops_per_token(cfg) * tokens
    out = {"workload": desc + "; forward included (Llama-3.1-8B random init, bf16, "
                              f"{prefix_len}-token agent prefixes re-encoded every pass)",
           "scorings_per_s": world * A * N / dt, "s_per_pass": dt, "passes": args.steps,
           "scored_tokens_per_gpu": A * N * T, "prefix_tokens_per_gpu": A * prefix_len,
           "tokens_per_s": world * A * N * T / dt, "model_init_s": init_s,
           "path": "ScoringEngine.score -> _score_fused (cs_rope_place + cs_prefix_attention per "
                   "layer; GEMMs hipBLASLt) -> cs_logsoftmax_gather -> folds",
           "model_tflops_per_s": flops / dt / 1e12,
           "mfma_frac": flops / dt / 1e12 / BF16_DENSE_TFLOPS}
    del eng, model
    _free()
    return out


def method_leg_bon(args, world, rank, dev):
    """BASELINE C2 through the product's Best-of-N API: ``BestOfNGenerator.score_candidates``
    (candidate texts re-encoded, the 8 agents' prompts prefilled, every (agent, candidate)
    scored on the stream kernels, the per-pair check of the reference's find() semantics,
    best_of_n.py:240-327) + ``combine_welfare`` + top-1 (best_of_n.py:329-418, 198) on the
    64 candidate TEXTS of ~150 tokens -- the host work of a BoN selection pass included.
    Candidate generation is not part of a pass."""
    R = importlib.import_module(PKG_DIR + ".runtime")
    methods = importlib.import_module(PKG_DIR + ".methods")
    ops = importlib.import_module(PKG_DIR + ".ops")
    par = importlib.import_module(PKG_DIR + ".parallel")
    A, N, T, V, wkind, desc = CONFIGS["c2"]
    t0 = time.perf_counter()
    eng, tok = R.random_engine("llama-3.1-8b", dev, reuse_caches=0, tokenizer_dir=BPE_FIXTURE)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    model_id = "random:llama-3.1-8b"
    R.register_engine(model_id, eng, tok)
    opinions = synthetic_opinions(A * world)
    shard = par.AgentShard(A * world, rank, world)
    # candidate texts: random pieces of the BPE fixture's own vocabulary, cut to T tokens
    g = torch.Generator().manual_seed(11)
    n_real = getattr(tok, "n_table", None) or 4000
    cands = []
    for _ in range(N):
        ids = torch.randint(300, min(n_real, 4000), (T,), generator=g).tolist()
        cands.append(tok.decode(tok.encode(tok.decode(ids))[:T]))
    toks = [len(tok.encode(c)) for c in cands]
    gen = methods.get_method_generator("best_of_n", {"n": N, "seed": 1}, model_id)

    def one_pass():
        U = gen.score_candidates(SCENARIO_ISSUE, opinions, cands, shard)
        W = par.combine_welfare(U, "min", shard, nonfinite="replace", nan_val=gen.DEFAULT_REWARD,
                                posinf_val=gen.REWARD_CLIP_MAX, neginf_val=gen.REWARD_CLIP_MIN)
        return int(ops.topk(W, 1)[0].item())

    for _ in range(max(1, args.warmup // 2)):
        one_pass()
    _barrier_sync(world)
    steps = max(2, args.steps // 4)
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    _barrier_sync(world)
    el = _max_over_ranks(time.perf_counter() - t0, world, dev)
    dt = el / steps
    R.clear_engines()
    del eng, gen
    _free()
    return {"workload": desc + "; product API (BestOfNGenerator.score_candidates + "
                               "combine_welfare + top-1) on candidate texts, forward included",
            "scorings_per_s": world * A * N / dt, "s_per_pass": dt, "passes": steps,
            "candidate_tokens_mean": sum(toks) / len(toks), "model_init_s": init_s,
            "note": "vs end_to_end: + text encoding, the agents' prompt rendering and the "
                    "per-(agent, candidate) find() check of the reference's span semantics"}


def method_leg_fl(name, args, world, rank, dev):
    """BASELINE C4 as the product's finite_lookahead generator on a random-init model
    (stream path: one prefill per statement, every step's 4-ary depth-4 tree decoded level
    by level under all agents + the reference prompt, one cs_logsoftmax_gather launch over
    the agent rows, Nash welfare): decode steps/s with the forward included, and the live
    roofline of that launch (the last step's launch replayed back to back between HIP events)."""
    R = importlib.import_module(PKG_DIR + ".runtime")
    methods = importlib.import_module(PKG_DIR + ".methods")
    mc = METHOD_CONFIGS[name]
    t0 = time.perf_counter()
    eng, tok = R.random_engine(mc["preset"], dev, reuse_caches=0, tokenizer_dir=BPE_FIXTURE)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    model_id = "random:" + mc["preset"]
    R.register_engine(model_id, eng, tok)
    opinions = synthetic_opinions(mc["agents"])
    # the committed token's id is appended (retokenize "ids", as the beam legs): with
    # random-init weights most committed tokens are byte fragments whose re-tokenization
    # merges, and the "text" semantics would re-encode every prompt every step
    gcfg = {"branching_factor": mc["branching_factor"], "max_depth": mc["max_depth"],
            "max_tokens": mc["max_tokens"], "seed": 1, "welfare": mc["welfare"],
            "retokenize": "ids"}
    warm = methods.get_method_generator("finite_lookahead", dict(gcfg, max_tokens=2), model_id)
    warm.generate_statement(SCENARIO_ISSUE, opinions)
    gen = methods.get_method_generator("finite_lookahead", dict(gcfg), model_id)
    gen._lsg_events = []
    _barrier_sync(world)
    t0 = time.perf_counter()
    gen.generate_statement(SCENARIO_ISSUE, opinions)
    _barrier_sync(world)
    el = _max_over_ranks(time.perf_counter() - t0, world, dev)
    st = np.asarray(gen.step_times + [t0 + el])
    d = np.diff(st)
    steady = d[1:] if d.size > 2 else d
    step_s = _max_over_ranks(float(np.median(steady)), world, dev)
    steps = len(gen.trace)
    n_paths = float(np.mean([len(t["paths"]) for t in gen.trace])) if gen.trace else 0.0
    A = mc["agents"]
    V = eng.model.cfg.vocab
    ev = gen._lsg_events
    k_inline = float(np.mean([a.elapsed_time(b) for a, b, _ in ev])) if ev else None
    k_ms, rows = None, 0.0
    last = getattr(gen, "_lsg_last", None)
    if last is not None:
        # the last step's launch again, 20 back to back between two events: the mean launch
        # duration without the per-launch event overhead of the inline timing
        lg, tg = last
        rows = float(lg.shape[0])
        ops_ = importlib.import_module(PKG_DIR + ".ops")
        ops_.logsoftmax_gather(lg, tg, softcap=eng.softcap, workspace=eng.ws)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops_.logsoftmax_gather(lg, tg, softcap=eng.softcap, workspace=eng.ws)
        e1.record()
        torch.cuda.synchronize()
        k_ms = e0.elapsed_time(e1) / 20
        del lg, tg, last
        gen._lsg_last = None
    alg = rows * V * 2 + rows * 4 * 4 * 2
    out = {"workload": mc["desc"], "agents": A,
           "agents_per_gpu": len(range(rank, A, max(world, args.emulate_ranks))),
           **({"emulated_ranks": args.emulate_ranks} if args.emulate_ranks > 1 else {}),
           "branching_factor": mc["branching_factor"], "max_depth": mc["max_depth"],
           "decode_steps_per_s": 1.0 / step_s, "ms_per_step": step_s * 1e3,
           "paths_per_step": n_paths, "scorings_per_s": A * n_paths / step_s,
           "statement_s": el, "steps_per_statement": steps, "model_init_s": init_s,
           "decode_path": gen.decode_path, "stream_stats": getattr(gen, "stream_stats", None),
           "timing": "median host step time of the generator's loop (tree of the step: one LM "
                     "head + reference draws + a forward segment per depth under every prompt; "
                     "one cs_logsoftmax_gather over the agent rows; welfare; top-1; the "
                     "committed token's K/V appended to every prompt), max over ranks; "
                     "statement_s includes the one prefill",
           "roofline": ({"bound": "hbm", "kernel": "lsg_stream_kernel (cs_logsoftmax_gather over "
                         "every agent row of the step's tree, 4 targets per row)",
                         "kernel_ms": k_ms, "rows": rows, "alg_bytes_per_launch": alg,
                         "achieved": alg / (k_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "kernel_ms_inline": k_inline,
                         "timing": "the statement's last launch replayed 20 times back to back "
                                   "between two HIP events (kernel_ms_inline: events around each "
                                   "launch inside the generator, mean over the steps)"}
                        if k_ms else None)}
    del eng, gen, warm
    _free()
    return out


def method_leg(name, args, world, rank, dev):
    """A BASELINE beam configuration as the product's beam_search generator on a random-init
    model: decode steps/s with the forward included (one captured graph replay + one
    device->host copy + the reference's host walk per step)."""
    R = importlib.import_module(PKG_DIR + ".runtime")
    E = importlib.import_module(PKG_DIR + ".engine")
    methods = importlib.import_module(PKG_DIR + ".methods")
    mc = METHOD_CONFIGS[name]
    if mc.get("method") == "finite_lookahead":
        return method_leg_fl(name, args, world, rank, dev)
    t0 = time.perf_counter()
    eng, tok = R.random_engine(mc["preset"], dev, reuse_caches=0, tokenizer_dir=BPE_FIXTURE)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    model_id = "random:" + mc["preset"]
    R.register_engine(model_id, eng, tok)
    opinions = synthetic_opinions(mc["agents"])
    # the timed statements score the appended token ids (retokenize "ids"); the BPE fixture
    # gives the prompts their real token counts.  The reference's re-tokenized semantics
    # ("text", the product default) are timed on a short statement below: with random-init
    # weights most proposals are byte fragments that merge across the append, so the text
    # path re-scores a far larger share of candidates than a trained model's would.
    gcfg = {"beam_width": mc["beam_width"], "max_tokens": mc["max_tokens"], "proposer": "topk",
            "top_k": mc["top_k"], "seed": 1, "retokenize": "ids"}
    warm = methods.get_method_generator("beam_search", dict(gcfg, max_tokens=4), model_id)
    warm.generate_statement(SCENARIO_ISSUE, opinions)
    runs = []
    for _ in range(max(1, args.method_statements)):
        gen = methods.get_method_generator("beam_search", dict(gcfg), model_id)
        _barrier_sync(world)
        t0 = time.perf_counter()
        gen.generate_statement(SCENARIO_ISSUE, opinions)
        _barrier_sync(world)
        el = _max_over_ranks(time.perf_counter() - t0, world, dev)
        st = np.asarray(gen.step_times)
        d = np.diff(st)
        steady = d[2:] if d.size > 4 else d           # past the two graph captures
        step_s = _max_over_ranks(float(np.median(steady)) if steady.size else el, world, dev)
        runs.append({"statement_s": el, "steps": gen.steps_run, "step_s": step_s,
                     "path": gen.decode_path,
                     "speculation": {"hits": getattr(gen, "spec_hits", 0),
                                     "misses": getattr(gen, "spec_misses", 0)}})
    step_s = float(np.median([r["step_s"] for r in runs]))
    steps = runs[-1]["steps"]
    A, B, K = mc["agents"], mc["beam_width"], mc["top_k"]
    # the step alone: the same graph (advance + LM head + cs_beam_decode_step) replayed with
    # no host walk in between -> what the host adds per step
    graph_ms = None
    n_ranks = max(world, args.emulate_ranks)
    mine = list(range(rank, A, n_ranks))
    if world == 1:
        # the rank's own agents' step (emulated ranks: the per-GPU shape, without the
        # sharded loop's all-reduce and select graphs)
        ops_l = list(opinions.items())
        graph_ms = _graph_step_ms(eng, tok, dict(ops_l[a] for a in mine),
                                  dict(mc, agents=len(mine)), dev)
    out = {"workload": mc["desc"], "agents": A, "beams": B, "top_k": K,
           "agents_per_gpu": len(mine),
           **({"emulated_ranks": n_ranks} if args.emulate_ranks > 1 else {}),
           "decode_steps_per_s": 1.0 / step_s, "ms_per_step": step_s * 1e3,
           "scorings_per_s": A * B * K / step_s,
           "statement_s": float(np.median([r["statement_s"] for r in runs])),
           "steps_per_statement": steps, "statements": len(runs), "model_init_s": init_s,
           "decode_path": runs[-1]["path"],
           "speculative_steps": runs[-1]["speculation"],
           "timing": "median host step time of the generator's loop (forward + LM head + "
                     "cs_beam_decode_step graph replay, device->host copy, reference walk; the "
                     "next step queued before the walk when it is the order's top B, redone "
                     "on a miss), max over ranks; statement_s includes prefill and the graph "
                     "captures"}
    if graph_ms is not None:
        out["graph_step_ms"] = graph_ms
        out["host_overhead_frac"] = step_s * 1e3 / graph_ms - 1.0
    if args.method_text_steps > 0:
        # the engine's prefix reuse as the product ships it (reuse_caches 4): a step's
        # re-tokenized texts extend the previous step's rows (agent prompt + statement)
        eng.reuse_caches = 4
        eng.reset_prefix_store()
        gen = methods.get_method_generator(
            "beam_search", dict(gcfg, retokenize="text", max_tokens=args.method_text_steps),
            model_id)
        _barrier_sync(world)
        gen.generate_statement(SCENARIO_ISSUE, opinions)
        _barrier_sync(world)
        d = np.diff(np.asarray(gen.step_times))
        # steps 0-2 run eagerly or capture the two step graphs: the steady steps after them
        ms = _max_over_ranks(float(np.median(d[3:] if d.size > 4 else d[1:] if d.size > 1 else d))
                             * 1e3, world, dev)
        n_cand = sum(len(s_["candidates"]) for s_ in gen.step_log)
        out["retokenize_text"] = {
            "ms_per_step": ms, "steps": gen.steps_run, "decode_path": gen.decode_path,
            "rescored_candidates": gen.text_compat_candidates, "candidates": n_cand,
            "from_decode_rows": gen.text_rows_candidates,
            "prefix_reuse": dict(eng.reuse_stats),
            "note": "the reference's re-tokenized last log-prob (product default): candidates "
                    "whose BPE re-tokenization differs from the id append are re-scored on the "
                    "text by a batched prefill; random-init proposals are mostly byte fragments"}
    del eng
    _free()
    if name == "c1":
        out["fp32"] = _method_leg_c1_fp32(mc, gcfg, opinions, world, dev)
    return out


def _method_leg_c1_fp32(mc, gcfg, opinions, world, dev):
    """C1 at its stated precision (BASELINE configs[0]: Llama-3.2-1B fp32 log-probs): the same
    generator on an fp32 random-init model.  The stream kernels serve bf16 models, so an fp32
    model runs the eager decode (engine.BeamState: torch fp32 forward, cs_beam_step scoring)
    with host proposals -- the path the fp32 method-trace replays pin to the reference at
    |delta| <= 5e-5."""
    R = importlib.import_module(PKG_DIR + ".runtime")
    methods = importlib.import_module(PKG_DIR + ".methods")
    eng, tok = R.random_engine(mc["preset"], dev, dtype=torch.float32, reuse_caches=0,
                               tokenizer_dir=BPE_FIXTURE)
    model_id = "random-fp32:" + mc["preset"]
    R.register_engine(model_id, eng, tok)
    warm = methods.get_method_generator("beam_search", dict(gcfg, max_tokens=3), model_id)
    warm.generate_statement(SCENARIO_ISSUE, opinions)
    gen = methods.get_method_generator("beam_search", dict(gcfg), model_id)
    _barrier_sync(world)
    t0 = time.perf_counter()
    gen.generate_statement(SCENARIO_ISSUE, opinions)
    _barrier_sync(world)
    el = _max_over_ranks(time.perf_counter() - t0, world, dev)
    d = np.diff(np.asarray(gen.step_times))
    step_s = _max_over_ranks(float(np.median(d[1:] if d.size > 2 else d)) if d.size else el,
                             world, dev)
    A, B, K = mc["agents"], mc["beam_width"], mc["top_k"]
    R.clear_engines()
    del eng, gen, warm
    _free()
    return {"workload": mc["desc"].replace("bf16", "fp32"), "dtype": "f32",
            "decode_path": "eager (BeamState, fp32)", "ms_per_step": step_s * 1e3,
            "decode_steps_per_s": 1.0 / step_s, "scorings_per_s": A * B * K / step_s,
            "statement_s": el, "steps_per_statement": len(d) + 1 if d.size else 1}


def _graph_step_ms(eng, tok, opinions, mc, dev, reps=20):
    """Replays of one decode step's graph (parents' history gather, forward of the new
    tokens, LM head, cs_beam_decode_step) back to back: the GPU cost of a step."""
    E = importlib.import_module(PKG_DIR + ".engine")
    ops = importlib.import_module(PKG_DIR + ".ops")
    P = importlib.import_module(PKG_DIR + ".methods.prompts")
    A, B, K = mc["agents"], mc["beam_width"], mc["top_k"]
    agent_prefixes = [tok.chat_prefix(P.BEAM["agent_system"],
                                      P.BEAM["agent_user"].format(issue=SCENARIO_ISSUE, opinion=o))
                      for o in opinions.values()]
    ref_user = P.BEAM["ref_user"].format(issue=SCENARIO_ISSUE,
                                         opinions_text=P.opinions_text(opinions))
    cache = eng.prefill_streams(agent_prefixes +
                                [tok.render_raw(f"{P.BEAM['ref_system']}\n\n{ref_user}")])
    st = E.DecodeState(eng, cache, n_prefix=A + 1, n_beams=B, max_steps=reps + 3)
    m = eng.model
    U = torch.empty(A, B * K, dtype=torch.float32, device=dev)
    W = torch.empty(B * K, dtype=torch.float32, device=dev)
    rw = torch.zeros(A, B, dtype=torch.float32, device=dev)
    ids = torch.empty(B, K, dtype=torch.int32, device=dev)
    order = torch.empty(B * K, dtype=torch.int32, device=dev)
    ws = ops.Workspace(zeroed=True)

    def post():
        lg = m.lm_head(st.hidden)
        ops.beam_decode_step(lg[A * B:], lg[:A * B], rw, K, "min", n_order=B * K,
                             softcap=eng.softcap, workspace=ws, out_U=U, out_W=W, out_ids=ids,
                             out_order=order)

    par = list(range(B))
    for _ in range(3):                       # eager step + the two captures
        st.advance(par, [5] * B, post=post)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        st.advance(par, [5] * B, post=post)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    st.release()
    return ms


def _host_cores():
    """The host cores this process may use: its affinity mask, capped by OMP_NUM_THREADS
    (the GPU box sets it to its CPU share; the mask shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def _const_model(M, name):
    """An architecture-exact fp32 CPU model with constant weights: a CPU forward's time does
    not depend on the values, and filling is seconds where sampling normals is minutes."""
    cfg = M.preset(name)
    model = M.Model.__new__(M.Model)
    model.cfg = cfg
    w = {n: torch.full(shp, 1.0 if "norm" in n else 0.01, dtype=torch.float32)
         for n, shp in model.shapes().items()}
    return M.Model(cfg, "cpu", torch.float32, weights=w)


def _per_call_scoring(model, P, Tc, seconds, seed=3, min_calls=1):
    """The reference's scoring primitive restated on the host: every (agent, candidate)
    scoring is one forward of the whole prompt + candidate (get_prompt_logprobs re-encodes
    every call, src/utils.py:249-259), then log-softmax over the vocabulary and the gather at
    the candidate tokens.  Returns (calls, seconds)."""
    cfg = model.cfg
    g = torch.Generator().manual_seed(seed)
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            ids = torch.randint(300, cfg.vocab, (1, P + Tc), generator=g)
            _, h, _ = model.prefill(ids, torch.tensor([P + Tc]))
            lg = model.lm_head(h[0, P - 1:P + Tc - 1]).float()
            lp = torch.log_softmax(lg, dim=-1).gather(1, ids[0, P:P + Tc, None])
            float(lp.mean())
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds and n >= min_calls:
                return n, el


def _np_log_softmax_rows(M):
    """core.log_softmax_rows (core.py:64-68) restated in NumPy fp64: M - max - log sum exp."""
    mx = M.max(axis=1, keepdims=True)
    Z = M - mx
    return Z - np.log(np.exp(Z).sum(axis=1, keepdims=True))


def cpu_baseline(seconds, V=128_256, T=150):
    """The reference's scoring path restated on the host cores (kind "port").

    ``value`` (BASELINE C2's config): Llama-3.1-8B fp32, one forward of a 200-token agent
    prompt + a 150-token candidate per (agent, candidate) scoring, as get_prompt_logprobs
    re-encodes the prompt every call, log-softmax + gather at the candidate's tokens -- the
    same workload the GPU headline (`value`) scores, on all host cores.  Also: the same per
    call at BASELINE C1's model (Llama-3.2-1B fp32, 200 + 10 tokens; C1 names "Llama-3.2-1B
    logprobs on CPU"), and the post-LM-head arithmetic on a C2 logits sample three ways: the
    fp64 C oracle, core.log_softmax_rows restated in NumPy fp64 (single thread), and
    torch.log_softmax(x.float()).gather.  BASELINE C3 (Gemma-2-9B fp32, one beam candidate
    token per call) and C4 (Llama-3.1-8B, one 4-token lookahead path per call): the same
    per-call restatement at their shapes (``c3_per_call``, ``c4_per_call``)."""
    M = importlib.import_module(PKG_DIR + ".model")
    cores = _host_cores()
    torch.set_num_threads(cores)
    out = {"unit": "scorings/s", "cores": cores, "kind": "port"}
    # (1) C2 config: 8B fp32, 200-token prompt + 150-token candidate per call
    t0 = time.perf_counter()
    model = _const_model(M, "llama-3.1-8b")
    init_s = time.perf_counter() - t0
    n, el = _per_call_scoring(model, 200, T, seconds, min_calls=2)
    out["value"] = n / el
    out["sample"] = (f"{n} scorings in {el:.1f} s: Llama-3.1-8B fp32 (constant weights) forward of a "
                     f"200-token agent prompt + {T}-token candidate (BASELINE C2's shape), "
                     f"log-softmax over {V} + gather at the candidate's tokens, per (agent, "
                     f"candidate) as get_prompt_logprobs re-encodes every call; torch {cores} "
                     f"threads (model init {init_s:.1f} s, not timed)")
    # (1b) BASELINE C4's scoring call on the same 8B model (Nash welfare over the same
    # per-call utilities): an agent prompt + statement (200 tokens) + one 4-token lookahead
    # path, the mean of the path's log-probs (finite_lookahead.py:490-520)
    n, el = _per_call_scoring(model, 200, 4, seconds / 2)
    out["c4_per_call"] = {
        "value": n / el, "unit": "scorings/s",
        "sample": f"{n} scorings in {el:.1f} s: Llama-3.1-8B fp32 (constant weights) forward of a "
                  f"200-token agent prompt + statement and a 4-token lookahead path, log-softmax + "
                  f"gather at the path's tokens, per (agent, path) as finite_lookahead.py:490-520 "
                  f"calls get_prompt_logprobs; torch {cores} threads"}
    del model
    import gc
    gc.collect()
    # (1c) BASELINE C3's scoring call: Gemma-2-9B fp32, the agent prompt + a 50-token beam
    # (260 tokens) + one candidate token, its last log-prob (beam_search.py:358-390)
    t0 = time.perf_counter()
    model = _const_model(M, "gemma-2-9b")
    init_s = time.perf_counter() - t0
    n, el = _per_call_scoring(model, 260, 1, seconds / 2)
    out["c3_per_call"] = {
        "value": n / el, "unit": "scorings/s",
        "sample": f"{n} scorings in {el:.1f} s: Gemma-2-9B fp32 (constant weights) forward of a "
                  f"260-token agent prompt + beam and one candidate token, log-softmax over 256,000 + "
                  f"the token's log-prob, per (agent, beam, token) as beam_search.py:358-390 calls "
                  f"get_prompt_logprobs; torch {cores} threads (model init {init_s:.1f} s, not timed)"}
    del model
    gc.collect()
    # (1d) BASELINE C5's scoring call: Llama-3.3-70B fp32, the agent prompt + a 60-token beam
    # (260 tokens) + one candidate token.  A whole 80-layer fp32 call is ~0.5 minute of host
    # time, so it is timed on 2- and 4-layer subsets of the full-width model and stated as
    # the extrapolation fixed + 80 x per-layer (per-layer = the difference / 2; fixed =
    # embedding, final norm, LM head over 128,256 and the log-softmax)
    sub = {}
    for nl in (2, 4):
        cfg_s = M.preset("llama-3.3-70b", n_layers=nl)
        ms = M.Model.__new__(M.Model)
        ms.cfg = cfg_s
        w = {n_: torch.full(shp, 1.0 if "norm" in n_ else 0.01, dtype=torch.float32)
             for n_, shp in ms.shapes().items()}
        model = M.Model(cfg_s, "cpu", torch.float32, weights=w)
        _per_call_scoring(model, 260, 1, 0.0)                 # warm (first-touch pages)
        n, el = _per_call_scoring(model, 260, 1, seconds / 8)
        sub[nl] = el / n
        del model, w, ms
        gc.collect()
    per_layer = max(0.0, (sub[4] - sub[2]) / 2)
    fixed = max(0.0, sub[2] - 2 * per_layer)
    call_s = fixed + 80 * per_layer
    out["c5_per_call"] = {
        "value": 1.0 / call_s, "unit": "scorings/s", "extrapolated": True,
        "sample": f"Llama-3.3-70B fp32 (constant weights, full widths) forward of a 260-token agent "
                  f"prompt + beam and one candidate token, log-softmax over 128,256 + the token's "
                  f"log-prob, per (agent, beam, token) as beam_search.py:358-390 calls "
                  f"get_prompt_logprobs; timed on 2 / 4 of its 80 layers ({sub[2]:.2f} / "
                  f"{sub[4]:.2f} s per call) and extrapolated: {fixed:.2f} s fixed + 80 x "
                  f"{per_layer:.3f} s per layer = {call_s:.1f} s per call; torch {cores} threads"}
    # (2) C1 config: 1B fp32, 200 + 10 tokens per call
    t0 = time.perf_counter()
    model = _const_model(M, "llama-3.2-1b")
    init_s = time.perf_counter() - t0
    n, el = _per_call_scoring(model, 200, 10, seconds / 2)
    out["c1_per_call"] = {
        "value": n / el, "unit": "scorings/s",
        "sample": f"{n} scorings in {el:.1f} s: Llama-3.2-1B fp32 (constant weights) forward of a "
                  f"200-token prompt + 10-token candidate, log-softmax + gather, per call; torch "
                  f"{cores} threads (model init {init_s:.1f} s, not timed)"}
    del model
    gc.collect()
    # (3) the post-LM-head arithmetic on C2 rows
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    orc.set_threads(cores)
    a_s, n_s = 2, 8
    rows = a_s * n_s * T
    rng = np.random.default_rng(99)
    x32 = rng.standard_normal((rows, V), dtype=np.float32) * 3.0
    logits = orc.bf16_bits(x32)
    tgt = rng.integers(0, V, size=(rows, 1)).astype(np.int32)
    off = np.arange(0, rows + 1, T, dtype=np.int32)
    iters, t0 = 0, time.perf_counter()
    while True:
        tok, _ = orc.logsoftmax_gather(logits, tgt, bf16=True)
        seg = orc.segment_reduce(tok, off)
        U = (seg["sum_lp"] / seg["count"]).reshape(a_s, n_s)
        orc.topk(orc.welfare(U, orc.MIN), 1)
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds / 4:
            break
    out["oracle_post_lm_head"] = {"value": a_s * n_s * iters / el, "unit": "scorings/s",
                                  "sample": f"{a_s} agents x {n_s} candidates x T={T} rows of "
                                            f"V={V} bf16, oracle/cs_oracle.c fp64, {iters} passes"}
    # core.log_softmax_rows (NumPy fp64) + gather + the reference's per-candidate mean / min
    xb = torch.from_numpy(x32).to(torch.bfloat16)
    x64 = xb.double().numpy()
    tg = tgt[:, 0].astype(np.int64)
    iters, t0 = 0, time.perf_counter()
    while True:
        ls = _np_log_softmax_rows(x64)
        lp = ls[np.arange(rows), tg]
        U = lp.reshape(a_s, n_s, T).mean(axis=2)
        int(np.argmax(U.min(axis=0)))
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds / 4:
            break
    out["numpy_fp64_log_softmax_rows"] = {
        "value": a_s * n_s * iters / el, "unit": "scorings/s",
        "gb_per_s": rows * V * 2 * iters / el / 1e9,
        "sample": f"core.log_softmax_rows (core.py:64-68) restated in NumPy fp64 + gather + mean "
                  f"+ min + argmax on [{rows}, {V}] (bf16 values), {iters} passes, NumPy threads"}
    iters, t0 = 0, time.perf_counter()
    tt = torch.from_numpy(tgt.astype(np.int64))
    while True:
        lp = torch.log_softmax(xb.float(), dim=-1).gather(1, tt)
        float(lp.sum())
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds / 4:
            break
    out["torch_log_softmax_gather"] = {
        "value": a_s * n_s * iters / el, "unit": "scorings/s",
        "gb_per_s": rows * V * 2 * iters / el / 1e9,
        "sample": f"torch.log_softmax(x.float()).gather on [{rows}, {V}] bf16, {iters} passes"}
    return out


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


_LEG = ["start", time.time()]


def _progress(name):
    """Mark the start of a bench leg on stderr (the JSON line stays the only stdout line)."""
    _LEG[0], _LEG[1] = name, time.time()
    print(f"bench: leg {name}", file=sys.stderr, flush=True)


def _heartbeat(period=45.0):
    """A daemon thread that reports the running leg every `period` s on stderr, so a long
    leg (a 70B model init, the first import on a fresh box) is visibly alive."""
    import threading

    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"bench: {time.time() - t0:.0f} s, leg {_LEG[0]} running for "
                  f"{time.time() - _LEG[1]:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    _heartbeat()
    world, rank, local = init_dist(args)
    if args.selftest_launch:
        selftest_launch(world, rank, local)
        return
    dev = torch.device("cuda", torch.cuda.current_device())
    par = importlib.import_module(PKG_DIR + ".parallel")
    gemm_tuning = importlib.import_module(PKG_DIR + ".runtime").use_gemm_tuning()

    errors = {}

    def guarded(name, fn, *a):
        """A failing leg is reported in the line (and on stderr), not a lost line."""
        try:
            return fn(*a)
        except Exception as e:   # noqa: BLE001
            import traceback
            traceback.print_exc()
            errors[name] = f"{type(e).__name__}: {e}"[:500]
            _free()
            return None

    _progress("kernel_only")
    kern = c2_kernel_leg(args, world, rank, dev)
    _free()
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
        _progress("beam_kernel." + name)
        r = guarded("beam_kernel." + name, run_beam, name, world, rank, dev, args.beam_steps, 20,
                    comm, args.pmc_json)
        if r is not None:
            beam[name] = r
    if comm is not None:
        comm.close()
    _free()
    _progress("end_to_end")
    e2e = (guarded("end_to_end", c2_e2e_leg, args, world, rank, dev)
           if args.e2e and args.config == "c2" else None)
    method = {}
    if args.e2e and args.config == "c2" and args.method_bon:
        _progress("method_bon.c2")
        r = guarded("method_bon.c2", method_leg_bon, args, world, rank, dev)
        if r is not None:
            method["c2_best_of_n"] = r
    for name in [m for m in args.method.split(",") if m]:
        _progress("method_decode." + name)
        r = guarded("method_decode." + name, method_leg, name, args, world, rank, dev)
        if r is not None:
            method[name] = r
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        _progress("cpu_baseline")
        cpu = guarded("cpu_baseline", cpu_baseline, args.cpu_seconds)

    if rank == 0:
        A, N, T, V, wkind, desc = CONFIGS[args.config]
        if e2e is not None:
            value, ms, note = e2e["scorings_per_s"], e2e["s_per_pass"] * 1e3, "end_to_end"
        else:
            value, ms, note = kern["scorings_per_s"], kern["ms_per_step"], "kernel_only"
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "scorings/s",
            "value_is": note,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "decode_steps_per_s": 1000.0 / ms,
            "higher_is_better": True,
            "scaling": "weak",
            # same-config pair: C2 forward-included scorings/s on the GPU over the same
            # workload's per-call scorings/s on the host cores (cpu_baseline.value, 8B fp32)
            "vs_baseline": (value / cpu["value"]) if (cpu and cpu.get("value") and e2e is not None)
            else None,
            "vs_baseline_is": "value / cpu_baseline.value (BASELINE C2 config on this box's host "
                              "cores; BASELINE.md publishes no number for this metric)",
            "dtype": "bf16",
            "data": "synthetic (random-init weights of the named architectures, synthetic token "
                    "ids / scenario-1 prompt texts)",
            "config": {"workload": desc + ("; forward included" if e2e is not None else
                                           "; post-LM-head kernels on resident logits"),
                       "agents_per_gpu": A, "candidates": N, "tokens_per_candidate": T,
                       "vocab": V, "welfare": wkind,
                       "parallelism": f"agents sharded over {world} GPU(s)"},
            "gemm_tuning": (os.path.relpath(gemm_tuning, os.path.dirname(os.path.abspath(__file__)))
                            if gemm_tuning else None),
            "roofline": kern["roofline"],
            "cpu_baseline": cpu,
            "kernel_only": {k: v for k, v in kern.items() if k != "roofline"},
        }
        if e2e is not None:
            line["end_to_end"] = e2e
        if method:
            for cname in ("c1", "c3", "c4", "c5"):
                ref = (cpu or {}).get(f"{cname}_per_call")
                if ref and cname in method and method[cname].get("scorings_per_s"):
                    method[cname]["vs_cpu"] = method[cname]["scorings_per_s"] / ref["value"]
                    if method[cname].get("fp32"):
                        method[cname]["fp32"]["vs_cpu"] = (method[cname]["fp32"]["scorings_per_s"]
                                                           / ref["value"])
            line["method_decode"] = method
        if beam:
            line["beam_kernel"] = beam
        if errors:
            line["errors"] = errors
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
