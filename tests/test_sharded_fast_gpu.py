"""Agent-sharded FAST paths on the MI355X, rehearsed as 2 ranks on the box's one GPU
(gloo collectives on device tensors; RCCL needs one GPU per rank):

  * beam search, proposer "topk": the sharded fast loop (step graph + rank 0's proposals
    broadcast + scoring graph + MIN all-reduce + selection graph, speculative steps) equals
    the sharded host loop (_loop: host proposals, combine_welfare, topk) on the same ranks
    -- identical candidates, min-rewards and kept beams at every step and the same
    statement (beam_search.py:439-667 on an agent shard);
  * finite lookahead on the stream kernels, agents sharded, Nash welfare: the same trees and
    rewards (bf16 tolerance) as the sharded general path, draws made a function of their
    seeds as in test_lookahead_stream_gpu.py.
Both on bf16 tiny models whose heads the stream kernels serve."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import importlib

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    out = {"rank": rank, "errors": []}
    try:
        import test_lookahead_stream_gpu as tl
        R = importlib.import_module(PKG + ".runtime")
        T = importlib.import_module(PKG + ".tokenizer")
        ops = importlib.import_module(PKG + ".ops")
        methods = importlib.import_module(PKG + ".methods")
        opinions = {f"Agent {i}": t for i, t in enumerate(
            ["We should fund public transit first.", "Lower the city's taxes before anything else.",
             "Protect parks and the environment above all.", "Build more housing near the center.",
             "Invest in schools and teachers."], 1)}
        issue = "How should the city spend its budget?"
        for family in ("llama3", "gemma2"):
            eng = tl._tiny(family, torch.device("cuda:0"), seed=7)
            tok = T.CharTokenizer(family, vocab_size=eng.model.cfg.vocab)
            R.register_engine("test/sharded", eng, tok)
            cfg = {"beam_width": 3, "max_tokens": 9, "proposer": "topk", "top_k": 6}
            for force in (0, 2):
                gf = methods.get_method_generator(
                    "beam_search", dict(cfg, speculative_force_miss=force), "test/sharded")
                sf = gf.generate_statement(issue, opinions)
                gh = methods.get_method_generator("beam_search", dict(cfg, fast_topk=False),
                                                  "test/sharded")
                sh = gh.generate_statement(issue, opinions)
                common = ("candidates", "min_rewards", "kept")
                same = ([{k: s_[k] for k in common} for s_ in gf.step_log]
                        == [{k: s_[k] for k in common} for s_ in gh.step_log])
                if gf.decode_path != "fused-topk-sharded":
                    out["errors"].append(f"{family}: decode path {gf.decode_path}")
                if not same or sf != sh:
                    out["errors"].append(f"{family} force {force}: fast {sf!r} vs host {sh!r}")
                if gf.spec_hits + gf.spec_misses == 0 or (force and gf.spec_misses == 0):
                    out["errors"].append(f"{family}: no speculation ({gf.spec_hits}, {gf.spec_misses})")
                out.setdefault("stmts", []).append(sf)
            R.clear_engines()
        # finite lookahead, stream tree, sharded, Nash
        eng = tl._tiny("llama3", torch.device("cuda:0"), seed=11)
        tok = T.CharTokenizer("llama3", vocab_size=eng.model.cfg.vocab)
        R.register_engine("test/sharded", eng, tok)
        real = ops.vocab_sample
        ops.vocab_sample = tl._seed_sampler(tok, 7, 11)
        try:
            fcfg = {"branching_factor": 3, "max_depth": 3, "max_tokens": 5, "seed": 5,
                    "welfare": "nash"}
            gs = methods.get_method_generator("finite_lookahead", dict(fcfg), "test/sharded")
            ss = gs.generate_statement(issue, opinions)
            ge = methods.get_method_generator("finite_lookahead", dict(fcfg, stream_tree=False),
                                              "test/sharded")
            se = ge.generate_statement(issue, opinions)
        finally:
            ops.vocab_sample = real
        if gs.decode_path != "stream-tree":
            out["errors"].append(f"FL decode path {gs.decode_path}")
        out["errors"] += [f"FL {e}" for e in
                          tl.check_fl_traces(gs.trace, ge.trace, len(opinions), "nash", ss, se)]
        out["fl"] = (ss, se)
        R.clear_engines()
        dist.barrier()
    except Exception as e:   # noqa: BLE001
        import traceback
        out["errors"].append(traceback.format_exc())
    dist.destroy_process_group()
    q.put(out)


def test_sharded_fast_paths_on_gpu_gloo_rehearsal():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert not r["errors"], f"rank {r['rank']}:\n" + "\n".join(r["errors"])
    by_rank = {r["rank"]: r for r in res}
    assert by_rank[0]["stmts"] == by_rank[1]["stmts"]      # every rank, the same statements
    assert by_rank[0]["fl"] == by_rank[1]["fl"]
