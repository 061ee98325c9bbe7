"""Choose, per decode-step projection GEMM shape, between hipBLASLt (torch, with the
committed TunableOp selection) and cs_gemm_bf16 (csrc/gemm.hip, each tile variant and K
split), measured on this MI355X with the weights streamed from HBM (distinct matrices
rotated past the Infinity Cache, 20 calls per captured graph), and write the selection the
model reads (ops.gemm_choice; read-only at run time).

Shapes: the q|k|v, output, gate|up (plain and with the gated activation fused), down and
LM-head GEMMs of the C1 / C3 / C5 beam-search decode steps, at every agent shard of 1, 2,
4 and 8 ranks (M = (agents / ranks + 1) * beams: the agents' streams plus the reference
policy's), and of C4's lookahead-tree segments (--configs c4).

    python tools/tune_gemm_dispatch.py [--out gpurun_out/gemm_dispatch.json] [--install]
"""
import argparse
import importlib
import json
import os
import shutil
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
R = importlib.import_module(PKG + ".runtime")
ops = importlib.import_module(PKG + ".ops")
model = importlib.import_module(PKG + ".model")

# projections whose K-split partials the stream forward folds in the consumer's launch
# (q|k|v in cs_rope_place_splitk, down in cs_add_rms_norm_splitk): their split forms are
# timed without cs_gemm_bf16's own fold
FOLDED_BY_CONSUMER = ("qkv", "down")
# the output projection's consumer is the residual add + RMSNorm, which folds its K-split
# partials itself (model._FOLD_IN_NORM, the default since round 6): every form of it is
# timed TOGETHER with that cs_add_rms_norm launch (hipBLASLt / unsplit: the bf16 product
# added; split: the partials folded in the norm), so the fold's bytes are priced where
# they are read ("with_norm" in the record)
WITH_NORM = ("o",) if model._FOLD_IN_NORM else ()

CONFIGS = {"c1": ("llama-3.2-1b", 4, 4), "c3": ("gemma-2-9b", 16, 16), "c5": ("llama-3.3-70b", 64, 8),
           "c4": ("llama-3.1-8b", 32, 0)}
# C4's lookahead tree (branching 4, depth 4): the forward segments of tree levels 1-3 under
# every prompt (the agents' plus the reference policy's: (a + 1) x 4^d rows) and the last
# level's segment with the committed token (a x 65 rows), a = agents on the rank
C4_LEVELS = (4, 16, 64)


def rows_of(cname: str, A: int, B: int, w: int):
    a = A // w + (1 if A % w else 0)
    if cname == "c4":
        return [(a + 1) * n for n in C4_LEVELS] + [a * 65]
    return [(a + 1) * B]


def shapes_of(preset: str):
    c = model.PRESETS[preset]
    d, H, Hkv, D, F = c.d_model, c.n_heads, c.n_kv_heads, c.head_dim, c.d_ff
    act = "gelu_tanh" if c.family == "gemma2" else "silu"
    return [("qkv", (H + 2 * Hkv) * D, d, 0, act), ("o", d, H * D, 0, act),
            ("gate_up", 2 * F, d, 0, act), ("gate_up_act", 2 * F, d, 1, act),
            ("down", d, F, 0, act), ("lm_head", c.vocab, d, 0, act)]


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps
        best = t if best is None else min(best, t)
    return best


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "gemm_dispatch.json"))
    ap.add_argument("--configs", default="c1,c3,c5")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--install", action="store_true")
    ap.add_argument("--packed", type=int, default=1,
                    help="1: also time cs_gemm_bf16_packed (weights in cs_gemm_pack's layout)")
    ap.add_argument("--merge", type=int, default=1,
                    help="1: keep the installed table's entries for shapes this run does not measure")
    ap.add_argument("--variants", default="2,3,4,5,6,7")
    ap.add_argument("--gemms", default="", help="only these shapes (e.g. qkv,down)")
    args = ap.parse_args()
    print("tuning:", R.use_gemm_tuning(), file=sys.stderr)
    dev = torch.device("cuda:0")
    L = ops._lib.load()
    table, record = {}, []
    calls = 20
    for cname in args.configs.split(","):
        preset, A, B = CONFIGS[cname]
        Ms = sorted({m for w in map(int, args.worlds.split(",")) for m in rows_of(cname, A, B, w)})
        for name, N, K, gated, act in shapes_of(preset):
            if args.gemms and name not in args.gemms.split(","):
                continue
            nw = max(2, min(20, (700 << 20) // (N * K * 2) + 1))
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05 for _ in range(nw)]
            pws = [ops.gemm_pack(w) for w in ws] if args.packed else []
            for M in Ms:
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                pair = name in WITH_NORM
                if pair:
                    h_res = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
                    n_w = torch.ones(N, device=dev, dtype=torch.bfloat16)

                    def norm(y):   # the residual add's launch in the stream forward
                        return ops.add_rms_norm(h_res, n_w, 1e-5, b=y, s_out=h_res)
                else:
                    def norm(y):
                        return y
                if gated:
                    Fh = N // 2

                    def tfn():
                        for i in range(calls):
                            gu = x @ ws[i % nw].t()
                            ops.gated_act(gu[:, :Fh], gu[:, Fh:], act)
                else:
                    def tfn():
                        for i in range(calls):
                            norm(x @ ws[i % nw].t())
                t_torch = timed(tfn) / calls * 1e3
                best = ("torch", 0, 0, t_torch)
                cands = []
                for var in map(int, args.variants.split(",")):
                    if var >= 5 and M > 80:
                        continue                 # the thin form takes at most 80 rows
                    for sp in ((1,) if gated or var >= 5 else (1, 2, 4, 8, 16)):
                        if var in (2, 4) and N % 256:
                            continue
                        if (K % (64 * sp) or K // (64 * sp) < 2):
                            continue
                        if sp > 1 and (name in FOLDED_BY_CONSUMER or pair):
                            t = timed(lambda: [norm(ops.gemm_partials(x, ws[i % nw], splits=sp,
                                                                      variant=var))
                                               for i in range(calls)]) / calls * 1e3
                        else:
                            t = timed(lambda: [norm(ops.gemm(x, ws[i % nw], gated=bool(gated),
                                                             act=act, splits=sp, variant=var))
                                               for i in range(calls)]) / calls * 1e3
                        cands.append({"variant": var, "splits": sp, "us": round(t, 2)})
                        if t < best[3]:
                            best = ("cs_gemm", var, sp, t)
                # the packed-weight form (cs_gemm_bf16_packed on cs_gemm_pack'ed copies): used
                # by a model that holds the packed copy of this weight, when it beats both
                pbest = None
                pcands = []
                for var in ((2, 3, 4) if args.packed else ()):
                    for sp in ((1,) if gated else (1, 2, 4, 8, 16)):
                        if var in (2, 4) and N % 256:
                            continue
                        if K % (64 * sp) or K // (64 * sp) < 2:
                            continue
                        if sp > 1 and (name in FOLDED_BY_CONSUMER or pair):
                            t = timed(lambda: [norm(ops.gemm_packed_partials(x, pws[i % nw],
                                                                             splits=sp, variant=var))
                                               for i in range(calls)]) / calls * 1e3
                        else:
                            t = timed(lambda: [norm(ops.gemm_packed(x, pws[i % nw], gated=bool(gated),
                                                                    act=act, splits=sp, variant=var))
                                               for i in range(calls)]) / calls * 1e3
                        pcands.append({"variant": var, "splits": sp, "us": round(t, 2)})
                        if pbest is None or t < pbest[2]:
                            pbest = (var, sp, t)
                rec = {"config": cname, "gemm": name, "M": M, "N": N, "K": K, "gated": gated,
                       "torch_us": round(t_torch, 2), "cs_gemm": cands, "choice": best[0],
                       "best_us": round(best[3], 2)}
                if pair:
                    rec["with_norm"] = True
                if args.packed:
                    rec["cs_gemm_packed"] = pcands
                record.append(rec)
                print(json.dumps(rec), flush=True)
                ent = {}
                if best[0] == "cs_gemm":
                    ent = {"variant": best[1], "splits": best[2], "us": round(best[3], 2),
                           "torch_us": round(t_torch, 2)}
                if pbest is not None and pbest[2] < best[3]:
                    ent["packed"] = {"variant": pbest[0], "splits": pbest[1],
                                     "us": round(pbest[2], 2)}
                    ent["torch_us"] = round(t_torch, 2)
                if ent:
                    table[f"{M},{N},{K},{gated}"] = ent
            del ws, pws
    if args.merge:
        # keep the installed table's choices for the shapes not measured in this run
        inst = os.path.join(REPO, PKG, "tuned", "gemm_dispatch_mi355x.json")
        if os.path.exists(inst):
            with open(inst) as f:
                old = json.load(f)
            seen = {f"{r['M']},{r['N']},{r['K']},{r['gated']}" for r in record}
            table = {**{k: v for k, v in old.get("table", {}).items() if k not in seen}, **table}
            record = [r for r in old.get("measured", [])
                      if f"{r['M']},{r['N']},{r['K']},{r['gated']}" not in seen] + record
    # fused gated entries that lose to the plain GEMM's best form + cs_gated_act
    importlib.import_module("tools.merge_gemm_dispatch").prune_gated(table, record)
    out = {"device": torch.cuda.get_device_name(0), "torch": torch.__version__,
           "hip": torch.version.hip, "library": ops._lib.version(),
           "note": "shapes absent here run on hipBLASLt (torch)", "table": table,
           "measured": record}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    if args.install:
        shutil.copy(args.out, os.path.join(REPO, PKG, "tuned", "gemm_dispatch_mi355x.json"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
