"""A/B of BeamState.advance (per-stream [prefix | history | slot] buffers) vs the
concatenating version it replaced, on a C3-like method step: 16 agents + the reference
prefix x 16 beams, 300-token prefixes, random-init bf16 Llama-3.2-1B architecture."""
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
M = importlib.import_module(PKG + ".model")
E = importlib.import_module(PKG + ".engine")


def advance_concat(st, parent, tokens):
    """The previous BeamState.advance (cat of prefix + history per layer, then again)."""
    dev = st.e.device
    m = st.e.model
    P, Bo, Bn = st.n_prefix, st.n_beams, len(parent)
    par = torch.as_tensor(list(parent), dtype=torch.long, device=dev)
    src = (torch.arange(P, device=dev)[:, None] * Bo + par[None, :]).reshape(-1)
    own = torch.arange(P, device=dev).repeat_interleave(Bn)
    tok = torch.as_tensor(list(tokens), dtype=torch.long, device=dev).repeat(P)[:, None]
    c = st.cache
    plen = c.lengths[own]
    pos = (plen + st.G)[:, None]
    pre_mask, pre_pos = c.valid[own], c.pos[own]
    if st.G > 0:
        gpos = plen[:, None] + torch.arange(st.G, device=dev)[None]
        cmask = torch.cat([pre_mask, torch.ones(len(own), st.G, dtype=torch.bool, device=dev)], 1)
        cpos = torch.cat([pre_pos, gpos], 1)
        ctx = [(torch.cat([pk[own], gk[src]], 2), torch.cat([pv[own], gv[src]], 2))
               for (pk, pv), (gk, gv) in zip(c.kv, st.gen_kv)]
    else:
        cmask, cpos = pre_mask, pre_pos
        ctx = [(pk[own], pv[own]) for pk, pv in c.kv]
    h, new = m.extend(tok, pos, ctx, cmask, cpos)
    if st.G > 0:
        st.gen_kv = [(torch.cat([gk[src], nk], 2), torch.cat([gv[src], nv], 2))
                     for (gk, gv), (nk, nv) in zip(st.gen_kv, new)]
    else:
        st.gen_kv = new
    st.G += 1
    st.n_beams = Bn
    st.next_hidden = h[:, 0, :]


def run(mode, steps=12):
    model = M.Model(M.preset("llama-3.2-1b"), "cuda", torch.bfloat16, seed=0)
    eng = E.ScoringEngine(model, reuse_caches=0)
    g = torch.Generator().manual_seed(1)
    prefixes = [torch.randint(300, 120000, (300,), generator=g).tolist() for _ in range(17)]
    st = E.BeamState(eng, eng.prefill(prefixes), n_prefix=17)
    B = 16
    times, hs = [], []
    for t in range(steps):
        parent = [0] * B if t == 0 else torch.randint(0, B, (B,), generator=g).tolist()
        tokens = torch.randint(300, 120000, (B,), generator=g).tolist()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "slots":
            st.advance(parent, tokens)
        else:
            advance_concat(st, parent, tokens)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        hs.append(st.next_hidden.float().cpu())
    return times, hs


if __name__ == "__main__":
    run("concat", steps=2)                    # warm the GEMM / attention paths first
    tc, hc = run("concat")
    ts, hs = run("slots")
    tc2, hc2 = run("concat")
    dh = max((a - b).abs().max().item() for a, b in zip(hs, hc2))
    dn = max((a - b).abs().max().item() for a, b in zip(hc2, hc))
    print(json.dumps({"streams": 17 * 16, "prefix": 300, "steps": len(ts),
                      "max_abs_hidden_diff_concat_vs_concat_rerun": dn,
                      "ms_per_step_slots": 1e3 * sum(ts[2:]) / len(ts[2:]),
                      "ms_per_step_concat": 1e3 * sum(tc[2:]) / len(tc[2:]),
                      "max_abs_hidden_diff": dh}), flush=True)
