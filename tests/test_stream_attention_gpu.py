"""GPU numerics of the stream-decode kernels (cs_prefix_attention, cs_rope_place) and of
the engine paths built on them, against plain PyTorch fp32 references of the same ops.

cs_prefix_attention is bf16 in / bf16 out with fp32 softmax and a bf16 P for the P.V
MFMA, so it is held to bf16 tolerance against an fp32 attention over the SAME bf16
inputs (|err| <= 2e-2 + 2e-2 |ref|; measured errors are ~4e-3).  The engine-level tests
compare the fused decode (forward_streams / DecodeState) with the eager SDPA path of the
same bf16 model: token log-probs within 3e-2 (both paths round activations to bf16 at
different points), and graph replay against eager execution of the fused path bit for
bit."""
import importlib
import math
import zlib

import pytest
import torch

pytestmark = pytest.mark.gpu

PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"


def _ceil32(n):
    return max(32, (n + 31) // 32 * 32)


def ref_attention(q, kp, vp, plen, kh, vh, hist_base, n_str, T, scale, softcap, gpfx=None,
                  window=0):
    """fp32 reference.  q [n_tok, H, D]; kp/vp [n_prefix, Hkv, ldp, D]; kh/vh [S, Hkv, ldh, D]."""
    n_tok, H, D = q.shape
    S, Hkv = kh.shape[0], kh.shape[1]
    rep = H // Hkv
    out = torch.zeros(n_tok, H, D, dtype=torch.float32, device=q.device)
    qf, kpf, vpf, khf, vhf = (x.float() for x in (q, kp, vp, kh, vh))
    for s in range(S):
        gi = s // n_str
        p = int(gpfx[gi]) if gpfx is not None else gi
        P = int(plen[p])
        for t in range(T):
            n_h = hist_base + t + 1
            K = torch.cat([kpf[p, :, :P], khf[s, :, :n_h]], dim=1)       # [Hkv, n, D]
            Vv = torch.cat([vpf[p, :, :P], vhf[s, :, :n_h]], dim=1)
            qq = qf[s * T + t].view(Hkv, rep, D)
            sc = torch.einsum("grd,gnd->grn", qq, K) * scale
            if softcap > 0:
                sc = softcap * torch.tanh(sc / softcap)
            if window > 0:     # key positions: prefix j -> j, history j -> P + j
                kpos = torch.cat([torch.arange(P), P + torch.arange(n_h)]).to(q.device)
                qpos = P + hist_base + t
                sc = sc.masked_fill((qpos - kpos >= window)[None, None], float("-inf"))
            pr = torch.softmax(sc, dim=-1)
            out[s * T + t] = torch.einsum("grn,gnd->grd", pr, Vv).reshape(H, D)
    return out


CASES = [
    # n_prefix, n_str, T, H, Hkv, D, plens, hist_base, softcap, group map
    (5, 4, 1, 32, 8, 64, [180, 201, 77, 160, 230], 3, 0.0, None),      # C1-like decode (1B)
    (3, 16, 1, 16, 8, 256, [90, 140, 33], 20, 50.0, None),             # C3-like (Gemma-2, cap)
    (4, 8, 1, 64, 8, 128, [300, 12, 64, 250], 47, 0.0, None),          # C5-like (70B, rep 8)
    (2, 6, 37, 32, 8, 128, [45, 96], 0, 0.0, None),                    # scoring chunk (T > 1)
    (3, 2, 5, 8, 2, 64, [40, 64, 1], 2, 0.0, [2, 0, 0]),               # group -> prefix map
    (1, 64, 1, 32, 8, 128, [400], 9, 0.0, None),                       # one prefix, 64 streams
    (2, 3, 1, 4, 4, 64, [31, 33], 0, 0.0, None),                       # rep 1, first step
    (2, 4, 3, 16, 8, 256, [300, 120], 40, 50.0, None, 64),             # Gemma sliding window
    (3, 8, 1, 16, 8, 256, [500, 64, 250], 30, 50.0, None, 100),        # window, decode shape
    (5, 8, 1, 64, 8, 128, [2000, 100, 90, 210, 150], 25, 0.0, None),   # C5 mix: long ref prompt
    (2, 4, 1, 32, 8, 64, [3000, 700], 60, 0.0, [1, 0]),                # long prefixes, mapped
    # C4 lookahead tree level: >= 1024 cells, the reference prompt 16x the agents' (a plan
    # with key splits for the imbalanced cells)
    (33, 64, 1, 32, 8, 128, [4100] + [250 + 3 * i for i in range(32)], 2, 0.0, None),
]


def _ragged(kp_list, Hkv, D):
    """Per-prefix [Hkv, len_p, D] tensors -> (flat [Hkv, Lp, D], offsets): prefix p at rows
    off[p] (multiples of 32), padding rows filled with finite garbage."""
    off, o = [], 0
    for k in kp_list:
        off.append(o)
        o += _ceil32(k.shape[1])
    flat = torch.randn(Hkv, o, D).to(kp_list[0].dtype).to(kp_list[0].device) * 3.0
    for k, o0 in zip(kp_list, off):
        flat[:, o0:o0 + k.shape[1]] = k
    return flat, off


@pytest.mark.parametrize("case", CASES)
def test_prefix_attention_matches_fp32_reference(ops, dev, case):
    n_prefix, n_str, T, H, Hkv, D, plens, hb, cap, gmap = case[:10]
    window = case[10] if len(case) > 10 else 0
    g = torch.Generator(device="cpu").manual_seed(zlib.crc32(repr(case).encode()))
    n_grp = len(gmap) if gmap is not None else n_prefix
    S = n_grp * n_str
    ldh = _ceil32(hb + T)
    bf = torch.bfloat16

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, generator=g) * s).to(bf).to(dev)

    q = rnd(S * T, H, D, s=1.0)
    kps = [rnd(Hkv, n, D) for n in plens]
    vps = [rnd(Hkv, n, D) for n in plens]
    kflat, off = _ragged(kps, Hkv, D)
    vflat, _ = _ragged(vps, Hkv, D)
    vtflat = ops.blocked_vt(vflat)
    kh, vh = rnd(S, Hkv, ldh, D), rnd(S, Hkv, ldh, D)
    plen = torch.tensor(plens, dtype=torch.int32, device=dev)
    offt = torch.tensor(off, dtype=torch.int64, device=dev)
    hbt = torch.tensor([hb], dtype=torch.int32, device=dev)
    gp = torch.tensor(gmap, dtype=torch.int32, device=dev) if gmap is not None else None
    scale = D ** -0.5 * (4.0 if cap else 1.0)      # the cap case drives scores into the cap

    vth = ops.blocked_vt(vh)

    def run(**kw):
        return ops.prefix_attention(q, kflat, vtflat, offt, plen, max(plens), kh,
                                    vth, hbt, n_str, T, scale=scale,
                                    softcap=cap, window=window, group_prefix=gp, **kw)

    out = run()
    # every work plan gives the same attention: exact host lengths (per-group key splits),
    # and no plan at all (one workgroup per (group, head, query group))
    outs = {"exact": run(prefix_len_host=plens, group_prefix_host=gmap),
            "plain": run(plan=ops.AttnPlan(None, 0, 0, None))}
    torch.cuda.synchronize()
    # reference on padded per-prefix tensors [n_prefix, Hkv, Pmax, D]
    Pm = max(plens)
    kp = torch.zeros(n_prefix, Hkv, Pm, D, dtype=bf, device=dev)
    vp = torch.zeros(n_prefix, Hkv, Pm, D, dtype=bf, device=dev)
    for i, (k, v) in enumerate(zip(kps, vps)):
        kp[i, :, :k.shape[1]] = k
        vp[i, :, :v.shape[1]] = v
    ref = ref_attention(q, kp, vp, plens, kh, vh, hb, n_str, T, scale, cap, gmap, window)
    bound = 2e-2 + 2e-2 * ref.abs()
    for name, o in [("default", out)] + list(outs.items()):
        err = (o.float() - ref).abs()
        assert bool((err <= bound).all()), f"{name}: max err {float(err.max()):.3e}"
    assert torch.equal(out, run())          # deterministic: bit-identical relaunch


@pytest.mark.parametrize("D,H,Hkv,T,col0", [(64, 8, 2, 3, 0), (128, 32, 8, 1, 0), (256, 16, 8, 2, 0),
                                             # T >= 32: V placed by 32-slot tiles (partial
                                             # tiles at both ends: slots 5 .. 5 + T)
                                             (128, 32, 8, 40, 0), (64, 8, 2, 64, 0),
                                             (256, 16, 8, 33, 0),
                                             # rows 8-byte but not 16-byte aligned: 4-pair items
                                             (128, 64, 8, 1, 4), (256, 16, 8, 2, 4)])
def test_rope_place_matches_torch(ops, dev, D, H, Hkv, T, col0):
    M = importlib.import_module(PKG + ".model")
    cfg = M.preset("tiny-llama", head_dim=D, n_heads=H, n_kv_heads=Hkv)
    inv = M.rope_inv_freq(cfg, dev)
    g = torch.Generator(device="cpu").manual_seed(D + H)
    n_prefix, n_str = 3, 2
    S = n_prefix * n_str
    plens = [17, 250, 1000]
    hb = 5
    ldh = _ceil32(hb + T)
    width = (H + 2 * Hkv) * D
    qkv = torch.randn(S * T, width + 8, generator=g).to(torch.bfloat16).to(dev)[:, col0:col0 + width]
    plen = torch.tensor(plens, dtype=torch.int32, device=dev)
    hbt = torch.tensor([hb], dtype=torch.int32, device=dev)
    q_out = torch.empty(S * T, H, D, dtype=torch.bfloat16, device=dev)
    kh = torch.zeros(S, Hkv, ldh, D, dtype=torch.bfloat16, device=dev)
    vth = torch.zeros(S, Hkv, ldh // 32, D, 32, dtype=torch.bfloat16, device=dev)
    ops.rope_place(qkv, inv, plen, hbt, n_str, T, H, Hkv, D, q_out, kh, vth)
    vrows = ops.rows_from_blocked(vth)              # [S, Hkv, ldh, D]
    torch.cuda.synchronize()
    # fp32 reference rotation
    pos = torch.tensor([plens[s // n_str] + hb + t for s in range(S) for t in range(T)],
                       dtype=torch.float32, device=dev)
    ang = pos[:, None] * inv[None]
    cos, sin = ang.cos(), ang.sin()
    x = qkv.float().view(S * T, H + 2 * Hkv, D)
    x1, x2 = x[..., :D // 2], x[..., D // 2:]
    rot = torch.cat([x1 * cos[:, None] - x2 * sin[:, None], x2 * cos[:, None] + x1 * sin[:, None]], -1)
    torch.testing.assert_close(q_out.float(), rot[:, :H], atol=2e-2, rtol=1e-2)
    for s in range(S):
        for t in range(T):
            tok = s * T + t
            torch.testing.assert_close(kh[s, :, hb + t].float(), rot[tok, H:H + Hkv], atol=2e-2, rtol=1e-2)
            assert torch.equal(vrows[s, :, hb + t], qkv[tok].view(-1, D)[H + Hkv:])
    assert kh[:, :, :hb].abs().sum() == 0 and vrows[:, :, hb + T:].abs().sum() == 0
    assert vrows[:, :, :hb].abs().sum() == 0


def _tiny(family, dev, seed=3, dtype=torch.bfloat16, weights=None):
    M = importlib.import_module(PKG + ".model")
    E = importlib.import_module(PKG + ".engine")
    if family == "llama3":
        cfg = M.preset("tiny-llama", vocab=512, d_model=256, n_heads=8, n_kv_heads=2, head_dim=64,
                       d_ff=512, n_layers=3, init_std=0.05)
    else:
        cfg = M.preset("tiny-gemma", vocab=512, d_model=256, n_heads=4, n_kv_heads=2, head_dim=128,
                       d_ff=512, n_layers=3, sliding_window=4096, query_pre_attn_scalar=128.0,
                       init_std=0.05)
    model = M.Model(cfg, dev, dtype, seed=seed, weights=weights)
    return E.ScoringEngine(model, reuse_caches=0)


def _fp32_twin(eng):
    w = {k: v.float() for k, v in eng.model.w.items()}
    fam = eng.model.cfg.family
    M = importlib.import_module(PKG + ".model")
    E = importlib.import_module(PKG + ".engine")
    model = M.Model(eng.model.cfg, eng.device, torch.float32, weights=w)
    return E.ScoringEngine(model, reuse_caches=0)


@pytest.mark.parametrize("family", ["llama3", "gemma2"])
def test_decode_state_matches_fp32_reference(dev, family):
    """DecodeState (static K/V, cs_prefix_attention, graphs) against the eager path of the
    SAME weights in fp32: next-token log-probs no further from fp32 than the eager bf16
    path's (BeamState, SDPA over gathered contexts) plus 1e-2, and graph replays
    bit-identical to the fused path run eagerly."""
    E = importlib.import_module(PKG + ".engine")
    eng = _tiny(family, dev)
    e32 = _fp32_twin(eng)
    g = torch.Generator().manual_seed(11)
    prefixes = [torch.randint(5, 500, (n,), generator=g).tolist() for n in (40, 23, 61)]
    B, steps = 4, 6
    cache = eng.prefill(prefixes)
    c32 = e32.prefill(prefixes)
    ref = E.BeamState(e32, c32, n_prefix=3)
    eag = E.BeamState(eng, cache, n_prefix=3)
    fus = E.DecodeState(eng, cache, n_prefix=3, n_beams=B, max_steps=steps)
    fus_eager = E.DecodeState(eng, cache, n_prefix=3, n_beams=B, max_steps=steps, use_graphs=False)
    V = eng.model.cfg.vocab
    tgt = torch.randint(0, V, (3 * B, 16), generator=g).to(dev).to(torch.int32)
    for step in range(steps):
        parent = [0] * B if step == 0 else torch.randint(0, B, (B,), generator=g).tolist()
        toks = torch.randint(5, 500, (B,), generator=g).tolist()
        for st in (ref, eag, fus, fus_eager):
            st.advance(parent, toks)
        lp32 = e32.rows_logprobs(ref.next_hidden, tgt)
        e_eag = float((eng.rows_logprobs(eag.next_hidden, tgt) - lp32).abs().max())
        e_fus = float((eng.rows_logprobs(fus.hidden, tgt) - lp32).abs().max())
        torch.cuda.synchronize()
        assert e_fus <= 1.5 * e_eag + 1e-2, (step, e_fus, e_eag)
        assert torch.equal(fus.hidden, fus_eager.hidden), step


def test_forward_streams_scoring_chunk_matches_fp32(dev):
    """T > 1 tokens per stream over shared prefixes (the Best-of-N scoring shape):
    forward_streams vs model.extend over per-stream gathered contexts, both against the
    fp32 twin of the model."""
    E = importlib.import_module(PKG + ".engine")
    eng = _tiny("llama3", dev, seed=5)
    e32 = _fp32_twin(eng)
    m = eng.model
    g = torch.Generator().manual_seed(2)
    prefixes = [torch.randint(5, 500, (n,), generator=g).tolist() for n in (30, 52)]
    n_str, T = 5, 13
    toks = torch.randint(5, 500, (2 * n_str, T), generator=g).to(dev)
    c = m.cfg
    tgt = torch.randint(0, c.vocab, (2 * n_str * T, 4), generator=g).to(dev).to(torch.int32)
    own = torch.arange(2, device=dev).repeat_interleave(n_str)

    def eager(e):
        cache = e.prefill(prefixes)
        pos = cache.lengths[own][:, None] + torch.arange(T, device=dev)[None]
        ctx = [(k[own], v[own]) for k, v in cache.kv]
        h, _ = e.model.extend(toks, pos, ctx, cache.valid[own], cache.pos[own])
        return e.rows_logprobs(h.reshape(-1, h.shape[-1]), tgt)

    cache = eng.prefill(prefixes)
    pfx = E.fused_prefix(cache)
    hk = [torch.zeros(2 * n_str, c.n_kv_heads, 32, c.head_dim, dtype=torch.bfloat16, device=dev)
          for _ in range(c.n_layers)]
    hv = [torch.zeros(2 * n_str, c.n_kv_heads, 1, c.head_dim, 32, dtype=torch.bfloat16, device=dev)
          for _ in range(c.n_layers)]
    hb = torch.zeros(1, dtype=torch.int32, device=dev)
    h = m.forward_streams(toks.reshape(-1), pfx, hk, hv, hb, n_str, T)
    lp = eng.rows_logprobs(h, tgt)
    lp32 = eager(e32)
    e_eag = float((eager(eng) - lp32).abs().max())
    e_fus = float((lp - lp32).abs().max())
    assert e_fus <= 1.5 * e_eag + 1e-2, (e_fus, e_eag)


@pytest.mark.parametrize("family,force_miss", [("llama3", 0), ("gemma2", 0), ("llama3", 2),
                                               ("gemma2", 1)])
def test_beam_search_fast_topk_equals_host_loop(dev, family, force_miss):
    """The fast top-K loop (one graph replay per step ending in cs_beam_decode_step, one
    device->host copy) and the general host loop (cs_vocab_topk + cs_beam_step per step)
    on the SAME fused decode state: identical candidates, min-rewards and kept beams at
    every step, and the same statement (both restate beam_search.py:439-667)."""
    R = importlib.import_module(PKG + ".runtime")
    T = importlib.import_module(PKG + ".tokenizer")
    methods = importlib.import_module(PKG + ".methods")
    eng = _tiny(family, dev, seed=7)
    tok = T.CharTokenizer(family, vocab_size=eng.model.cfg.vocab)
    R.register_engine("test/fused-tiny", eng, tok)
    try:
        ops_ = {"Agent 1": "We should fund public transit.", "Agent 2": "Lower taxes first.",
                "Agent 3": "Protect the environment above all."}
        cfg = {"beam_width": 3, "max_tokens": 9, "proposer": "topk", "top_k": 6}
        # speculative steps; force_miss n: every n-th step's speculation is treated as a
        # miss (rewind + redo with the walk's inputs), as a duplicate or EOS candidate in
        # the order's top B would make it
        gf = methods.get_method_generator("beam_search",
                                          dict(cfg, speculative_steps=True,
                                               speculative_force_miss=force_miss),
                                          "test/fused-tiny")
        sf = gf.generate_statement("How should the city spend its budget?", ops_)
        gh = methods.get_method_generator("beam_search", dict(cfg, fast_topk=False), "test/fused-tiny")
        sh = gh.generate_statement("How should the city spend its budget?", ops_)
        assert gf.decode_path == "fused-topk" and gh.decode_path == "fused"
        # the fast loop queued steps speculatively (and redid any the walk rejected)
        assert gf.spec_hits + gf.spec_misses > 0
        if force_miss:
            assert gf.spec_misses > 0 and len(gf.step_log) > 2
        # the host loop also logs per-agent increments (the BPE log-prob check); compare the
        # fields both paths record
        common = ("candidates", "min_rewards", "kept")
        assert ([{k: s[k] for k in common} for s in gf.step_log]
                == [{k: s[k] for k in common} for s in gh.step_log])
        assert sf == sh
    finally:
        R.clear_engines()


@pytest.mark.parametrize("family", ["llama3", "gemma2"])
def test_prefill_streams_matches_padded_prefill(dev, family):
    """prefill_streams (length buckets, ragged K/V) and the padded prefill + fused_prefix
    give the same prefix K/V (within bf16 rounding of differently padded forwards) and
    DecodeStates over them the same next-token log-probs."""
    E = importlib.import_module(PKG + ".engine")
    eng = _tiny(family, dev, seed=9)
    g = torch.Generator().manual_seed(4)
    lens = (40, 23, 61, 300, 45)
    prefixes = [torch.randint(5, 500, (n,), generator=g).tolist() for n in lens]
    sp = eng.prefill_streams(prefixes)
    pc = eng.prefill(prefixes)
    fp = E.fused_prefix(pc)
    for li in range(eng.model.cfg.n_layers):
        for i, n in enumerate(lens):
            a = sp.fused.k[li][:, int(sp.fused.off[i]):int(sp.fused.off[i]) + n].float()
            b = fp.k[li][:, int(fp.off[i]):int(fp.off[i]) + n].float()
            assert float((a - b).abs().max()) < 5e-2 * max(1.0, float(b.abs().max()))
    assert torch.allclose(sp.last_hidden.float(), pc.last_hidden.float(), atol=5e-2, rtol=5e-2)
    B = 3
    s1 = E.DecodeState(eng, sp, n_prefix=5, n_beams=B, max_steps=4)
    s2 = E.DecodeState(eng, pc, n_prefix=5, n_beams=B, max_steps=4)
    tgt = torch.randint(0, eng.model.cfg.vocab, (5 * B, 8), generator=g).to(dev).to(torch.int32)
    for step in range(3):
        par = [0] * B if step == 0 else [1, 0, 2]
        tk = torch.randint(5, 500, (B,), generator=g).tolist()
        s1.advance(par, tk)
        s2.advance(par, tk)
        d = (eng.rows_logprobs(s1.hidden, tgt) - eng.rows_logprobs(s2.hidden, tgt)).abs().max()
        assert float(d) < 5e-2, step


@pytest.mark.parametrize("plus_one,d,with_b", [(False, 2048, True), (True, 3584, True),
                                               (False, 8192, False), (True, 256, False),
                                               (False, 16384, True)])
def test_add_rms_norm_matches_torch(ops, dev, plus_one, d, with_b):
    g = torch.Generator(device="cpu").manual_seed(d)
    rows = 37
    a = (torch.randn(rows, d, generator=g) * 2).to(torch.bfloat16).to(dev)
    b = (torch.randn(rows, d, generator=g)).to(torch.bfloat16).to(dev) if with_b else None
    w = (torch.randn(d, generator=g) * 0.1 + (0.0 if plus_one else 1.0)).to(torch.bfloat16).to(dev)
    s_ref = (a + b) if with_b else a
    sf = s_ref.float()
    y_ref = sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + 1e-6)
    y_ref = (y_ref * ((1.0 + w.float()) if plus_one else w.float())).to(torch.bfloat16)
    a2 = a.clone()
    y = ops.add_rms_norm(a2, w, 1e-6, b=b, s_out=a2, plus_one=plus_one)
    torch.cuda.synchronize()
    assert torch.equal(a2, s_ref)                    # the residual stream, bf16 add
    diff = (y.float() - y_ref.float()).abs()
    assert float(diff.max()) <= float(y_ref.float().abs().max()) * 2 ** -7


@pytest.mark.parametrize("plus_one,d", [(True, 3584), (True, 256), (False, 2048), (True, 8192)])
def test_add_rms_norm_branch_prenorm_is_the_two_launches(ops, dev, plus_one, d):
    """b_weight (Gemma-2's post-attention / post-MLP norm of the branch) inside the residual
    add's launch is bitwise the separate launch over the branch followed by the add + norm."""
    g = torch.Generator(device="cpu").manual_seed(d + 1)
    rows = 41
    a = (torch.randn(rows, d, generator=g) * 2).to(torch.bfloat16).to(dev)
    b = (torch.randn(rows, d, generator=g) * 3).to(torch.bfloat16).to(dev)
    wb = (torch.randn(d, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    w = (torch.randn(d, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    a_two, a_one = a.clone(), a.clone()
    bn = ops.add_rms_norm(b, wb, 1e-6, plus_one=plus_one)
    y_two = ops.add_rms_norm(a_two, w, 1e-6, b=bn, s_out=a_two, plus_one=plus_one)
    y_one = ops.add_rms_norm(a_one, w, 1e-6, b=b, b_weight=wb, s_out=a_one, plus_one=plus_one)
    torch.cuda.synchronize()
    assert torch.equal(a_one, a_two)
    assert torch.equal(y_one, y_two)


@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
def test_gated_act_matches_torch(ops, dev, act):
    import torch.nn.functional as F
    g = torch.Generator(device="cpu").manual_seed(7)
    gu = (torch.randn(29, 2 * 1536, generator=g) * 3).to(torch.bfloat16).to(dev)
    gate, up = gu[:, :1536], gu[:, 1536:]
    a = F.silu(gate) if act == "silu" else F.gelu(gate, approximate="tanh")
    ref = a * up
    out = ops.gated_act(gate, up, act)
    torch.cuda.synchronize()
    diff = (out.float() - ref.float()).abs()
    assert float(diff.max()) <= 2 ** -6 * float(ref.float().abs().max())


def test_captured_decode_state_is_freed_by_refcount_and_plans_survive_eviction(dev):
    """A DecodeState whose ``post`` closure references it is freed as soon as its last
    reference goes (no reference cycle through the graph keys), so the cyclic collector
    can never destroy its graphs in the middle of a later capture -- checked by running
    gc.collect() INSIDE the next state's capture.  And a captured graph's attention work
    plans stay alive when more than the plan cache's 64 other shapes are built between its
    replays (ops.retain_plans): the replays after the eviction storm still equal an eager
    run bit for bit."""
    import gc
    import weakref
    E = importlib.import_module(PKG + ".engine")
    ops = importlib.import_module(PKG + ".ops")
    eng = _tiny("llama3", dev, seed=13)
    m = eng.model
    g = torch.Generator().manual_seed(5)
    prefixes = [torch.randint(5, 500, (n,), generator=g).tolist() for n in (37, 20, 45)]
    cache = eng.prefill(prefixes)
    B = 3

    def run(use_graphs, storm_at=None, collect_in_post=False):
        st = E.DecodeState(eng, cache, n_prefix=3, n_beams=B, max_steps=10, use_graphs=use_graphs)
        out = []

        def post():                      # references st: the old cycle's shape
            st.hidden.mul_(1.0)
            if collect_in_post:
                gc.collect()             # inside the capture on the graph steps
        toks = torch.Generator().manual_seed(6)
        for step in range(8):
            if step == storm_at:
                # > 64 new plan shapes: every cached plan of the state is evicted
                for n in range(70):
                    ops.attention_plan([40 + n, 21, 50], None, 3, B, 1, m.cfg.n_heads,
                                       m.cfg.n_kv_heads, m.cfg.head_dim, 32, dev)
                torch.cuda.empty_cache()
                gc.collect()
            par = [0] * B if step == 0 else [step % B, 0, (step + 1) % B]
            st.advance(par, torch.randint(5, 500, (B,), generator=toks).tolist(), post=post)
            out.append(st.hidden.clone())
        torch.cuda.synchronize()
        return st, out

    st, _ = run(True)
    ref = weakref.ref(st)
    was = gc.isenabled()
    gc.disable()
    try:
        del st
        assert ref() is None, "a captured DecodeState is only freed by the cyclic collector"
    finally:
        if was:
            gc.enable()
    # garbage to collect while capturing, then a capture that collects it
    for _ in range(3):
        run(True)
    _, got = run(True, storm_at=4, collect_in_post=True)
    _, want = run(False)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


def test_append_prefix_tokens_equals_prefill_of_the_longer_prompts(dev):
    """engine.append_prefix_tokens (a token's K/V copied from the stream that forwarded it
    into the ragged prefix buffers) then a TokenTree level == the same level over a fresh
    prefill_streams of the prompts with the token appended (bf16 rounding of differently
    batched forwards)."""
    E = importlib.import_module(PKG + ".engine")
    eng = _tiny("llama3", dev, seed=21)
    g = torch.Generator().manual_seed(6)
    prompts = [torch.randint(5, 500, (n,), generator=g).tolist() for n in (31, 64, 17)]
    sp = eng.prefill_streams(prompts, reserve=3)
    tree = E.TokenTree(eng, sp, 2)
    toks = [77, 301, 12]
    seg = tree.forward(-1, [0, 0, 0], toks)
    j = 1                                           # commit token 301
    tree.append_to_prefix(seg, j)
    assert sp.lens == [32, 65, 18]
    sp2 = eng.prefill_streams([p + [toks[j]] for p in prompts])
    torch.testing.assert_close(sp.last_hidden.float(), sp2.last_hidden.float(), atol=5e-2, rtol=5e-2)
    nxt = [5, 9, 400, 33]
    t1 = E.TokenTree(eng, sp, 1)
    t2 = E.TokenTree(eng, sp2, 1)
    h1 = t1.segs[t1.forward(-1, [0] * 4, nxt)]["hidden"]
    h2 = t2.segs[t2.forward(-1, [0] * 4, nxt)]["hidden"]
    tgt = torch.randint(0, 512, (12, 6), generator=g).to(dev).to(torch.int32)
    d = (eng.rows_logprobs(h1.reshape(12, -1), tgt) - eng.rows_logprobs(h2.reshape(12, -1), tgt)).abs().max()
    assert float(d) < 5e-2


@pytest.mark.parametrize("D,H,Hkv,T,splits", [(64, 8, 2, 3, 4), (128, 32, 8, 1, 2),
                                               (256, 16, 8, 2, 8), (128, 64, 8, 1, 1)])
def test_rope_place_folds_split_partials_bitwise(ops, dev, D, H, Hkv, T, splits):
    """cs_rope_place_splitk on a K-split projection's fp32 partials == the partials summed in
    split order, rounded to bf16 (cs_gemm_bf16's own fold), then cs_rope_place -- bitwise, for
    q, the rotated K and the placed V."""
    M = importlib.import_module(PKG + ".model")
    cfg = M.preset("tiny-llama", head_dim=D, n_heads=H, n_kv_heads=Hkv)
    inv = M.rope_inv_freq(cfg, dev)
    g = torch.Generator(device="cpu").manual_seed(D + H + splits)
    n_prefix, n_str = 3, 2
    S = n_prefix * n_str
    hb = 5
    ldh = _ceil32(hb + T)
    width = (H + 2 * Hkv) * D
    part = (torch.randn(splits, S * T, width, generator=g) * 2).to(dev)
    folded = part[0].clone()
    for sp in range(1, splits):
        folded = folded + part[sp]
    folded = folded.to(torch.bfloat16)
    plen = torch.tensor([17, 250, 1000], dtype=torch.int32, device=dev)
    hbt = torch.tensor([hb], dtype=torch.int32, device=dev)
    outs = []
    for src in (folded, ops.SplitPartials(part)):
        q_out = torch.empty(S * T, H, D, dtype=torch.bfloat16, device=dev)
        kh = torch.zeros(S, Hkv, ldh, D, dtype=torch.bfloat16, device=dev)
        vth = torch.zeros(S, Hkv, ldh // 32, D, 32, dtype=torch.bfloat16, device=dev)
        ops.rope_place(src, inv, plen, hbt, n_str, T, H, Hkv, D, q_out, kh, vth)
        outs.append((q_out, kh, vth))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
