"""The shipped bf16 forward at the BASELINE models' REAL sizes.

Every method-trace replay runs a 2-layer fixture; here the decode forward behind every
scoring call (src/utils.py:249-259, the remote forward the reference calls) runs at the
architectures BASELINE.json names, random-init bf16 weights (seeded), through the product's
stream path: DecodeState (engine.prefill_streams, cs_prefix_attention_rows, captured step
graphs) with the decode-step GEMMs the committed dispatch table routes -- packed, gated and
the 7-wave packed gated form at <= 80 rows -- and the fused cs_beam_decode_step over the LM
head's logits at the end:

  * Llama-3.1-8B, all 32 layers (C2 / C4's model), 17 prefixes x 16 beams = 272 streams;
  * Gemma-2-9B, all 42 layers (C3's model: head_dim 256, both soft-caps), 272 streams;
  * Llama-3.3-70B at its full widths (d 8192, d_ff 28672, 64 / 8 heads) with 3 of its 80
    layers, at C5's per-rank row count (9 prefixes x 8 beams = 72 streams: the 7-wave packed
    gate|up 72 x 57,344 x 8,192) and its one-GPU row count (65 x 8 = 520 streams).

The reference for each is the eager fp32 twin holding the SAME bf16-representable weights
(BeamState on an fp32 copy: torch fp32 matmuls and attention).  The bound is derived from
that twin, not tuned: per decode step, the product's per-row log-probs (at the fp32 twin's
top tokens and random tokens) are no further from the fp32 twin than torch's own bf16 eager
forward of the same weights (BeamState on the bf16 model: torch matmuls + SDPA), times 1.5,
plus 1e-2 -- the criterion tests/test_stream_attention_gpu.py holds the 3-layer fixtures
to.  The fused decode launch's U (proposer + agent log-probs in one launch) is checked the
same way against the twin's log-probs of the tokens it proposed."""
import gc
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu

PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"

CASES = [
    # preset, overrides, n_prefix, n_beams, steps
    ("llama-3.1-8b", {}, 17, 16, 3),
    ("gemma-2-9b", {}, 17, 16, 3),
    ("llama-3.3-70b", {"n_layers": 3}, 9, 8, 3),
    ("llama-3.3-70b", {"n_layers": 3}, 65, 8, 2),
]


def _free():
    gc.collect()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name,over,P,B,steps", CASES,
                         ids=[f"{c[0]}-{c[2] * c[3]}rows" for c in CASES])
def test_real_size_stream_decode_against_fp32_twin(dev, name, over, P, B, steps):
    M = importlib.import_module(PKG + ".model")
    E = importlib.import_module(PKG + ".engine")
    ops = importlib.import_module(PKG + ".ops")
    cfg = M.preset(name, **over)
    model = M.Model(cfg, dev, torch.bfloat16, seed=17)
    eng = E.ScoringEngine(model, reuse_caches=0)
    m32 = M.Model(cfg, dev, torch.float32, weights={k: v.float() for k, v in model.w.items()})
    e32 = E.ScoringEngine(m32, reuse_caches=0)
    g = torch.Generator().manual_seed(P * B + cfg.n_layers)
    V = cfg.vocab
    prefixes = [torch.randint(1000, V - 1000, (int(n),), generator=g).tolist()
                for n in torch.randint(40, 120, (P,), generator=g)]
    try:
        fus = E.DecodeState(eng, eng.prefill_streams(prefixes), n_prefix=P, n_beams=B,
                            max_steps=steps)
        eag = E.BeamState(eng, eng.prefill(prefixes), n_prefix=P)
        ref = E.BeamState(e32, e32.prefill(prefixes), n_prefix=P)
        worst = []
        for step in range(steps):
            parent = [0] * B if step == 0 else torch.randint(0, B, (B,), generator=g).tolist()
            toks = torch.randint(1000, V - 1000, (B,), generator=g).tolist()
            for st in (fus, eag, ref):
                st.advance(parent, toks)
            # targets: the fp32 twin's 8 most likely tokens of every row + 8 random ones
            top = m32.lm_head(ref.next_hidden).topk(8, dim=1).indices
            tgt = torch.cat([top, torch.randint(0, V, (P * B, 8), generator=g).to(dev)],
                            1).to(torch.int32)
            lp32 = e32.rows_logprobs(ref.next_hidden, tgt)
            e_fus = float((eng.rows_logprobs(fus.hidden, tgt) - lp32).abs().max())
            e_eag = float((eng.rows_logprobs(eag.next_hidden, tgt) - lp32).abs().max())
            torch.cuda.synchronize()
            worst.append((e_fus, e_eag))
            assert e_fus <= 1.5 * e_eag + 1e-2, (step, e_fus, e_eag)
        # the fused decode launch on the stream path's logits: proposer (top-K of the last
        # prefix's rows) + every agent row's log-prob of every proposal in ONE launch
        A, K = P - 1, 8
        lg = model.lm_head(fus.hidden)
        ids, U, _, _, _ = ops.beam_decode_step(lg[A * B:], lg[:A * B],
                                               torch.zeros(A, B, device=dev), K, "min",
                                               n_order=B, softcap=eng.softcap)
        tgt = ids.repeat(A, 1)                                        # row a * B + b
        lp32 = e32.rows_logprobs(ref.next_hidden[:A * B], tgt).view(A, B * K)
        lp_e = eng.rows_logprobs(eag.next_hidden[:A * B], tgt).view(A, B * K)
        e_dec = float((U - lp32).abs().max())
        e_eag = float((lp_e - lp32).abs().max())
        print(f"{name} {cfg.n_layers} layers, {P * B} rows: per-step max |dlp| (stream, "
              f"torch bf16) {[(round(a, 4), round(b, 4)) for a, b in worst]}; fused decode "
              f"{e_dec:.4f} vs torch bf16 {e_eag:.4f}")
        assert e_dec <= 1.5 * e_eag + 1e-2, (e_dec, e_eag)
        # the proposals are the bf16 reference rows' own top-K (ties broken by id)
        ref_rows = lg[A * B:].float()
        want = ref_rows.topk(K, dim=1).values
        got = ref_rows.gather(1, ids.long())
        assert torch.equal(got, want)
        fus.release()
    finally:
        del eng, e32, model, m32
        _free()
