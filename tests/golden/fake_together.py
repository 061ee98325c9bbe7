"""Offline stand-in for the `together` client — TEST INFRASTRUCTURE ONLY.

Used by make_method_traces.py to run the reference's own method code (imported
from /root/reference in the build container) against a local model, so that the
reference's control flow (prompts, span extraction, reward folding, selection)
produces golden fixtures.  The model forward here is INDEPENDENT of the product:
Hugging Face transformers (LlamaForCausalLM / Gemma2ForCausalLM) on the CPU in
fp32, loaded with the same seeded weights as the product's model.  Shared
definitions (tokenizer + chat template, seed schedule, counter-based RNG) are the
product's documented conventions; the RNG is oracle.cs_uniform.

Response shapes mirror what the reference parses:
  chat.completions.create(echo=True, logprobs=True) -> .prompt[0].logprobs.{tokens,
      token_logprobs, token_ids} (src/utils.py:262-263, 505-506), first logprob None
  chat.completions.create(...)                      -> .choices[0].message.content
  completions.create(logprobs=1)                    -> .choices[0].text and
      .choices[0].logprobs.{tokens, token_logprobs} (beam_search.py:288-297)
  embeddings.create                                 -> raises (no embeddings offline)
"""
from __future__ import annotations

import math
import os
import sys
from types import SimpleNamespace
from typing import Dict, List, Optional

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402

M64 = (1 << 64) - 1


def draw_seed(seed: int, t: int) -> int:
    """Product convention (runtime.draw_seed): token t of a generation seeded with s."""
    return (int(seed) * 1000003 + int(t)) & M64


class Backend:
    """CPU fp32 transformers model + the product's char tokenizer."""

    def __init__(self, hf_model, tokenizer, softcap: float = 0.0,
                 tail_positions: Optional[int] = None, kv_cache: int = 0):
        """tail_positions: echo log-probs of the prompt's last tail_positions tokens only
        (NaN before them) -- the LM head over a few rows instead of the whole prompt, for
        traces whose recorded calls keep only the span's tail (beam search sums [-1:]).
        kv_cache: keep the K/V of the last kv_cache prompts and run a new prompt's forward
        from the longest cached token prefix (a causal prefix's K/V depend on that prefix
        alone; the forward differs from a full one by fp32 summation order only) -- for
        the wide-model fixtures whose thousands of calls share their long prompts."""
        self.tail = tail_positions
        self.m = hf_model.eval()
        self.tok = tokenizer
        self.softcap = softcap
        self.rng = np.random.default_rng(0)
        self.calls: List[Dict] = []
        self.kv_cache = int(kv_cache)
        self._kv: List = []          # [(ids tuple, DynamicCache)], most recent last
        # every draw of sample(): the Gumbel-max margin (best perturbed score minus the
        # runner-up) -- how far the draw is from a tie, so a bf16 replay that draws another
        # token can be checked to do so only at a near-tie
        self.draw_log: List[Dict] = []
        self.last_margins: List[float] = []

    @torch.no_grad()
    def _forward(self, ids: List[int], keep: int) -> torch.Tensor:
        """logits of the last `keep` positions of `ids` ([keep, V] fp32)."""
        if not self.kv_cache:
            kw = {} if keep == len(ids) else {"logits_to_keep": keep}
            return self.m(torch.tensor([ids]), **kw).logits[0]
        import copy
        from transformers import DynamicCache

        best, blen = None, 0
        for key, cache in self._kv:
            n = 0
            lim = min(len(key), len(ids))
            while n < lim and key[n] == ids[n]:
                n += 1
            if n > blen:
                best, blen = cache, n
        blen = min(blen, len(ids) - keep)
        if best is not None and blen > 0:
            cache = copy.deepcopy(best)
            cache.crop(blen)
        else:
            cache, blen = DynamicCache(), 0
        out = self.m(torch.tensor([ids[blen:]]), past_key_values=cache, use_cache=True,
                     logits_to_keep=keep)
        self._kv.append((tuple(ids), out.past_key_values))
        if len(self._kv) > self.kv_cache:
            self._kv.pop(0)
        return out.logits[0]

    @torch.no_grad()
    def logits(self, ids: List[int], last_only: bool = False) -> np.ndarray:
        """fp32 logits as float64 (softcap applied by HF); last_only: the last position's
        row alone (the LM head over one position instead of the whole prompt)."""
        return self._forward(ids, 1 if last_only else len(ids)).double().numpy()

    @torch.no_grad()
    def prompt_logprobs(self, ids: List[int]) -> List[Optional[float]]:
        """log_softmax(logits)[i, ids[i + 1]] in float64 for every prompt position."""
        P = len(ids)
        K = P if self.tail is None else min(P, int(self.tail) + 1)
        lg = self._forward(ids, K).double()                              # positions P-K .. P-1
        nxt = torch.tensor(ids[P - K + 1:], dtype=torch.long)
        ls = lg[:-1].gather(1, nxt[:, None])[:, 0] - torch.logsumexp(lg[:-1], dim=1)
        return [None] + [float("nan")] * (P - K) + [float(v) for v in ls.tolist()]

    def sample(self, ids: List[int], max_tokens: int, temperature: float, seed: Optional[int],
               bias: Dict[int, float]):
        """Seeded Gumbel-max sampling; returns (ids drawn incl. a final stop id, logprobs)."""
        if seed is None:
            seed = int(self.rng.integers(0, 2**63))
        cur = list(ids)
        drawn, lps = [], []
        self.last_margins = []
        for t in range(max_tokens):
            x = self.logits(cur, last_only=True)[-1].copy()
            for i, v in bias.items():
                x[i] += v
            i, lp = oracle.gumbel_sample(x, draw_seed(seed, t), temperature)
            drawn.append(i)
            lps.append(lp)
            self.last_margins.append(gumbel_margin(x, draw_seed(seed, t), temperature))
            if i in self.tok.eos_ids:
                break
            cur.append(i)
        self.last_drawn = list(drawn)
        return drawn, lps


def gumbel_margin(x: np.ndarray, seed: int, temperature: float) -> float:
    """Top-1 minus top-2 of the perturbed scores x/T + g(seed, v) that gumbel_sample takes
    the argmax of."""
    u = oracle.cs_uniform(seed, np.arange(x.shape[0])).astype(np.float64)
    s = np.asarray(x, dtype=np.float64) / temperature - np.log(-np.log(u))
    top2 = np.partition(s, -2)[-2:]
    return float(top2[1] - top2[0])


_BACKEND: Optional[Backend] = None


def set_backend(b: Backend) -> None:
    global _BACKEND
    _BACKEND = b


def _bias_map(logit_bias) -> Dict[int, float]:
    return {int(k): float(v) for k, v in (logit_bias or {}).items()}


class _ChatCompletions:
    def create(self, model=None, messages=None, max_tokens=16, temperature=1.0, stop=None,
               seed=None, logprobs=False, echo=False, stream=False, logit_bias=None,
               repetition_penalty=1.0, **kw):
        b = _BACKEND
        system = None
        user = ""
        for msg in messages:
            if msg["role"] == "system":
                system = msg["content"]
            elif msg["role"] == "user":
                user = msg["content"]
        ids, _ = b.tok.render_chat(system, user)
        resp = SimpleNamespace(prompt=[], choices=[])
        if echo:
            lps = b.prompt_logprobs(ids)
            resp.prompt = [SimpleNamespace(logprobs=SimpleNamespace(
                tokens=b.tok.tokens(ids), token_logprobs=lps, token_ids=list(ids)))]
            b.calls.append({"kind": "echo", "system": system, "user": user})
            drawn = []
        else:
            drawn, _ = b.sample(ids, max_tokens, temperature, seed, _bias_map(logit_bias))
        text = b.tok.decode([i for i in drawn if i not in b.tok.eos_ids])
        resp.choices = [SimpleNamespace(message=SimpleNamespace(content=text))]
        return resp


class _Completions:
    def create(self, model=None, prompt="", max_tokens=16, temperature=1.0, seed=None,
               logprobs=None, logit_bias=None, stream=False, stop=None, repetition_penalty=1.0,
               **kw):
        b = _BACKEND
        ids = b.tok.render_raw(prompt)
        drawn, lps = b.sample(ids, max_tokens, temperature, seed, _bias_map(logit_bias))
        b.draw_log.append({"prompt": prompt, "seed": seed, "id": drawn[0] if drawn else None,
                           "margin": b.last_margins[0] if b.last_margins else None})
        text = b.tok.decode([i for i in drawn if i not in b.tok.eos_ids])
        lp_ns = SimpleNamespace(tokens=b.tok.tokens(drawn), token_logprobs=lps)
        return SimpleNamespace(choices=[SimpleNamespace(text=text, logprobs=lp_ns)])


class _Embeddings:
    def create(self, model=None, input=None, **kw):
        raise RuntimeError("embeddings are not available offline")


class Together:
    def __init__(self, *a, **k):
        self.chat = SimpleNamespace(completions=_ChatCompletions())
        self.completions = _Completions()
        self.embeddings = _Embeddings()


def hf_model_for(model, cfg):
    """transformers model with the product model's weights (CPU fp32)."""
    from transformers import Gemma2Config, Gemma2ForCausalLM, LlamaConfig, LlamaForCausalLM

    import importlib
    M = importlib.import_module(
        "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.model")
    if cfg.family == "llama3":
        hc = LlamaConfig(vocab_size=cfg.vocab, hidden_size=cfg.d_model, intermediate_size=cfg.d_ff,
                         num_hidden_layers=cfg.n_layers, num_attention_heads=cfg.n_heads,
                         num_key_value_heads=cfg.n_kv_heads, head_dim=cfg.head_dim,
                         rope_theta=cfg.rope_theta, rms_norm_eps=cfg.rms_eps,
                         rope_scaling=dict(rope_type="llama3", **cfg.rope_scaling)
                         if cfg.rope_scaling else None,
                         tie_word_embeddings=cfg.tie_embeddings, max_position_embeddings=131072)
        hf = LlamaForCausalLM(hc)
    else:
        hc = Gemma2Config(vocab_size=cfg.vocab, hidden_size=cfg.d_model, intermediate_size=cfg.d_ff,
                          num_hidden_layers=cfg.n_layers, num_attention_heads=cfg.n_heads,
                          num_key_value_heads=cfg.n_kv_heads, head_dim=cfg.head_dim,
                          rope_theta=cfg.rope_theta, rms_norm_eps=cfg.rms_eps,
                          final_logit_softcapping=cfg.final_softcap,
                          attn_logit_softcapping=cfg.attn_softcap,
                          sliding_window=cfg.sliding_window,
                          query_pre_attn_scalar=int(cfg.query_pre_attn_scalar),
                          hidden_activation="gelu_pytorch_tanh", tie_word_embeddings=True,
                          attn_implementation="eager")
        hf = Gemma2ForCausalLM(hc)
    sd = {k: v.float() for k, v in M.hf_state_dict(model).items()}
    missing = hf.load_state_dict(sd, strict=False)
    assert not missing.missing_keys, missing.missing_keys
    return hf.float()
