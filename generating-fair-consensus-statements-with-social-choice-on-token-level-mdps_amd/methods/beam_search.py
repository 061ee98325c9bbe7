"""Egalitarian beam search on the local engine (src/methods/beam_search.py).

Reference step (beam_search.py:439-617), same config keys:
  * per beam, up to beam_width unique next tokens sampled from the reference prompt
    (raw completions prompt, logit bias, seeds step_base_seed + beam + attempt,
    :199-333, 444-482)  ->  proposer="sample" (default): all beams' reference rows in
    one cs_vocab_sample launch, max_sampling_attempts draws per row, first
    beam_width unique in draw order.  proposer="topk": the deterministic top-K
    tokens per beam (cs_vocab_topk), K = config "top_k" (BASELINE configs).
  * per (beam, token, agent): log p(token | agent prompt + beam) (:335-404,
    495-538), cumulative agent rewards and the stable sort by min over agents
    (:534-560)  ->  ONE logits row per (agent, beam) from the incremental beam state
    and ONE cs_beam_step launch: stream every row, gather every candidate token of
    its beam, U = R + lp, min over agents, stable order over all B*K candidates.
  * dedupe / EOS / keep beam_width walk (:562-600) and final >= 5-word filter +
    selection (:619-667): host logic over the kernel's order, as in the reference.
Under torchrun over several ranks the agents are sharded (parallel.method_shard): each
rank holds its agents' prefix K/V and beam streams (plus the reference prompt's), scores
its agents, and the candidates' min welfare is an all-reduce(MIN) before the same stable
order on every rank; rank 0's proposals are used everywhere.
"""
from __future__ import annotations

import logging
from typing import List, Optional, Tuple

import torch

from .. import ops, parallel, runtime
from ..engine import BeamState
from .base import BaseGenerator
from .prompts import BEAM, opinions_text

logger = logging.getLogger(__name__)


class BeamSearchGenerator(BaseGenerator):
    LLAMA3_EOS_TOKENS = BEAM["eos_tokens"]
    BIAS_AGAINST_TOKENS = BEAM["bias_against"]
    DEFAULT_BIAS_VALUE = BEAM["bias_value"]

    def __init__(self, model_identifier: str, config: dict):
        super().__init__(model_identifier, config)
        logger.setLevel(getattr(logging, str(config.get("log_level", "INFO")).upper(), logging.INFO))
        c = self.config
        self.beam_width = c.get("beam_width", 3)
        self.max_tokens = c.get("max_tokens", 50)
        self.api_delay = c.get("api_delay", 0.1)      # compatibility only
        self.seed = c.get("seed")
        self.max_sampling_attempts = c.get("max_sampling_attempts", self.beam_width)
        self.beta = c.get("beta", 1.0)
        self.brushup = c.get("brushup", False)
        self.use_token_biasing = c.get("use_token_biasing", True)
        self.bias_value = c.get("bias_value", self.DEFAULT_BIAS_VALUE)
        self.bias_against_tokens = list(c.get("bias_against_tokens", self.BIAS_AGAINST_TOKENS))
        if "additional_bias_tokens" in c:
            self.bias_against_tokens.extend(c["additional_bias_tokens"])
        self.proposer = c.get("proposer", "sample")
        self.top_k = c.get("top_k", self.beam_width)
        self.step_log: List[dict] = []

    # --- candidate proposal ------------------------------------------------------
    def _propose(self, st: BeamState, ref_idx: int, bias: List[int], step_base_seed: Optional[int],
                 tok) -> List[List[int]]:
        logits = st.next_logits(ref_idx).float()
        if bias:
            logits = runtime.apply_bias(logits, bias, float(self.bias_value))
        B = st.n_beams
        if self.proposer == "topk":
            ids, _ = ops.vocab_topk(logits, int(self.top_k), softcap=st.e.softcap)
            return ids.cpu().tolist()
        n_att = int(self.max_sampling_attempts)
        if n_att <= 0:
            return [[] for _ in range(B)]
        seeds = []
        for b in range(B):
            base = (step_base_seed + b) if step_base_seed is not None else None
            seeds.append([runtime.to_i64(runtime.draw_seed(base + a if base is not None else runtime.fresh_seed(), 0))
                          for a in range(1, n_att + 1)])
        out: List[List[int]] = []
        for a0 in range(0, n_att, 16):   # at most 16 draws per launch
            sd = torch.tensor([r[a0:a0 + 16] for r in seeds], dtype=torch.int64,
                              device=st.e.device)
            ids, _ = ops.vocab_sample(logits, sd, temperature=1.0, softcap=st.e.softcap)
            part = ids.cpu().tolist()
            out = part if not out else [o + p for o, p in zip(out, part)]
        uniq = []
        for row in out:
            got: List[int] = []
            seen = set()
            for v in row:
                s = tok.token_str(v)
                if s not in seen:
                    seen.add(s)
                    got.append(v)
                    if len(got) >= self.beam_width:
                        break
            uniq.append(got)
        return uniq

    # --- main loop -----------------------------------------------------------------
    def generate_statement(self, issue: str, agent_opinions: dict) -> str:
        A = len(agent_opinions)
        if A == 0:
            return ""
        engine, tok = runtime.get_engine(self.model_identifier)
        shard = parallel.method_shard(A, self.config)
        ops_all = list(agent_opinions.values())
        agent_prefixes = [tok.chat_prefix(BEAM["agent_system"],
                                          BEAM["agent_user"].format(issue=issue, opinion=ops_all[a]))
                          for a in shard.local]
        A_loc = len(agent_prefixes)      # this rank's agents (all of them on one rank)
        ref_user = BEAM["ref_user"].format(issue=issue, opinions_text=opinions_text(agent_opinions))
        ref_prefix = tok.render_raw(f"{BEAM['ref_system']}\n\n{ref_user}")
        cache = engine.prefill(agent_prefixes + [ref_prefix])
        st = BeamState(engine, cache, n_prefix=A_loc + 1)
        bias = (runtime.bias_token_ids(tok, self.bias_against_tokens)
                if self.use_token_biasing and self.bias_against_tokens else [])
        dev = engine.device

        beams: List[Tuple[str, List[float]]] = [("", [0.0] * A_loc)]
        rewards = torch.zeros(A_loc, 1, dtype=torch.float32, device=dev)   # cumulative, per beam
        completed: List[Tuple[str, List[float]]] = []
        self.step_log = []
        for step in range(self.max_tokens):
            if not beams:
                break
            step_base_seed = (self.seed + step * self.max_sampling_attempts * len(beams) * (A + 1)
                              if self.seed is not None else None)
            props = parallel.same_on_all_ranks(self._propose(st, A_loc, bias, step_base_seed, tok),
                                               shard)
            cb, ct = [], []                           # candidate (beam, token id), insertion order
            for b, toks in enumerate(props):
                for v in toks:
                    cb.append(b)
                    ct.append(v)
            if not cb:
                break
            K = max(len(t) for t in props)
            tgt = torch.full((st.n_beams, K), -1, dtype=torch.int32)   # -1 = padded slot
            for b, toks in enumerate(props):
                if toks:
                    tgt[b, :len(toks)] = torch.as_tensor(toks, dtype=torch.int32)
            pos_in_beam, cnt = [], {}
            for b in cb:
                pos_in_beam.append(cnt.get(b, 0))
                cnt[b] = cnt.get(b, 0) + 1
            slots = [b * K + k for b, k in zip(cb, pos_in_beam)]
            # agent rows -> lp at every candidate, U = R + lp, min over agents, stable
            # order over the B*K slots (padded slots are NaN: ranked after every real one,
            # so the order of the real candidates is the reference's stable sort)
            slot_t = torch.as_tensor(slots, dtype=torch.long, device=dev)
            if shard.world == 1:
                Up, Wp, order, _ = ops.beam_step(st.agent_logits(A), tgt.to(dev), rewards, "min",
                                                 softcap=st.e.softcap, workspace=st.e.beam_ws)
                U = Up[:, slot_t].contiguous()                                # [A, n_cand]
                W = Wp[slot_t]
                cand_of = {s: i for i, s in enumerate(slots)}
                order = [cand_of[c] for c in order.cpu().tolist() if c in cand_of]
            else:
                # this rank's agents (no order in the launch), min over ALL agents by an
                # all-reduce, then the same stable order on every rank
                if A_loc:
                    Up, _, _, _ = ops.beam_step(st.agent_logits(A_loc), tgt.to(dev), rewards, "min",
                                                n_order=0, softcap=st.e.softcap,
                                                workspace=st.e.beam_ws)
                    U = Up[:, slot_t].contiguous()                            # [A_loc, n_cand]
                else:
                    U = torch.empty(0, len(slots), dtype=torch.float32, device=dev)
                W = parallel.combine_welfare(U, "min", shard)
                order = ops.topk(W, len(slots))[0].cpu().tolist()
            Uh = U.double().cpu().numpy()
            new_beams, new_idx, seen = [], [], set()
            for i in order:
                b, v = cb[i], ct[i]
                s_tok = tok.token_str(v)
                seq = beams[b][0] + s_tok
                if seq in seen:
                    continue
                r = Uh[:, i].tolist()
                if s_tok in self.LLAMA3_EOS_TOKENS:
                    completed.append((seq, r))
                elif len(new_beams) < self.beam_width:
                    new_beams.append((seq, r))
                    new_idx.append(i)
                    seen.add(seq)
            self.step_log.append({"candidates": [(beams[b][0] + tok.token_str(v)) for b, v in zip(cb, ct)],
                                  "min_rewards": W.double().cpu().tolist(), "kept": [s for s, _ in new_beams]})
            beams = new_beams
            if not beams:
                break
            rewards = U[:, torch.as_tensor(new_idx, device=dev)].contiguous()
            st.advance([cb[i] for i in new_idx], [ct[i] for i in new_idx])

        completed.extend(beams)
        if not completed:
            return ""
        pool = [(s, r) for s, r in completed if len(s.strip().split()) >= 5] or completed
        Uf = torch.tensor([r for _, r in pool], dtype=torch.float32,
                          device=dev).reshape(len(pool), A_loc).t().contiguous()
        Wf = parallel.combine_welfare(Uf, "min", shard)
        best, _ = ops.topk(Wf, 1)
        final = pool[int(best.item())][0].strip()
        self.pre_brushup_statement = final
        if self.brushup:
            logger.warning("brushup (a remote LLM rewrite of the ending) is not part of the "
                           "local scoring path; returning the statement unchanged")
        return final
