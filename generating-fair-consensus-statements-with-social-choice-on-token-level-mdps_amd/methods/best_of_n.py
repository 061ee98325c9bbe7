"""Best-of-N with egalitarian welfare on the local engine (src/methods/best_of_n.py).

Reference flow (best_of_n.py:53-207), same config keys and outputs:
  1. N candidates from the reference policy: generate_text(chat, max_tokens,
     temperature, seed + i) (:104-136)  ->  one batched seeded generation of N streams
     sharing the reference prompt's prefix K/V (runtime.generate, cs_vocab_sample).
  2. Per (candidate, agent): mean log-prob of the candidate under
     system = agent_system + "\\n\\n" + agent_user(issue, opinion), user = candidate
     (:266-321)  ->  all A x N continuations in one batched scoring pass:
     per-agent prefix K/V, LM head, cs_logsoftmax_gather, cs_segment_reduce.
  3. nan_to_num(nan -> -10, +inf -> 20, -inf -> -20), min over agents (:384-408)
     -> cs_welfare_reduce(MIN, REPLACE);  np.argmax (:198) -> cs_segmented_topk(k=1).
Under torchrun (one process per GPU, default process group over several ranks) the agents
are sharded (parallel.method_shard): each rank scores its agents x all candidates and the
welfare is combined with an all-reduce(MIN); every rank returns the same statement.
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional

import torch

from .. import ops, parallel, runtime, utils
from .base import BaseGenerator
from .prompts import BON, opinions_text

logger = logging.getLogger(__name__)


def clean_generated_text(text: str) -> str:
    """strip; drop one known instruction prefix (case-insensitive); drop trailing EOS
    strings (src/methods/best_of_n.py:209-238)."""
    if not text:
        return ""
    out = text.strip()
    low = out.lower()
    for p in BON["clean_prefixes"]:
        if low.startswith(p.lower()):
            out = out[low.find(p.lower()) + len(p):].strip()
            break
    for eos in BON["eos_tokens"]:
        if out.endswith(eos):
            out = out[: -len(eos)].strip()
    return out


class BestOfNGenerator(BaseGenerator):
    DEFAULT_REWARD = BON["default_reward"]
    REWARD_CLIP_MIN = BON["clip_min"]
    REWARD_CLIP_MAX = BON["clip_max"]

    def __init__(self, model_identifier: str, config: dict):
        super().__init__(model_identifier, config)
        logger.setLevel(getattr(logging, str(config.get("log_level", "INFO")).upper(), logging.INFO))
        self.api_delay = config.get("api_delay", 0.1)  # accepted for compatibility; no remote calls
        self.last_candidates: List[str] = []
        self.last_agent_rewards: Dict[str, List[float]] = {}
        self.last_welfare: List[float] = []

    @runtime.serialized()
    def generate_statement(self, issue: str, agent_opinions: dict) -> str:
        cfg = self.config
        n = cfg.get("num_best_of_n", cfg.get("n", 3))
        max_tokens = cfg.get("max_tokens", 50)
        seed = cfg.get("seed")
        temperature = cfg.get("temperature", 1.0)
        engine, tok = runtime.get_engine(self.model_identifier)

        ref_user = BON["ref_user"].format(issue=issue, opinions_text=opinions_text(agent_opinions))
        ref_ids, _ = tok.render_chat(BON["ref_system"], ref_user)
        seeds = [seed + i if seed is not None else None for i in range(n)]
        outs = runtime.generate(engine, tok, ref_ids, seeds, max_tokens, float(temperature))
        cands = [c for c in (clean_generated_text(tok.decode(o)) for o in outs) if c]
        shard = parallel.method_shard(len(agent_opinions), cfg)
        cands = parallel.same_on_all_ranks(cands, shard)   # seed=None draws differ per rank
        self.last_candidates = cands
        if not cands:
            logger.error("No valid candidate statements were generated.")
            return "[ERROR: Failed to generate any candidates]"

        U = self.score_candidates(issue, agent_opinions, cands, shard)   # [A_local, N] device
        W = parallel.combine_welfare(U, "min", shard, nonfinite="replace",
                                     nan_val=self.DEFAULT_REWARD, posinf_val=self.REWARD_CLIP_MAX,
                                     neginf_val=self.REWARD_CLIP_MIN)
        best, _ = ops.topk(W, 1)
        b = int(best.item())
        self.last_welfare = W.double().cpu().tolist()
        logger.info("Selected best candidate index: %d (Score: %.4f)", b, self.last_welfare[b])
        return cands[b]

    def score_candidates(self, issue: str, agent_opinions: dict, cands: List[str],
                         shard: Optional[parallel.AgentShard] = None) -> torch.Tensor:
        """Mean log-prob utility U[a, c] of every candidate under every agent of this
        rank's shard (all agents on one rank; device, fp32, rows in agent order)."""
        engine, tok = runtime.get_engine(self.model_identifier)
        shard = shard or parallel.AgentShard(len(agent_opinions))
        ops_all = list(agent_opinions.values())
        mine = [ops_all[a] for a in shard.local]
        C = len(cands)
        if not mine:   # more ranks than agents: nothing to score here
            U = torch.empty(0, C, dtype=torch.float32, device=engine.device)
            self._record_rewards(agent_opinions, U, shard)
            return U
        prefixes = []
        for op in mine:
            system = BON["agent_system"] + "\n\n" + BON["agent_user"].format(issue=issue, opinion=op)
            prefixes.append(tok.chat_prefix(system, ""))
        cache = engine.prefill(prefixes)
        A = len(prefixes)
        cand_ids = [tok.encode(c) for c in cands]
        owner = [a for a in range(A) for _ in range(C)]
        conts = [cand_ids[c] for _ in range(A) for c in range(C)]
        lp = engine.score(cache, owner, conts)
        seg = ops.segment_reduce(lp, engine.offsets(conts, engine.device))
        cnt = seg["count"].to(torch.float32)
        U = torch.where(cnt > 0, seg["sum_lp"] / cnt.clamp(min=1.0),
                        torch.full_like(cnt, self.DEFAULT_REWARD)).view(A, C)
        # candidates the reference's find() would locate inside the prompt: text-compat path
        for a, op in enumerate(mine):
            system = BON["agent_system"] + "\n\n" + BON["agent_user"].format(issue=issue, opinion=op)
            for c, cand in enumerate(cands):
                where = utils.span_check(tok, system, cand)
                if where == utils.SPAN_NONE:          # the reference's call returns ([], [])
                    U[a, c] = self.DEFAULT_REWARD
                elif where == utils.SPAN_ELSEWHERE:
                    m_lp, _, n_ok = utils.text_compat_mean(self.model_identifier, system, cand)
                    U[a, c] = m_lp if n_ok else self.DEFAULT_REWARD
        U = U.contiguous()
        self._record_rewards(agent_opinions, U, shard)
        return U

    def _record_rewards(self, agent_opinions: dict, U: torch.Tensor, shard) -> None:
        """last_agent_rewards for every agent (gathered from the ranks when sharded)."""
        allU = parallel.gather_agents(U, shard)
        self.last_agent_rewards = {aid: allU[i].double().cpu().tolist()
                                   for i, aid in enumerate(agent_opinions)}
