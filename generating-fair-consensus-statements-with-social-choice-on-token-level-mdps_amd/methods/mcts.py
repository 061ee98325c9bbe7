"""Monte Carlo tree search with egalitarian rewards on the local engine (src/methods/mcts.py).

Same class name, config keys, tree policy and seed schedule as the reference
(mcts.py:47-1044); every remote call is replaced by a batched engine call:

  * expansion proposals (mcts.py:162-245): up to ``max_sampling_attempts`` one-token
    draws from the raw reference prompt with seeds base+1, base+2, ... until
    ``expansion_sample_width`` distinct tokens are found.  The draws are independent,
    so all of them come from ONE logits row and ONE cs_vocab_sample launch; the
    distinct-token walk over them in attempt order is the reference's loop.
  * immediate reward (mcts.py:730-782): min over agents of the summed user-span
    log-probs of the new token under system = agent_system + "\\n\\n" + agent_user +
    statement (mcts.py:247-320);
  * rollout (mcts.py:470-651): ``rollout_depth`` tokens sampled from the reference
    prompt (runtime.generate, seed = rollout seed), then min over agents of the summed
    log-probs of the rollout text (mcts.py:322-368).
    Both rewards of one simulation are scored in ONE pass (utils.user_span_sums: one
    prefill of the 2A prompts, cs_logsoftmax_gather, cs_segment_reduce) and reduced
    over agents by cs_welfare_reduce(MIN).
  * UCB1 selection over children in token-string order, backpropagation from the
    expanded node, most-visited child advances the root (mcts.py:370-468, 884-930).
Under torchrun over several ranks the agents are sharded (parallel.method_shard): every
rank runs the same search (one run seed drawn on rank 0 when ``seed`` is None) and scores
only its agents' prompts; each reward is an all-reduce(MIN) over the ranks.

Reference defect, documented rather than reproduced: mcts.py:615 formats
``final_statement`` (commented out at :593) in a debug f-string inside the rollout's
agent loop, so every non-empty rollout raises NameError and src/experiment.py:196-201
records the run as "ERROR".  This generator implements the evident intent (score the
rollout); the golden traces come from the reference with that name bound.  Set config
``reference_rollout_nameerror: true`` to raise the reference's NameError instead.
"""
from __future__ import annotations

import logging
import math
import random
from typing import Dict, List, Optional, Tuple

import torch

from .. import ops, parallel, runtime, utils
from .base import BaseGenerator
from .prompts import MCTS, opinions_text

logger = logging.getLogger(__name__)


class Node:
    """Search-tree node (mcts.py:18-44)."""

    __slots__ = ("statement", "parent", "token", "children", "visits", "total_reward", "value",
                 "immediate_reward", "untried_tokens", "is_terminal")

    def __init__(self, statement: str, parent: Optional["Node"] = None,
                 token: Optional[str] = None, is_terminal: bool = False):
        self.statement = statement
        self.parent = parent
        self.token = token
        self.children: Dict[str, "Node"] = {}
        self.visits = 0
        self.total_reward = 0.0
        self.value = 0.0
        self.immediate_reward: Optional[float] = None
        self.untried_tokens: Optional[List[Tuple[str, float]]] = None
        self.is_terminal = is_terminal


class MCTSGenerator(BaseGenerator):
    LLAMA3_EOS_TOKENS = MCTS["eos_tokens"]
    FAIL = MCTS["failure_reward"]

    def __init__(self, model_identifier: str, config: dict):
        super().__init__(model_identifier, config)
        logger.setLevel(getattr(logging, str(config.get("log_level", "INFO")).upper(), logging.INFO))
        self.num_simulations = config.get("num_simulations", 50)
        self.exploration_constant = config.get("exploration_constant", 1.414)
        self.max_tokens = config.get("max_tokens", 100)
        self.api_delay = config.get("api_delay", 0.1)   # compatibility only: no remote calls
        self.seed = config.get("seed")
        self.expansion_sample_width = config.get("expansion_sample_width", 5)
        self.max_sampling_attempts = config.get("max_sampling_attempts",
                                                self.expansion_sample_width * 3)
        self.rollout_depth = config.get("rollout_depth", 10)
        self.gamma = config.get("gamma", 0.99)
        self.brushup = config.get("brushup", False)
        self.strict_nameerror = bool(config.get("reference_rollout_nameerror", False))
        self.trace: List[dict] = []
        self._shard = parallel.AgentShard(0)

    # --- prompts (mcts.py:126-158) -----------------------------------------------------
    def _reference_prompt(self, issue: str, agent_opinions: dict, statement: str) -> str:
        user = MCTS["ref_user"].format(issue=issue, opinions_text=opinions_text(agent_opinions))
        return f"{MCTS['ref_system']}\n\n{user}{statement}"

    def _agent_systems(self, issue: str, agent_opinions: dict, statement: str) -> List[str]:
        """system text of the scoring calls: agent_system + "\\n\\n" + agent_user + statement
        (mcts.py:262, 619-621)."""
        return [f"{MCTS['agent_system']}\n\n" + MCTS["agent_user"].format(issue=issue, opinion=op)
                + statement for op in agent_opinions.values()]

    # --- expansion proposals (mcts.py:162-245) -----------------------------------------
    @torch.no_grad()
    def _sample_next_tokens(self, prompt: str, num_desired: int, max_attempts: int,
                            temperature: float, base_seed: Optional[int]) -> List[Tuple[str, float]]:
        if num_desired <= 0 or max_attempts <= 0:
            return []
        engine, tok = runtime.get_engine(self.model_identifier)
        cache = engine.prefill([tok.render_raw(prompt)])
        row = engine.model.lm_head(cache.last_hidden[:1]).float()
        seeds = [runtime.draw_seed(base_seed + a if base_seed is not None else runtime.fresh_seed(), 0)
                 for a in range(1, max_attempts + 1)]
        per = 16                                        # cs_vocab_sample draws per row
        n_rows = (len(seeds) + per - 1) // per
        pad = n_rows * per - len(seeds)
        sd = torch.tensor([runtime.to_i64(s) for s in seeds] + [0] * pad, dtype=torch.int64,
                          device=engine.device).view(n_rows, per)
        ids, lp = ops.vocab_sample(row.expand(n_rows, -1).contiguous(), sd,
                                   temperature=float(temperature), softcap=engine.softcap)
        ids = ids.view(-1)[:len(seeds)].tolist()
        lp = lp.view(-1)[:len(seeds)].double().tolist()
        collected: Dict[str, float] = {}
        for v, l in zip(ids, lp):           # attempt order; stop once enough are distinct
            if len(collected) >= num_desired:
                break
            s = tok.token_str(v)
            if s not in collected:
                collected[s] = l
        return list(collected.items())

    # --- rewards ------------------------------------------------------------------------
    @torch.no_grad()
    def _rollout_text(self, issue: str, agent_opinions: dict, statement: str, seed: int) -> str:
        engine, tok = runtime.get_engine(self.model_identifier)
        ids = tok.render_raw(self._reference_prompt(issue, agent_opinions, statement))
        out = runtime.generate(engine, tok, ids, [seed], self.rollout_depth, 1.0)[0]
        return tok.decode(out)

    def _evaluate(self, issue: str, agent_opinions: dict, parent_statement: str, token: str,
                  child_statement: str, rollout: Optional[str]) -> Tuple[float, Optional[float]]:
        """(immediate reward, rollout reward or None): each the min over agents of the
        summed user-span log-probs, FAIL when any agent's call fails (mcts.py:742-782,
        611-651)."""
        shard = self._shard
        local = shard.local
        A = len(local)                    # this rank's agents (all of them on one rank)
        cols = 2 if rollout else 1
        par_sys = self._agent_systems(issue, agent_opinions, parent_statement)
        systems = [par_sys[a] for a in local]
        users = [token] * A
        if rollout:
            child_sys = self._agent_systems(issue, agent_opinions, child_statement)
            systems += [child_sys[a] for a in local]
            users += [rollout] * A
        engine, _ = runtime.get_engine(self.model_identifier)
        if A:
            sums = utils.user_span_sums(self.model_identifier, systems, users, device_out=True)
            sums = sums.to(engine.device)
        else:
            sums = torch.empty(0, dtype=torch.float64, device=engine.device)
        U = sums.view(cols, A).t().to(torch.float32).contiguous()       # [A_local, cols]
        W = parallel.combine_welfare(U, "min", shard).double().cpu().tolist()
        bad = parallel.any_rank(torch.isnan(sums).view(cols, A).any(dim=1), shard).cpu().tolist()
        imm = self.FAIL if bad[0] else W[0]
        roll = None
        if rollout:
            roll = self.FAIL if bad[1] else W[1]
        return imm, roll

    # --- tree policy (mcts.py:370-468) --------------------------------------------------
    def _ucb1(self, node: Node, parent_visits: int) -> float:
        if node.visits == 0:
            return float("inf")
        if parent_visits == 0:
            parent_visits = 1
        return node.value + self.exploration_constant * math.sqrt(math.log(parent_visits) / node.visits)

    def _select(self, node: Node) -> Node:
        while not node.is_terminal:
            if node.untried_tokens is None or len(node.untried_tokens) > 0:
                return node
            if not node.children:
                node.is_terminal = True
                return node
            best_child, best_score = None, -float("inf")
            for _token, child in sorted(node.children.items()):
                score = self._ucb1(child, node.visits)
                if score > best_score:
                    best_score, best_child = score, child
                elif score == float("inf") and best_score != float("inf"):
                    best_score, best_child = score, child
            if best_child is None:
                node.is_terminal = True
                return node
            node = best_child
        return node

    def _expand_and_evaluate(self, node: Node, issue: str, agent_opinions: dict,
                             step_seed: Optional[int]) -> float:
        """mcts.py:653-837."""
        reward = self.FAIL
        if node.untried_tokens is None:
            base = (step_seed if step_seed is not None else random.randint(0, 10000)) + node.visits
            node.untried_tokens = self._sample_next_tokens(
                self._reference_prompt(issue, agent_opinions, node.statement),
                self.expansion_sample_width, self.max_sampling_attempts, 1.0, base)
            node.untried_tokens = [t for t in node.untried_tokens if t[0] not in node.children]
        if node.untried_tokens:
            next_token = node.untried_tokens.pop(0)[0]
            new_statement = node.statement + next_token
            child = Node(new_statement, node, next_token,
                         is_terminal=next_token.strip() in self.LLAMA3_EOS_TOKENS)
            node.children[next_token] = child
            A = len(agent_opinions)
            rollout = None
            if not child.is_terminal:
                rseed = ((step_seed if step_seed is not None else random.randint(0, 10000))
                         + node.visits * (A + 1) + 5000)
                rollout = self._rollout_text(issue, agent_opinions, child.statement, rseed)
                if rollout and self.strict_nameerror:
                    raise NameError("name 'final_statement' is not defined")
            imm, roll = self._evaluate(issue, agent_opinions, node.statement, next_token,
                                       child.statement, rollout)
            child.immediate_reward = imm
            if child.is_terminal:
                reward = imm
            else:
                roll = self.FAIL if roll is None else roll   # empty rollout (mcts.py:585-588)
                reward = imm + self.gamma * roll
            return reward
        if not node.children and not node.is_terminal:
            node.is_terminal = True
        return 0.0

    @staticmethod
    def _backpropagate(node: Node, reward: Optional[float]) -> None:
        if reward is None:
            reward = MCTS["failure_reward"]
        cur = node
        while cur is not None:
            cur.visits += 1
            cur.total_reward += reward
            cur.value = cur.total_reward / cur.visits if cur.visits > 0 else 0.0
            cur = cur.parent

    @staticmethod
    def _select_best_child(node: Node) -> Optional[Node]:
        if not node.children:
            return None
        return sorted(node.children.values(), key=lambda c: c.visits, reverse=True)[0]

    # --- main loop (mcts.py:932-1044) ---------------------------------------------------
    @runtime.serialized()
    def generate_statement(self, issue: str, agent_opinions: dict) -> str:
        A = len(agent_opinions)
        self.trace = []
        if A == 0:
            logger.warning("No agent opinions provided.")
            return ""
        self._shard = parallel.method_shard(A, self.config)
        seed_cfg = self.seed
        if self._shard.world > 1 and self.seed is None:   # one search on every rank
            self.seed = parallel.same_on_all_ranks(random.randint(0, 2 ** 30), self._shard)
        try:
            return self._search(issue, agent_opinions)
        finally:
            self.seed = seed_cfg

    def _search(self, issue: str, agent_opinions: dict) -> str:
        A = len(agent_opinions)
        root = Node(statement="")
        current = ""
        for step in range(self.max_tokens):
            if root.is_terminal:
                break
            step_seed = (self.seed + step * self.num_simulations * (A + 1) * 2
                         if self.seed is not None else None)
            for sim in range(self.num_simulations):
                sim_seed = step_seed + sim if step_seed is not None else None
                selected = self._select(root)
                reward = 0.0
                if not selected.is_terminal:
                    reward = self._expand_and_evaluate(selected, issue, agent_opinions, sim_seed)
                self._backpropagate(selected, reward)
            if not root.children:
                logger.warning("Root node has no children after simulations. Stopping.")
                break
            best = self._select_best_child(root)
            if best is None:
                break
            self.trace.append({"visits": {t: c.visits for t, c in root.children.items()},
                               "chosen": best.token})
            current = best.statement
            root = best
            root.parent = None
            if best.token and best.token.strip() in self.LLAMA3_EOS_TOKENS:
                root.is_terminal = True
                break
        final = current.strip()
        self.pre_brushup_statement = final
        if self.brushup:
            logger.warning("brushup (a remote LLM rewrite of the ending) is not part of the "
                           "local scoring path; returning the statement unchanged")
        return final
