"""Finite lookahead on the local engine (src/methods/finite_lookahead.py).

Per committed token (finite_lookahead.py:99-153):
  1. Lookahead tree from the reference policy (raw completions prompt), branching
     factor b, depth d, one seeded one-token draw per (node, branch) with the
     reference's seed schedule gen_seed = path_seed + i*(d+1), child path_seed =
     gen_seed + 1 (:297-301, 375-377); terminal tokens end a path (:350-355);
     paths listed in the recursion's depth-first order, order-preserving dedupe
     (:402-413).  Here: one level at a time, every node of a level in one batched
     forward and one cs_vocab_sample launch (b draws per node row).
  2. For every (path, agent): mean of the last len(path) user-span log-probs of
     agent_user + statement + path (:490-520); best path = first max of the min over
     agents (:527).  Here: the paths form a token tree; every tree node is scored ONCE
     per agent (engine.score_tree: one extend over the internal nodes with a tree
     attention mask, one logits row per node, cs_logsoftmax_gather), each path's
     log-probs are its nodes' (cs_segment_reduce over the path -> node lists), then
     cs_welfare_reduce(MIN), cs_segmented_topk(k=1).  A depth-d, branching-b tree needs
     b + ... + b^d rows per agent instead of d * b^d.
  3. Commit the best path's first token; stop on "DONE" / newline tokens (:141-144).

Under torchrun over several ranks the agents are sharded (parallel.method_shard): each
rank scores its agents' rows of the tree, the welfare is an all-reduce(MIN), and rank 0's
lookahead paths are used everywhere.

Reference quirk kept: a one-token draw that hits an end-of-sequence token returns
"" (generate_text drops stop tokens), so a path element can be empty; the reward
then still averages the last len(path) log-probs of the user span, reaching back
into the statement/template tokens (prefix_tail_logprobs).
"""
from __future__ import annotations

import logging
from typing import List, Optional, Tuple

import torch

from .. import ops, parallel, runtime
from .base import BaseGenerator
from .prompts import FL, opinions_text

logger = logging.getLogger(__name__)


class _Node:
    __slots__ = ("strs", "ids", "seed", "children", "terminal")

    def __init__(self, strs, ids, seed, terminal=False):
        self.strs: List[str] = strs
        self.ids: List[int] = ids
        self.seed: Optional[int] = seed
        self.children: List["_Node"] = []
        self.terminal = terminal


class FiniteLookaheadGenerator(BaseGenerator):
    DEFAULT_REWARD = FL["default_reward"]

    def __init__(self, model_identifier: str, config: dict):
        super().__init__(model_identifier, config)
        logger.setLevel(getattr(logging, str(config.get("log_level", "INFO")).upper(), logging.INFO))
        self.api_delay = config.get("api_delay", 0.1)   # compatibility only
        self.brushup = config.get("brushup", False)
        self.trace: List[dict] = []

    # --- tree ---------------------------------------------------------------------
    def tree_paths(self, issue: str, agent_opinions: dict, current: str, bf: int, depth: int,
                   seed: Optional[int]) -> List[Tuple[List[str], List[int]]]:
        engine, tok = runtime.get_engine(self.model_identifier)
        ref_user = FL["ref_user"].format(issue=issue, opinions_text=opinions_text(agent_opinions))
        prompt = tok.render_raw(f"{FL['ref_system']}\n\n{ref_user}{current}")
        cache = engine.prefill([prompt])
        bias = runtime.bias_token_ids(tok, FL["bias_against"])
        eos = set(tok.eos_ids)
        terminal = set(FL["terminal_tokens"])
        root = _Node([], [], seed)
        frontier = [root]
        for _level in range(depth):
            if not frontier or bf <= 0:
                break
            h = engine.next_hidden(cache, [0] * len(frontier), [n.ids for n in frontier])
            logits = runtime.apply_bias(engine.model.lm_head(h).float(), bias, FL["bias_value"])
            seeds = []
            for n in frontier:
                row = []
                for i in range(bf):
                    s = n.seed + i * (depth + 1) if n.seed is not None else runtime.fresh_seed()
                    row.append(runtime.to_i64(runtime.draw_seed(s, 0)))
                seeds.append(row)
            sd = torch.tensor(seeds, dtype=torch.int64, device=engine.device)
            ids, _ = ops.vocab_sample(logits, sd, temperature=1.0, softcap=engine.softcap)
            ids = ids.cpu().tolist()
            nxt = []
            for n, row_ids, row_seeds in zip(frontier, ids, seeds):
                for i, v in enumerate(row_ids):
                    s = (n.seed + i * (depth + 1)) if n.seed is not None else None
                    text = "" if v in eos else tok.token_str(v)   # stop tokens are dropped
                    child = _Node(n.strs + [text], n.ids + ([] if text == "" else [v]),
                                  (s + 1) if s is not None else None, terminal=text in terminal)
                    n.children.append(child)
                    if not child.terminal:
                        nxt.append(child)
            frontier = nxt
        leaves: List[_Node] = []

        def dfs(node: _Node, d: int) -> None:
            for c in node.children:
                if c.terminal or d + 1 == depth or not c.children:
                    leaves.append(c)
                else:
                    dfs(c, d + 1)

        if depth == 0:
            return []
        dfs(root, 0)
        seen, uniq = set(), []
        for lf in leaves:
            key = tuple(lf.strs)
            if lf.strs and key not in seen:
                seen.add(key)
                uniq.append((lf.strs, lf.ids))
        return uniq

    # --- scoring ------------------------------------------------------------------
    def path_rewards(self, issue: str, agent_opinions: dict, current: str,
                     paths: List[Tuple[List[str], List[int]]],
                     shard: Optional[parallel.AgentShard] = None) -> torch.Tensor:
        """U[a, p] = mean of the last len(path) user-span log-probs (device fp32), for the
        agents of this rank's shard (every agent on one rank), rows in agent order."""
        engine, tok = runtime.get_engine(self.model_identifier)
        shard = shard or parallel.AgentShard(len(agent_opinions))
        ops_all = list(agent_opinions.values())
        prefixes = [tok.chat_prefix(FL["agent_system"],
                                    FL["agent_user"].format(issue=issue, opinion=ops_all[a]) + current)
                    for a in shard.local]
        A, R = len(prefixes), len(paths)
        if A == 0:   # more ranks than agents
            return torch.empty(0, R, dtype=torch.float32, device=engine.device)
        cache = engine.prefill(prefixes)
        # the paths form a token tree: every node is scored once per agent (shared
        # prefixes of the lookahead paths are not re-scored), then each path's log-probs
        # are its nodes'
        node_of, tokens, parents, path_nodes = {}, [], [], []
        for _strs, ids in paths:
            cur, lst = -1, []
            for t in range(len(ids)):
                key = tuple(ids[:t + 1])
                if key not in node_of:
                    node_of[key] = len(tokens)
                    tokens.append(ids[t])
                    parents.append(cur)
                cur = node_of[key]
                lst.append(cur)
            path_nodes.append(lst)
        dev = engine.device
        node_lp = engine.score_tree(cache, list(range(A)), tokens, parents)   # [A, N]
        flat = [n for lst in path_nodes for n in lst]
        total = len(flat)
        lp = node_lp[:, torch.as_tensor(flat, dtype=torch.long, device=dev)].contiguous()
        offs = [0]
        for a in range(A):
            for lst in path_nodes:
                offs.append(offs[-1] + len(lst))
        seg = ops.segment_reduce(lp.reshape(-1), torch.as_tensor(offs, dtype=torch.int32,
                                                                  device=dev))
        assert offs[-1] == A * total
        sums = seg["sum_lp"].view(A, R).double()
        cnt = seg["count"].view(A, R).double()
        # empty path elements: the last len(path) span log-probs reach into the prefix
        extra = [len(s) - len(i) for s, i in paths]
        m = max(extra) if extra else 0
        if m > 0:
            tail = engine.prefix_tail_logprobs(cache, m).double()        # [A, m]
            for p, e in enumerate(extra):
                if e > 0:
                    sums[:, p] += tail[:, m - e:].sum(dim=1)
                    cnt[:, p] += e
        return (sums / cnt).to(torch.float32).contiguous()

    @runtime.serialized()
    def generate_statement(self, issue: str, agent_opinions: dict) -> str:
        cfg = self.config
        bf = cfg.get("branching_factor", 2)
        depth = cfg.get("max_depth", 3)
        max_tokens = cfg.get("max_tokens", 50)
        seed = cfg.get("seed")
        current, count = "", 0
        self.trace = []
        shard = parallel.method_shard(len(agent_opinions), cfg)
        while count < max_tokens:
            paths = self.tree_paths(issue, agent_opinions, current, bf, depth, seed)
            paths = parallel.same_on_all_ranks(paths, shard)   # seed=None draws differ per rank
            if not paths:
                logger.warning("No valid tree paths generated. Ending generation.")
                break
            U = self.path_rewards(issue, agent_opinions, current, paths, shard)
            W = parallel.combine_welfare(U, "min", shard)
            best, _ = ops.topk(W, 1)
            b = int(best.item())
            nxt = paths[b][0][0]
            self.trace.append({"paths": [p[0] for p in paths], "best": b,
                               "rewards": parallel.gather_agents(U, shard)[:, b].double().cpu().tolist()})
            if nxt.strip() in ["DONE"]:
                break
            if nxt in FL["stop_tokens"]:
                break
            current = nxt if not current else current + nxt
            count += 1
        final = current.strip()
        self.pre_brushup_statement = final
        if self.brushup:
            logger.warning("brushup (a remote LLM rewrite of the ending) is not part of the "
                           "local scoring path; returning the statement unchanged")
        return final
