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

Stream path (bf16 models, the default there; config ``stream_tree: false`` selects the
general path above): the agents' prompts and the reference prompt are prefilled ONCE per
statement (engine.prefill_streams with room for max_tokens more keys) and the lookahead
tree of every step is decoded level by level under all of them at once
(engine.TokenTree): at depth d one LM head over the frontier nodes' rows of every prefix,
the reference rows' biased seeded draws (cs_vocab_sample) give the children, the agent rows
are gathered at those children (cs_logsoftmax_gather, bf targets per row) -- so a node's
agent log-prob comes from its PARENT's row and the tree needs 1 + b + ... + b^(d-1) rows per
agent, not one per node -- and the children that will be expanded are forwarded as one
segment of streams inheriting their parents' K/V by slot table, without any copy
(cs_hist_rows_update + cs_prefix_attention_rows on the tree's row-layout pool).  The committed token's
K/V are copied from its level-1 stream into every prefix (engine.append_prefix_tokens): no
re-prefill between steps.

Welfare (config ``welfare``): "min" (default; the reference's max-min,
finite_lookahead.py:527), "nash" (sum over agents of log max(u, 1e-9) with
u = exp(mean log-prob), the geometric-mean token probability -- the evaluator's Nash form,
src/evaluation.py:337-349; BASELINE C4) or "utilitarian" (sum of u).
"""
from __future__ import annotations

import logging
import time
from typing import List, Optional, Tuple

import torch

from .. import ops, parallel, runtime
from ..engine import TokenTree, tree_pool
from .base import BaseGenerator
from .prompts import FL, opinions_text

logger = logging.getLogger(__name__)


class _Node:
    __slots__ = ("strs", "ids", "seed", "children", "terminal", "owner", "par_owner", "lp_idx")

    def __init__(self, strs, ids, seed, terminal=False):
        self.strs: List[str] = strs
        self.ids: List[int] = ids
        self.seed: Optional[int] = seed
        self.children: List["_Node"] = []
        self.terminal = terminal
        # stream path: (segment, index) whose hidden predicts this node's children, and the
        # column of this node's agent log-probs
        self.owner: Optional[Tuple[int, int]] = None
        self.par_owner: Optional[Tuple[int, int]] = None
        self.lp_idx = -1


WELFARE = {"min": "min", "egalitarian": "min", "nash": "sumlog", "utilitarian": "sum"}


def _leaf_paths(root: _Node, depth: int) -> List[List[_Node]]:
    """Root-to-leaf node chains in the reference recursion's depth-first order, deduped
    by their strings in order (finite_lookahead.py:271-413)."""
    out: List[List[_Node]] = []

    def dfs(node: _Node, d: int, chain: List[_Node]) -> None:
        for c in node.children:
            ch = chain + [c]
            if c.terminal or d + 1 == depth or not c.children:
                out.append(ch)
            else:
                dfs(c, d + 1, ch)

    if depth > 0:
        dfs(root, 0, [])
    seen, uniq = set(), []
    for ch in out:
        key = tuple(ch[-1].strs)
        if ch[-1].strs and key not in seen:
            seen.add(key)
            uniq.append(ch)
    return uniq


class FiniteLookaheadGenerator(BaseGenerator):
    DEFAULT_REWARD = FL["default_reward"]

    def __init__(self, model_identifier: str, config: dict):
        super().__init__(model_identifier, config)
        logger.setLevel(getattr(logging, str(config.get("log_level", "INFO")).upper(), logging.INFO))
        self.api_delay = config.get("api_delay", 0.1)   # compatibility only
        self.brushup = config.get("brushup", False)
        self.trace: List[dict] = []
        # bench hook: a list to collect (start, end, rows) HIP events of every step's
        # cs_logsoftmax_gather launch over the agent rows (stream path)
        self._lsg_events: Optional[list] = None
        # parity-test hook (None in the product): an object whose draws(frontier, seeds, kid)
        # returns the tree's draws and choose(chains, U, W, b) the committed path, so a
        # replay can teacher-force the stream path onto a reference trace
        self._teacher = None
        # stream path, tokenizers that are not merge-free: "text" (default) = the reference's
        # re-tokenized prompt + statement every step; "ids" = the committed token id appended
        self.retokenize = config.get("retokenize", "text")
        if self.retokenize not in ("text", "ids"):
            raise ValueError("retokenize must be 'text' or 'ids'")

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

    def welfare(self, U: torch.Tensor, shard) -> torch.Tensor:
        """W [R] over ALL agents of the per-(agent, path) mean log-probs U [A_local, R]."""
        kind = WELFARE.get(str(self.config.get("welfare", "min")).lower())
        if kind is None:
            raise ValueError("welfare must be one of min / egalitarian / nash / utilitarian")
        if kind == "min":
            return parallel.combine_welfare(U, "min", shard)
        return parallel.combine_welfare(torch.exp(U), kind, shard, eps=FL["eps"])

    @runtime.serialized()
    def generate_statement(self, issue: str, agent_opinions: dict) -> str:
        cfg = self.config
        bf = cfg.get("branching_factor", 2)
        depth = cfg.get("max_depth", 3)
        max_tokens = cfg.get("max_tokens", 50)
        seed = cfg.get("seed")
        self.trace = []
        self.step_times: List[float] = []
        shard = parallel.method_shard(len(agent_opinions), cfg)
        engine, tok = runtime.get_engine(self.model_identifier)
        self.decode_path = ("stream-tree" if cfg.get("stream_tree", True) and engine.model.fused_ok()
                            and max_tokens > 0 else "eager")
        if self.decode_path == "stream-tree":
            current = self._generate_streams(engine, tok, issue, agent_opinions, bf, depth,
                                             max_tokens, seed, shard)
        else:
            current = self._generate_eager(issue, agent_opinions, bf, depth, max_tokens, seed, shard)
        final = current.strip()
        self.pre_brushup_statement = final
        if self.brushup:
            logger.warning("brushup (a remote LLM rewrite of the ending) is not part of the "
                           "local scoring path; returning the statement unchanged")
        return final

    def _generate_eager(self, issue, agent_opinions, bf, depth, max_tokens, seed, shard) -> str:
        current, count = "", 0
        while count < max_tokens:
            self.step_times.append(time.perf_counter())
            paths = self.tree_paths(issue, agent_opinions, current, bf, depth, seed)
            paths = parallel.same_on_all_ranks(paths, shard)   # seed=None draws differ per rank
            if not paths:
                logger.warning("No valid tree paths generated. Ending generation.")
                break
            U = self.path_rewards(issue, agent_opinions, current, paths, shard)
            W = self.welfare(U, shard)
            best, _ = ops.topk(W, 1)
            b = int(best.item())
            nxt = paths[b][0][0]
            self.trace.append({"paths": [p[0] for p in paths], "best": b,
                               "rewards": parallel.gather_agents(U, shard)[:, b].double().cpu().tolist(),
                               "welfare": W.double().cpu().tolist()})
            if nxt.strip() in ["DONE"]:
                break
            if nxt in FL["stop_tokens"]:
                break
            current = nxt if not current else current + nxt
            count += 1
        return current

    # --- stream path ----------------------------------------------------------------
    def _prompts(self, tok, issue, agent_opinions, shard, current):
        ops_all = list(agent_opinions.values())
        agents = [tok.chat_prefix(FL["agent_system"],
                                  FL["agent_user"].format(issue=issue, opinion=ops_all[a]) + current)
                  for a in shard.local]
        ref_user = FL["ref_user"].format(issue=issue, opinions_text=opinions_text(agent_opinions))
        return agents + [tok.render_raw(f"{FL['ref_system']}\n\n{ref_user}{current}")]

    def _generate_streams(self, engine, tok, issue, agent_opinions, bf, depth, max_tokens, seed,
                          shard) -> str:
        A_loc = len(shard.local)
        bias = runtime.bias_token_ids(tok, FL["bias_against"])
        current, count = "", 0
        ids = self._prompts(tok, issue, agent_opinions, shard, current)
        # the trees' history buffers, reused step to step: sized for the largest tree before
        # the first stream forward packs the decode weights around what is left
        pool = tree_pool(engine, A_loc + 1, bf, depth)
        sp = engine.prefill_streams(ids, reserve=max_tokens)
        self.stream_stats = {"prefills": 1, "appended": 0, "segments": 0, "rows": 0}
        while count < max_tokens:
            self.step_times.append(time.perf_counter())
            if depth <= 0 or bf <= 0:
                logger.warning("No valid tree paths generated. Ending generation.")
                break
            tree = TokenTree(engine, sp, max(depth, 1), pool=pool)
            root, chains, lp = self._stream_tree(engine, tok, tree, A_loc, bf, depth, seed, bias,
                                                 shard)
            if not chains:
                logger.warning("No valid tree paths generated. Ending generation.")
                break
            U = self._stream_rewards(engine, tok, issue, agent_opinions, current, shard, chains, lp)
            W = self.welfare(U, shard)
            best, _ = ops.topk(W, 1)
            b = int(best.item())
            if self._teacher is not None:
                b = self._teacher.choose(chains, U, W, b)
            first = chains[b][0]
            nxt = first.strs[0]
            self.trace.append({"paths": [ch[-1].strs for ch in chains], "best": b,
                               "rewards": parallel.gather_agents(U, shard)[:, b].double().cpu().tolist(),
                               "welfare": W.double().cpu().tolist()})
            if nxt.strip() in ["DONE"]:
                break
            if nxt in FL["stop_tokens"]:
                break
            current = nxt if not current else current + nxt
            count += 1
            if count >= max_tokens:
                break
            if nxt == "":
                continue                   # an end-of-sequence draw adds no token
            # the committed token's K/V: its level-1 stream under every prefix (forwarded now
            # when the tree did not expand it: depth 1 or a terminal token)
            if first.owner is None:
                first.owner = (tree.forward(-1, [0], [first.ids[0]]), 0)
            seg, j = first.owner
            # the reference re-tokenizes the grown prompts (retokenize "text", default); with a
            # tokenizer that is not merge-free the id append can differ from that, and then the
            # prompts are encoded afresh; retokenize "ids" appends the committed token's id
            # (the token-level MDP; what the bench times, as for beam search)
            want = [i + [first.ids[0]] for i in ids] if self.retokenize == "ids" else \
                self._prompts(tok, issue, agent_opinions, shard, current)
            if getattr(tok, "merge_free", True) or all(w == i + [first.ids[0]] for w, i in zip(want, ids)):
                tree.append_to_prefix(seg, j)
                self.stream_stats["appended"] += 1
            else:
                # the re-tokenized prompts differ from the id append (a BPE merge across
                # the boundary): encode them afresh, as the reference does every step
                sp = engine.prefill_streams(want, reserve=max_tokens - count)
                self.stream_stats["prefills"] += 1
            ids = want
            del tree
        return current

    def _stream_tree(self, engine, tok, tree: TokenTree, A_loc, bf, depth, seed, bias, shard):
        """The lookahead tree of one step (same draws, seeds and order as tree_paths) and
        every non-empty node's agent log-prob: (root, deduped leaf chains, lp [A_loc, n]).
        Depth d: one LM head over the frontier's rows under every prefix; the reference rows'
        draws; the agent rows gathered at the children; the expanded children forwarded."""
        dev = engine.device
        m = engine.model
        P, ref = A_loc + 1, A_loc
        eos = set(tok.eos_ids)
        terminal = set(FL["terminal_tokens"])
        root = _Node([], [], seed)
        root.owner = (-1, 0)
        frontier = [root]
        blocks, base = [], 0
        # the agent rows of every depth go to ONE logits block and ONE cs_logsoftmax_gather
        # launch after the tree is built (the gathers need only the drawn ids), when the
        # block's bound (frontier <= b^d nodes at depth d) fits 8 GB
        V = m.cfg.vocab
        bound = A_loc * sum(bf ** d for d in range(depth))
        esz = torch.finfo(m.dtype).bits // 8
        defer = A_loc > 0 and bound * V * esz <= (8 << 30)
        lg_all = torch.empty(bound, V, dtype=m.dtype, device=dev) if defer else None
        tg_all, sizes, row0 = [], [], 0
        for d in range(depth):
            if not frontier:
                break
            F = len(frontier)
            H = torch.empty(P, F, m.cfg.d_model, dtype=m.dtype, device=dev)
            by_seg = {}
            for r, n in enumerate(frontier):
                by_seg.setdefault(n.owner[0], []).append(r)
            for sg, rows in by_seg.items():
                H[:, rows] = tree.hidden(sg, [frontier[r].owner[1] for r in rows])
            ref_lg = runtime.apply_bias(m.lm_head(H[ref]).float(), bias, FL["bias_value"])
            if A_loc:
                ha = H[:A_loc].reshape(A_loc * F, -1)
                agent_lg = m.lm_head(ha, out=lg_all[row0:row0 + A_loc * F]) if defer else \
                    m.lm_head(ha)
            seeds = []
            for n in frontier:
                seeds.append([runtime.to_i64(runtime.draw_seed(
                    n.seed + i * (depth + 1) if n.seed is not None else runtime.fresh_seed(), 0))
                    for i in range(bf)])
            sd = torch.tensor(seeds, dtype=torch.int64, device=dev)
            kid, _ = ops.vocab_sample(ref_lg, sd, temperature=1.0, softcap=engine.softcap)
            kid = parallel.broadcast_from_rank0(kid.contiguous(), shard)   # one tree on every rank
            if self._teacher is not None:
                kid = self._teacher.draws(frontier, bf, depth, kid)
            if A_loc:
                if defer:
                    tg_all.append(kid.repeat(A_loc, 1))
                    sizes.append(F)
                    row0 += A_loc * F
                else:
                    lp, _ = ops.logsoftmax_gather(agent_lg, kid.repeat(A_loc, 1),
                                                  softcap=engine.softcap, workspace=engine.ws)
                    blocks.append(lp.view(A_loc, F * bf))
            self.stream_stats["rows"] += P * F
            kid_h = kid.cpu().tolist()
            nxt: List[_Node] = []
            for r, (n, row) in enumerate(zip(frontier, kid_h)):
                for i, v in enumerate(row):
                    s = (n.seed + i * (depth + 1)) if n.seed is not None else None
                    text = "" if v in eos else tok.token_str(v)   # stop tokens are dropped
                    ch = _Node(n.strs + [text], n.ids + ([] if text == "" else [v]),
                               (s + 1) if s is not None else None, terminal=text in terminal)
                    ch.lp_idx = base + r * bf + i
                    ch.par_owner = n.owner
                    if text == "":
                        ch.owner = n.owner          # no token: the parent's stream
                    n.children.append(ch)
                    if not ch.terminal:
                        nxt.append(ch)
            base += F * bf
            if d + 1 < depth:
                # forward the children that carry a new token, one segment per parent segment
                groups = {}
                for ch in nxt:
                    if ch.owner is None:
                        groups.setdefault(ch.par_owner[0], []).append(ch)
                for sg, chs in groups.items():
                    new = tree.forward(sg, [c_.par_owner[1] for c_ in chs],
                                       [c_.ids[-1] for c_ in chs])
                    self.stream_stats["segments"] += 1
                    for j, c_ in enumerate(chs):
                        c_.owner = (new, j)
            frontier = nxt
        if defer and row0:
            ev = self._lsg_events
            tg = torch.cat(tg_all, 0)
            if ev is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            lp, _ = ops.logsoftmax_gather(lg_all[:row0], tg, softcap=engine.softcap,
                                          workspace=engine.ws)
            if ev is not None:
                e1.record()
                ev.append((e0, e1, row0))
                self._lsg_last = (lg_all[:row0], tg)   # the bench re-times this launch
            r = 0
            for F in sizes:
                blocks.append(lp[r:r + A_loc * F].view(A_loc, F * bf))
                r += A_loc * F
        del lg_all
        lp_all = torch.cat(blocks, dim=1) if blocks else \
            torch.empty(A_loc, 0, dtype=torch.float32, device=dev)
        return root, _leaf_paths(root, depth), lp_all

    def _stream_rewards(self, engine, tok, issue, agent_opinions, current, shard, chains, lp):
        """U [A_local, R]: each path's mean over its nodes' agent log-probs; an empty element
        (an end-of-sequence draw) takes one more log-prob from the end of the prompt, as the
        reference's last-len(path) slice does (finite_lookahead.py:508-520)."""
        dev = engine.device
        A = lp.shape[0]
        R = len(chains)
        if A == 0:
            return torch.empty(0, R, dtype=torch.float32, device=dev)
        flat, offs = [], [0]
        extra = []
        for ch in chains:
            cols = [n.lp_idx for n in ch if n.strs[-1] != ""]
            flat.append(cols)
            extra.append(len(ch) - len(cols))
        idx = [c for cols in flat for c in cols]
        sel = lp[:, torch.as_tensor(idx, dtype=torch.long, device=dev)].contiguous() if idx else \
            torch.empty(A, 0, dtype=torch.float32, device=dev)
        for a in range(A):
            for cols in flat:
                offs.append(offs[-1] + len(cols))
        seg = ops.segment_reduce(sel.reshape(-1), torch.as_tensor(offs, dtype=torch.int32, device=dev))
        sums = seg["sum_lp"].view(A, R).double()
        cnt = seg["count"].view(A, R).double()
        mx = max(extra)
        if mx > 0:
            # the prompt's last tokens' log-probs (rare: only trees with an end-of-sequence
            # draw): one plain prefill of the agents' prompts
            pre = self._prompts(tok, issue, agent_opinions, shard, current)[:-1]
            tail = engine.prefix_tail_logprobs(engine.prefill(pre), mx).double()
            for p, e in enumerate(extra):
                if e > 0:
                    sums[:, p] += tail[:, mx - e:].sum(dim=1)
                    cnt[:, p] += e
        return (sums / cnt).to(torch.float32).contiguous()
