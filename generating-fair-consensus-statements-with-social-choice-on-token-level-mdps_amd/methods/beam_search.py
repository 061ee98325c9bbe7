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

Decode state: bf16 models run engine.DecodeState (static per-stream K/V, the prefix
shared by a prefix's beams through cs_prefix_attention, one captured hipGraph per
step); other models the eager engine.BeamState.  With proposer="topk" on one rank the
whole step after the host walk is ONE graph replay: parents' histories, the forward of
the new tokens, the LM head, the reference rows' logit bias and the fused
cs_beam_decode_step (proposer + agent scoring + welfare + stable order) — then one
device->host copy of (ids, order, W, U) for the walk.
Under torchrun over several ranks the agents are sharded (parallel.method_shard): each
rank holds its agents' prefix K/V and beam streams (plus the reference prompt's), scores
its agents, and the candidates' min welfare is an all-reduce(MIN) before the same stable
order on every rank; rank 0's proposals are used everywhere.
"""
from __future__ import annotations

import logging
import os
import time
from typing import List, Optional, Tuple

import numpy as np
import torch

from .. import ops, parallel, runtime
from ..engine import BeamState, DecodeState
from .base import BaseGenerator
from .prompts import BEAM, opinions_text

logger = logging.getLogger(__name__)


class _LiveBeams:
    """DecodeState seen through the BeamState interface.  The state always holds
    beam_width streams per prefix (n_beams); the first n_live are the reference's beams,
    the rest padded copies whose candidates the loop drops.  The LM head runs once per
    step over every stream (the shape the fast top-K step uses, so both loops see
    bit-identical logits)."""

    def __init__(self, st: DecodeState):
        self.st = st
        self.e = st.e
        self.n_live = 1                   # step 0: every stream holds the prefix's last hidden
        self._logits = None

    @property
    def n_beams(self) -> int:
        return self.st.B

    def _all(self) -> torch.Tensor:
        if self._logits is None:
            self._logits = self.e.model.lm_head(self.st.hidden)
        return self._logits

    def next_logits(self, prefix_idx: int) -> torch.Tensor:
        B = self.st.B
        return self._all()[prefix_idx * B:(prefix_idx + 1) * B]

    def agent_logits(self, n_prefix: int) -> torch.Tensor:
        return self._all()[:n_prefix * self.st.B]

    def advance(self, parent, tokens) -> None:
        n = len(parent)
        pad = self.st.B - n
        self.st.advance(list(parent) + [parent[0]] * pad, list(tokens) + [tokens[0]] * pad)
        self.n_live = n
        self._logits = None


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
        self.fused_decode = c.get("fused_decode", True)
        self.fast_topk = c.get("fast_topk", True)
        # fast top-K loop: queue the next step before walking this one (redone on a miss)
        self.speculate = c.get("speculative_steps",
                               os.environ.get("CS_SPECULATIVE_STEPS", "1") != "0")
        # test hook: treat every n-th step's speculation as a miss (rewind + redo)
        self._force_miss = int(c.get("speculative_force_miss", 0))
        # how a candidate's log-prob is read with a tokenizer that is not merge-free (BPE):
        # "text" (default) = the reference's re-tokenized prompt + statement + token, last
        # log-prob (beam_search.py:358-390), candidates whose re-tokenization differs from
        # the id append scored on the text; "ids" = the log-prob of the appended token id
        # (standard token-level beam search; every step one captured graph)
        self.retokenize = c.get("retokenize", "text")
        if self.retokenize not in ("text", "ids"):
            raise ValueError("retokenize must be 'text' or 'ids'")
        self.text_compat_candidates = 0
        self.text_rows_candidates = 0
        # text path on the stream state: candidates whose re-tokenization changes only their
        # last token are scored from rows the decode already has (False: every unstable
        # candidate re-encoded as the reference's whole prompt)
        self.text_incremental = c.get("text_incremental", True)
        self.step_log: List[dict] = []
        self.decode_path = None
        self.steps_run = 0
        self.step_times: List[float] = []     # perf_counter at the start of every step
        self.prefill_s = 0.0

    # --- candidate proposal ------------------------------------------------------
    def _propose(self, st, ref_idx: int, bias: List[int], step_base_seed: Optional[int],
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

    # --- the reference's walk over the sorted candidates (beam_search.py:562-600) -------
    def _walk(self, order, seq_of, tok_str_of, rewards_of, completed):
        """order: candidate indices in (min reward desc, index asc) order.  Returns the new
        beams [(seq, rewards)] and their candidate indices; EOS candidates go to
        ``completed`` (every one of them, as in the reference, which walks all of them)."""
        new_beams, new_idx, seen = [], [], set()
        for i in order:
            seq = seq_of(i)
            if seq in seen:
                continue
            if tok_str_of(i) in self.LLAMA3_EOS_TOKENS:
                completed.append((seq, rewards_of(i)))
            elif len(new_beams) < self.beam_width:
                new_beams.append((seq, rewards_of(i)))
                new_idx.append(i)
                seen.add(seq)
        return new_beams, new_idx

    # --- main loop -----------------------------------------------------------------
    def generate_statement(self, issue: str, agent_opinions: dict) -> str:
        A = len(agent_opinions)
        if A == 0:
            return ""
        engine, tok = runtime.get_engine(self.model_identifier)
        with runtime.device_lock(engine.device):
            return self._generate(engine, tok, issue, agent_opinions)

    def _generate(self, engine, tok, issue: str, agent_opinions: dict) -> str:
        A = len(agent_opinions)
        shard = parallel.method_shard(A, self.config)
        ops_all = list(agent_opinions.values())
        agent_prefixes = [tok.chat_prefix(BEAM["agent_system"],
                                          BEAM["agent_user"].format(issue=issue, opinion=ops_all[a]))
                          for a in shard.local]
        A_loc = len(agent_prefixes)      # this rank's agents (all of them on one rank)
        ref_user = BEAM["ref_user"].format(issue=issue, opinions_text=opinions_text(agent_opinions))
        ref_prefix = tok.render_raw(f"{BEAM['ref_system']}\n\n{ref_user}")
        all_prefixes = agent_prefixes + [ref_prefix]
        # the agents' user prompts (text): the reference re-tokenizes prompt + statement +
        # token on every call; candidates whose id-level append differs from that
        # (tokenizers that are not merge-free) are scored on the text (_text_compat_patch)
        self._agent_users = [BEAM["agent_user"].format(issue=issue, opinion=ops_all[a])
                             for a in shard.local]
        bias = (runtime.bias_token_ids(tok, self.bias_against_tokens)
                if self.use_token_biasing and self.bias_against_tokens else [])
        fused = (self.fused_decode and int(self.max_tokens) > 0 and int(self.beam_width) > 0
                 and engine.model.fused_ok())
        t0 = time.perf_counter()
        # the stream decode prefills in length buckets into ragged K/V (the reference prompt
        # lists every opinion and is many times longer than an agent prompt)
        cache = engine.prefill_streams(all_prefixes) if fused else engine.prefill(all_prefixes)
        self.prefill_s = time.perf_counter() - t0     # host-side (asynchronous launches)
        self.step_times = []
        self.step_log = []
        self.steps_run = 0
        merge_free = getattr(tok, "merge_free", True) or self.retokenize == "ids"
        self._merge_free = merge_free
        self.text_compat_candidates = 0
        self.text_rows_candidates = 0
        if fused and self.proposer == "topk" and self.fast_topk and merge_free:
            self.decode_path = "fused-topk" if shard.world == 1 else "fused-topk-sharded"
            ds = DecodeState(engine, cache, n_prefix=A_loc + 1, n_beams=int(self.beam_width),
                             max_steps=int(self.max_tokens))
            try:
                completed, beams = self._loop_fused_topk(engine, tok, ds, A_loc, bias, shard)
            finally:
                ds.release()
        else:
            ds = None
            if fused:
                self.decode_path = "fused"
                ds = DecodeState(engine, cache, n_prefix=A_loc + 1, n_beams=int(self.beam_width),
                                 max_steps=int(self.max_tokens))
                st = _LiveBeams(ds)
            else:
                self.decode_path = "eager"
                st = BeamState(engine, cache, n_prefix=A_loc + 1)
            try:
                completed, beams = self._loop(engine, tok, st, A, A_loc, shard, bias)
            finally:
                if ds is not None:
                    ds.release()
        return self._final(completed, beams, engine.device, A_loc, shard)

    def _loop(self, engine, tok, st, A, A_loc, shard, bias):
        """Per-step proposals on the host (sample / top-k / sharded), cs_beam_step scoring."""
        dev = engine.device
        beams: List[Tuple[str, List[float]]] = [("", [0.0] * A_loc)]
        beam_ids: List[List[int]] = [[]]           # each beam's token ids as the streams hold them
        rewards = torch.zeros(A_loc, st.n_beams, dtype=torch.float32, device=dev)   # per beam
        completed: List[Tuple[str, List[float]]] = []
        # the re-tokenized text path on the stream state: every step's final hidden of every
        # stream and each beam's ancestry, so a candidate whose re-tokenization only changes
        # its last token is scored from the row of the context it keeps (no forward)
        inc = None
        if (not self._merge_free and isinstance(st, _LiveBeams) and self.text_incremental):
            inc = {"h0": st.st.hidden.clone(), "hid_log": [], "anc": [[]], "B": st.n_beams}
        for step in range(self.max_tokens):
            if not beams:
                break
            self.steps_run += 1
            self.step_times.append(time.perf_counter())
            step_base_seed = (self.seed + step * self.max_sampling_attempts * len(beams) * (A + 1)
                              if self.seed is not None else None)
            n_live = getattr(st, "n_live", st.n_beams)
            props = parallel.same_on_all_ranks(self._propose(st, A_loc, bias, step_base_seed, tok),
                                               shard)
            props = props[:n_live] + [[] for _ in range(st.n_beams - n_live)]   # padded beams
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
            tstr = [tok.token_str(v) for v in ct]
            if not self._merge_free:
                U, W, order = self._text_compat_patch(engine, tok, U, W, order, rewards, cb, ct,
                                                      tstr, beams, beam_ids, shard, inc)
            Uh = U.double().cpu().numpy()
            new_beams, new_idx = self._walk(order, lambda i: beams[cb[i]][0] + tstr[i],
                                            lambda i: tstr[i], lambda i: Uh[:, i].tolist(),
                                            completed)
            par_t = torch.as_tensor(cb, dtype=torch.long, device=dev)
            self.step_log.append({"candidates": [(beams[b][0] + s) for b, s in zip(cb, tstr)],
                                  "min_rewards": W.double().cpu().tolist(),
                                  # this rank's agents' log-prob of each candidate's token
                                  "increments": (U - rewards[:, par_t]).double().cpu().tolist(),
                                  "kept": [s for s, _ in new_beams]})
            beams = new_beams
            beam_ids = [beam_ids[cb[i]] + [ct[i]] for i in new_idx]
            if not beams:
                break
            if step + 1 < self.max_tokens:
                st.advance([cb[i] for i in new_idx], [ct[i] for i in new_idx])
                keep = new_idx + [new_idx[0]] * (st.n_beams - len(new_idx))   # padded beams
                rewards = U[:, torch.as_tensor(keep, device=dev)].contiguous()
                if inc is not None:
                    inc["hid_log"].append(st.st.hidden.clone())
                    inc["anc"] = [inc["anc"][cb[i]] + [j] for j, i in enumerate(new_idx)]
        return completed, beams

    def _text_compat_patch(self, engine, tok, U, W, order, rewards, cb, ct, tstr, beams,
                           beam_ids, shard, inc=None):
        """Tokenizers that are not merge-free (BPE): the reference scores a candidate as the
        last log-prob of the re-tokenized ``agent_user + statement + token``
        (_get_agent_token_logprob, beam_search.py:335-404 via get_prompt_logprobs).  The
        id-level score equals it only when that re-tokenization is the stream's ids plus the
        candidate's id and the token strings spell the text; every other candidate (a merge
        across the append, a byte fragment, a beam that already diverged) is scored on the
        text in one batched pass, and the welfare and order are recomputed."""
        from .. import utils
        tail = BEAM["agent_user"].rsplit("\n\n", 1)[-1]
        tail_ids = tok.encode(tail)
        nt = len(tail_ids)
        bad = []
        texts = [beams[b][0] + tstr[i] for i, b in enumerate(cb)]
        apis = [t + utils.MARKER if t.endswith(("\n", " ")) else t for t in texts]
        many = getattr(tok, "encode_many", None)
        encs = many([tail + a for a in apis]) if many is not None else \
            [tok.encode(tail + a) for a in apis]
        for i, (b, v) in enumerate(zip(cb, ct)):
            ids = beam_ids[b] + [v]
            enc = encs[i]
            if (enc[:nt] != tail_ids or enc[nt:nt + len(ids)] != ids
                    or "".join(tok.tokens(ids)) != texts[i]):
                bad.append(i)
        if not bad:
            return U, W, order
        A_loc = U.shape[0]
        dev = U.device
        U = U.clone()
        self.text_compat_candidates += len(bad)
        rest = bad
        if inc is not None and A_loc:
            rest = self._text_rows(engine, U, rewards, cb, encs, nt, tail_ids, apis, texts,
                                   beam_ids, bad, inc)
        if rest:
            # agent a's user text of candidate i is agent_user[a] + beam text + token: each
            # (agent, beam) prompt re-tokenized once, each candidate's tail once
            lps = utils.text_compat_last_stems(engine, tok, BEAM["agent_system"], self._agent_users,
                                               [s for s, _ in beams], [cb[i] for i in rest],
                                               [tstr[i] for i in rest])
            bi = torch.as_tensor(rest, dtype=torch.long, device=dev)
            par = torch.as_tensor([cb[i] for i in rest], dtype=torch.long, device=dev)
            lp = torch.as_tensor(lps, dtype=torch.float32, device=dev).view(A_loc, len(rest))
            U[:, bi] = rewards[:, par] + lp
        W = parallel.combine_welfare(U, "min", shard)
        order = ops.topk(W, U.shape[1])[0].cpu().tolist()
        return U, W, order

    def _text_rows(self, engine, U, rewards, cb, encs, nt, tail_ids, apis, texts, beam_ids,
                   bad, inc):
        """The text path's common case without any forward: when the re-tokenized user text
        keeps the first j ids of the beam and then ends in ONE token t (a merge of the
        appended token into the last ones: " the" + "ir" -> " their"), the reference's
        last log-prob is log p(t | agent prompt + beam ids[:j]) -- a row the stream decode
        already computed (the prefix's last hidden for j = 0, else the hidden the beam's
        ancestor stream had after its j-th token).  All such candidates of a step share
        one LM head over their distinct (agent, beam, j) rows and one
        cs_logsoftmax_gather.  Returns the candidates left for the full text path
        (re-tokenizations that change two or more tokens, marker texts)."""
        dev = U.device
        A_loc = U.shape[0]
        B = inc["B"]
        groups, rest = {}, []
        for i in bad:
            enc = encs[i]
            if apis[i] != texts[i] or enc[:nt] != tail_ids:
                rest.append(i)
                continue
            suf, bid = enc[nt:], beam_ids[cb[i]]
            j = 0
            n = min(len(suf), len(bid))
            while j < n and suf[j] == bid[j]:
                j += 1
            if len(suf) - j != 1:
                rest.append(i)
                continue
            groups.setdefault((cb[i], j), []).append((i, suf[-1]))
        if not groups:
            return rest
        keys = list(groups)
        rows = []
        for b, j in keys:
            if j == 0:
                src, sidx = inc["h0"], [a * B for a in range(A_loc)]
            else:
                src = inc["hid_log"][j - 1]
                sidx = [a * B + inc["anc"][b][j - 1] for a in range(A_loc)]
            rows.append(src[torch.as_tensor(sidx, dtype=torch.long, device=dev)])   # [A_loc, d]
        H = torch.stack(rows, dim=1).reshape(A_loc * len(keys), -1)            # row a, key g
        kmax = max(len(v) for v in groups.values())
        tgt = torch.full((len(keys), kmax), -1, dtype=torch.int32)
        for g, key in enumerate(keys):
            tgt[g, :len(groups[key])] = torch.as_tensor([t for _, t in groups[key]], dtype=torch.int32)
        lp = engine.rows_logprobs(H, tgt.to(dev).repeat(A_loc, 1)).view(A_loc, len(keys), kmax)
        cand, par, col = [], [], []
        for g, key in enumerate(keys):
            for k, (i, _t) in enumerate(groups[key]):
                cand.append(i)
                par.append(key[0])
                col.append(g * kmax + k)
        ci = torch.as_tensor(cand, dtype=torch.long, device=dev)
        U[:, ci] = rewards[:, torch.as_tensor(par, dtype=torch.long, device=dev)] + \
            lp.reshape(A_loc, -1)[:, torch.as_tensor(col, dtype=torch.long, device=dev)]
        self.text_rows_candidates += len(cand)
        return rest

    def _loop_fused_topk(self, engine, tok, st: DecodeState, A: int, bias, shard=None):
        """Top-K proposer: after the host walk a decode step is one graph replay ending in
        cs_beam_decode_step on one rank; with the agents sharded over ranks it is the
        step graph (advance + LM head + cs_vocab_topk), rank 0's proposals broadcast, a
        scoring graph (cs_beam_step, no order), the MIN all-reduce of the welfare and a
        selection graph (cs_beam_select: stable order of every candidate) -- the two
        exchanges on the stream between graph replays -- or, when the direct RCCL
        communicator's collectives are capturable (parallel.StepComm.capturable), all of it
        inside the step graph.  One device->host copy per step."""
        dev = engine.device
        m = engine.model
        B, K = st.B, int(self.top_k)
        C = B * K
        if K > m.cfg.vocab:
            raise ValueError("top_k exceeds the vocabulary")
        sharded = shard is not None and shard.world > 1
        bias_t = torch.as_tensor(bias, dtype=torch.long, device=dev) if bias else None
        bias_v = float(self.bias_value)
        U_buf = torch.empty(A, C, dtype=torch.float32, device=dev)
        W_buf = torch.empty(C, dtype=torch.float32, device=dev)
        rewards = torch.zeros(A, B, dtype=torch.float32, device=dev)
        kidx = torch.zeros(B, dtype=torch.long, device=dev)
        kidx_h = torch.zeros(B, dtype=torch.long, pin_memory=True)   # read back every step first
        ids_buf = torch.empty(B, K, dtype=torch.int32, device=dev)
        order_buf = torch.empty(C, dtype=torch.int32, device=dev)
        ws = ops.Workspace(zeroed=True)
        # every output the host reads is a persistent buffer: the captured step graphs
        # (ping-pong parities) must write to the same storage
        P = st.P
        p_base = torch.arange(P, device=dev)[:, None] * B

        def spec_inputs():
            # the next step's inputs as the walk will most often choose them: the B best
            # candidates of this step's order (no duplicate text or EOS among them); the
            # host overwrites them whenever its walk differs
            k_s = order_buf[:B].long()
            kidx.copy_(k_s)
            st.src.copy_((p_base + torch.div(k_s, K, rounding_mode="floor")[None, :]).reshape(-1))
            st.tok.copy_(ids_buf.view(-1)[k_s].repeat(P))

        if not sharded:
            def score():
                logits = m.lm_head(st.hidden)                                # [(A + 1) * B, V]
                ref = logits[A * B:]
                if bias_t is not None:
                    ref.index_add_(1, bias_t, torch.full((B, bias_t.numel()), bias_v,
                                                         dtype=ref.dtype, device=dev))
                ops.beam_decode_step(ref, logits[:A * B], rewards, K, "min", n_order=C,
                                     softcap=engine.softcap, workspace=ws, out_U=U_buf,
                                     out_W=W_buf, out_ids=ids_buf, out_order=order_buf)

            def post():
                torch.index_select(U_buf, 1, kidx, out=rewards)
                score()
                if spec:
                    spec_inputs()

            def first_step():
                score()

            def launch(host=None):
                if host is None:
                    st.advance_device(post=post)
                else:
                    st.advance(*host, post=post)
        else:
            comm = parallel.StepComm(shard)
            V = m.cfg.vocab
            lg_buf = torch.empty(P * B, V, dtype=m.dtype, device=dev)
            ws_p = ops.Workspace()
            Wx = torch.empty(C, dtype=torch.float32, device=dev)
            # the score / select graphs live on the DecodeState, so ds.release() frees them
            # with the step graphs (not whenever the cyclic collector reaches this frame)
            graphs = st._graphs

            def propose():                     # in the step graph: LM head + proposer
                m.lm_head(st.hidden, out=lg_buf)
                ref = lg_buf[A * B:]
                if bias_t is not None:
                    ref.index_add_(1, bias_t, torch.full((B, bias_t.numel()), bias_v,
                                                         dtype=ref.dtype, device=dev))
                ids, _ = ops.vocab_topk(ref, K, softcap=engine.softcap, workspace=ws_p)
                ids_buf.copy_(ids)

            def post():
                torch.index_select(U_buf, 1, kidx, out=rewards)
                propose()

            def score_w():                     # this rank's agents, no order
                if A:
                    ops.beam_step(lg_buf[:A * B], ids_buf, rewards, "min", n_order=0,
                                  softcap=engine.softcap, workspace=ws, out_U=U_buf, out_W=Wx)
                    # a column with no usable utility here must not win the MIN all-reduce
                    Wx.nan_to_num_(nan=float("inf"))
                else:
                    Wx.fill_(float("inf"))

            def select():                      # after the all-reduce: the stable order
                if C <= 1024:
                    order, _ = ops.beam_select(Wx, C, unfill="min", W_out=W_buf)
                else:
                    W_buf.copy_(torch.where(torch.isinf(Wx) & (Wx > 0),
                                            torch.full_like(Wx, float("nan")), Wx))
                    order, _ = ops.topk(W_buf, C, with_values=False)
                order_buf.copy_(order)
                if spec:
                    spec_inputs()

            def replay(name, fn):
                name = ("sharded", name)
                g = graphs.get(name)
                if g is None and st.use_graphs and st.steps >= 2:
                    g = torch.cuda.CUDAGraph()
                    cs = torch.cuda.Stream(device=dev)
                    cs.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(cs):
                        with torch.cuda.graph(g, stream=cs):
                            fn()
                    torch.cuda.current_stream().wait_stream(cs)
                    graphs[name] = g
                if g is None:
                    fn()                       # warm-up steps run eagerly
                else:
                    g.replay()

            def exchange_and_select():
                comm.bcast0(ids_buf)           # rank 0's proposals on every rank
                replay("score", score_w)
                comm.min_(Wx)                  # welfare over every agent
                replay("select", select)

            if comm.capturable:
                # the collectives record into the step graph: a sharded step (forward, LM
                # head, proposer, broadcast, scoring, MIN all-reduce, selection) is ONE
                # replay, no host call between its parts
                def exchange_in_graph():
                    comm.bcast0(ids_buf)
                    score_w()
                    comm.min_(Wx)
                    select()

                def post():
                    torch.index_select(U_buf, 1, kidx, out=rewards)
                    propose()
                    exchange_in_graph()

                def first_step():
                    propose()
                    exchange_in_graph()

                def launch(host=None):
                    if host is None:
                        st.advance_device(post=post)
                    else:
                        st.advance(*host, post=post)
                self.decode_path = "fused-topk-sharded-graph"
            else:
                def first_step():
                    propose()
                    exchange_and_select()

                def launch(host=None):
                    if host is None:
                        st.advance_device(post=post)
                    else:
                        st.advance(*host, post=post)
                    exchange_and_select()

        # speculative steps: the next step is queued from the device-side order before the
        # host has walked this one, and redone (rewind + host inputs) when the walk differs
        spec = bool(self.speculate) and st.use_graphs
        self.spec_hits = self.spec_misses = 0
        first_step()                              # step 0 (eager): every beam = the prefix
        hosts = (_HostCopy(), _HostCopy())
        pending = hosts[0].start(ids_buf, order_buf, W_buf, U_buf)
        nxt = None                                # the queued speculative step's results
        beams: List[Tuple[str, List[float]]] = [("", [0.0] * A)]
        n_live = 1
        completed: List[Tuple[str, List[float]]] = []
        for step in range(self.max_tokens):
            self.steps_run += 1
            # queue step + 1 now when this step's beams will most likely be its B best
            # candidates (every beam live; the inputs are written on the device); the GPU
            # runs it while the host walks this step
            if spec and step >= 1 and n_live == B and step + 1 < self.max_tokens:
                launch()
                nxt = hosts[(step + 1) & 1].start(ids_buf, order_buf, W_buf, U_buf)
            else:
                nxt = None
            ids_h, order_h, W_h, U_h = pending.wait()
            self.step_times.append(time.perf_counter())   # this step's results are on the host
            ids_f = ids_h.reshape(-1)
            live = order_h[order_h < n_live * K]                          # beams b < n_live
            tstr = {}

            def ts(i):
                s = tstr.get(i)
                if s is None:
                    s = tstr[i] = tok.token_str(int(ids_f[i]))
                return s

            new_beams, new_idx = self._walk_fast(live, beams, K, ts, U_h, completed,
                                                 ids_f, tok)
            self.step_log.append(_StepRecord([s for s, _ in new_beams], beams, ids_f.copy(),
                                             W_h[:n_live * K].copy(), n_live * K, K, tok))
            beams = new_beams
            if not beams or step + 1 >= self.max_tokens:
                break
            n = len(new_idx)
            kept = new_idx + [new_idx[0]] * (B - n)
            forced = self._force_miss > 0 and step % self._force_miss == 0
            if nxt is not None and n == B and new_idx == order_h[:B].tolist() and not forced:
                self.spec_hits += 1               # the queued step is this walk's step
                pending = nxt
            else:
                if nxt is not None:
                    self.spec_misses += 1
                    st.rewind()
                    # post() of the redo reads this step's U: restore it from the host copy
                    U_buf.copy_(pending.outs[3], non_blocking=True)
                kidx_h.numpy()[:] = kept    # its last copy finished before this step's results
                kidx.copy_(kidx_h, non_blocking=True)
                launch(([i // K for i in kept], [int(ids_f[i]) for i in kept]))
                pending = hosts[(step + 1) & 1].start(ids_buf, order_buf, W_buf, U_buf)
            n_live = n
        return completed, beams

    def _walk_fast(self, order, beams, K, ts, U_h, completed, ids=None, tok=None):
        """The reference walk (beam_search.py:562-600) over a full candidate order: once
        beam_width beams are kept only EOS candidates still matter, and only they are
        visited (found by token id through a per-generator id -> is-EOS cache, without
        building the other candidates' strings)."""
        new_beams, new_idx, seen = [], [], set()
        eos = self.LLAMA3_EOS_TOKENS
        rest = None
        if ids is not None:
            ido = np.asarray(ids)[order]
            flags = self._eos_flags(ido, tok)
        order = order.tolist()
        for pos, i in enumerate(order):
            if ids is not None and len(new_beams) >= self.beam_width:
                rest = [order[p] for p in (np.nonzero(flags[pos:])[0] + pos).tolist()]
                break
            s = ts(i)
            is_eos = s in eos
            if len(new_beams) >= self.beam_width and not is_eos:
                continue
            seq = beams[i // K][0] + s
            if seq in seen:
                continue
            if is_eos:
                completed.append((seq, U_h[:, i].astype(np.float64).tolist()))
            else:
                new_beams.append((seq, U_h[:, i].astype(np.float64).tolist()))
                new_idx.append(i)
                seen.add(seq)
        for i in rest or ():      # the EOS candidates after the kept beams, in order
            seq = beams[i // K][0] + ts(i)
            if seq not in seen:
                completed.append((seq, U_h[:, i].astype(np.float64).tolist()))
        return new_beams, new_idx

    def _eos_flags(self, ids: np.ndarray, tok) -> np.ndarray:
        """Whether each token id's string is an EOS string, from a per-generator table
        filled on first sight of an id."""
        tab = self.__dict__.get("_eos_tab")
        top = int(ids.max()) + 1 if ids.size else 0
        if tab is None or tab.shape[0] < top:
            grown = np.full(max(top, 1024), -1, dtype=np.int8)
            if tab is not None:
                grown[:tab.shape[0]] = tab
            tab = self._eos_tab = grown
        f = tab[ids]
        for v in np.unique(ids[f < 0]).tolist():
            tab[v] = 1 if tok.token_str(int(v)) in self.LLAMA3_EOS_TOKENS else 0
        return tab[ids] == 1

    def _final(self, completed, beams, dev, A_loc, shard) -> str:
        completed = completed + beams
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


class _StepRecord(dict):
    """One step of the fast loop's log: "kept" now; "candidates" (every live candidate's
    text) and "min_rewards" built on first access — building them for all B*K candidates
    every step was a third of the host time of a C3 step."""

    def __init__(self, kept, beams, ids, W, n, K, tok):
        super().__init__(kept=kept)
        self._src = (beams, ids, W, n, K, tok)

    def __missing__(self, key):
        beams, ids, W, n, K, tok = self._src
        if key == "candidates":
            v = [beams[i // K][0] + tok.token_str(int(ids[i])) for i in range(n)]
        elif key == "min_rewards":
            v = W.astype(np.float64).tolist()
        else:
            raise KeyError(key)
        self[key] = v
        return v


class _HostCopy:
    """Device -> pinned host copies of several tensors, ONE stream synchronisation."""

    def __init__(self):
        self.bufs = {}

    def fetch(self, *ts):
        self.start(*ts)
        torch.cuda.current_stream().synchronize()
        return [o.numpy() for o in self.outs]

    def start(self, *ts):
        """Queue the copies (after everything queued so far) and an event behind them."""
        self.outs = []
        for j, t in enumerate(ts):
            b = self.bufs.get(j)
            if b is None or b.shape != t.shape or b.dtype != t.dtype:
                b = self.bufs[j] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            b.copy_(t, non_blocking=True)
            self.outs.append(b)
        self.ev = torch.cuda.Event()
        self.ev.record()
        return self

    def wait(self):
        self.ev.synchronize()
        return [o.numpy() for o in self.outs]
