"""Drop-in for the reference's LLM access shim (src/utils.py), served locally.

Same function names, arguments, return shapes and failure sentinels as the
reference; the remote Together calls are replaced by the local scoring engine:

  get_prompt_logprobs(model, system_prompt, user_prompt, ...)     src/utils.py:201-281
      chat-template render (with the reference's U+200B marker when the user prompt
      ends in a space or newline, :224-233) -> one forward over the whole prompt ->
      cs_logsoftmax_gather over every prompt position (the echo=True prompt
      log-probs) -> the user span by character overlap (:284-373).
      Never raises: ([], []) on any failure (:274-281).
  extract_user_prompt_logprobs(logprobs_data, user_prompt)         src/utils.py:284-373
  generate_text(...)                                                src/utils.py:77-198
  get_token_ids(model, text)                                        src/utils.py:466-525
  create_method_identifier(...)                                     src/utils.py:19-62

This text-compat path reproduces the reference's string-level semantics exactly
(including its first-occurrence ``find`` of the user prompt).  The methods use the
batched id-level engine instead (engine.py), which scores the true user span.
"""
from __future__ import annotations

import bisect
import itertools
import logging
from types import SimpleNamespace
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import torch

from . import ops
from . import runtime

logger = logging.getLogger(__name__)

MARKER = "\u200b"  # zero-width space appended by src/utils.py:224-233

IMPORTANT_PARAMETERS = ["n", "num_candidates", "num_rounds", "branching_factor", "max_depth",
                        "beam_width"]


def create_method_identifier(method_name: str, params_dict: Optional[Dict[str, Any]] = None,
                             include_seed: bool = False,
                             seed_value: Optional[Union[int, str]] = None) -> str:
    """'name (k=v, ...) [seed=s]' with the important parameters only, sorted (utils.py:19-62)."""
    parts = []
    for key, value in (params_dict or {}).items():
        name = key[len("param_"):] if key.startswith("param_") else key
        if name in IMPORTANT_PARAMETERS and value is not None:
            parts.append(f"{name}={value}")
    ident = f"{method_name} ({', '.join(sorted(parts))})" if parts else method_name
    if include_seed and seed_value is not None:
        ident += f" [seed={seed_value}]"
    return ident


@torch.no_grad()
def prompt_logprobs_ids(model: str, ids: Sequence[int]) -> List[Optional[float]]:
    """log p(ids[i] | ids[:i]) for every position (None for position 0): the echo=True
    prompt log-probs, computed by one forward + cs_logsoftmax_gather."""
    engine, _ = runtime.get_engine(model)
    if len(ids) < 2:
        return [None] * len(ids)
    with runtime.device_lock(engine.device):
        t = torch.as_tensor(list(ids), dtype=torch.long, device=engine.device)[None]
        h = engine.prefill([list(ids)]).hidden          # reuses a stored common prefix
        rows = h[0, :-1]
        tgt = t[0, 1:].to(torch.int32)[:, None]
        lp = engine.rows_logprobs(rows, tgt).view(-1).double().cpu().tolist()
    return [None] + lp


def get_prompt_logprobs(model, system_prompt, user_prompt, temperature=1.0, terminators=(),
                        seed=None) -> Tuple[List[str], List[Optional[float]]]:
    """(user_tokens, user_logprobs) of the user prompt under the chat template."""
    try:
        _, tok = runtime.get_engine(model)
        api_user = user_prompt
        if user_prompt.endswith("\n") or user_prompt.endswith(" "):
            api_user += MARKER
        ids, _ = tok.render_chat(system_prompt or None, api_user)
        lps = prompt_logprobs_ids(model, ids)
        data = SimpleNamespace(tokens=tok.tokens(ids), token_logprobs=lps, token_ids=list(ids))
        return extract_user_prompt_logprobs(data, user_prompt)
    except Exception as e:  # the reference never raises here (src/utils.py:274-281)
        logger.error("get_prompt_logprobs failed: %s", e)
        return [], []


def extract_user_prompt_logprobs(logprobs_data, user_prompt):
    """Tokens whose character span overlaps the first occurrence of ``user_prompt`` in
    the concatenated token strings, with their log-probs (src/utils.py:284-373)."""
    if (not logprobs_data or not hasattr(logprobs_data, "tokens")
            or not hasattr(logprobs_data, "token_logprobs")):
        return [], []
    toks, lps = logprobs_data.tokens, logprobs_data.token_logprobs
    if len(toks) != len(lps):
        return [], []
    text = "".join(toks)
    lo = text.find(user_prompt)
    if lo == -1:
        return [], []
    hi = lo + len(user_prompt)
    keep = []
    pos = 0
    for i, t in enumerate(toks):
        a, b = pos, pos + len(t)
        if max(a, lo) < min(b, hi):
            keep.append(i)
        pos = b
        if a >= hi:
            break
    if not keep:
        return [], []
    return [toks[i] for i in keep], [lps[i] for i in keep]


def last_user_span_index(tokens: Sequence[str], user_prompt: str) -> int:
    """Index of the LAST token ``extract_user_prompt_logprobs`` keeps (the last token whose
    characters overlap the first occurrence of ``user_prompt`` in the joined token
    strings), or -1 when it keeps none — by one C-speed find and a bisect over the tokens'
    end offsets instead of the per-token loop."""
    if not user_prompt:
        return -1
    lo = "".join(tokens).find(user_prompt)
    if lo == -1:
        return -1
    ends = list(itertools.accumulate(map(len, tokens)))
    # the first token ending at or after the span's end: it starts before the end (the
    # first such token has a non-empty string) and is the last one that can overlap
    return bisect.bisect_left(ends, lo + len(user_prompt))


SPAN_AT_USER, SPAN_NONE, SPAN_ELSEWHERE = 1, 0, -1


def _ascii_text_of(tok):
    """tok.chat_text when the tokenizer's ASCII token strings join to the rendered text
    (BPETokenizer.ascii_joins_text, checked once per tokenizer), else None: only then may
    "the rendered ASCII text does not contain the user text" stand for the reference's
    failed ``find`` in the joined token strings."""
    chat_text = getattr(tok, "chat_text", None)
    check = getattr(tok, "ascii_joins_text", None)
    if chat_text is None or check is None or not check():
        return None
    return chat_text


def span_check(tok, system_prompt, user_prompt) -> int:
    """Where the reference's first-occurrence ``find`` of the user prompt lands in the
    rendered prompt's token strings (src/utils.py:321-327): SPAN_AT_USER (the user turn
    itself: the batched engine path holds the reference's value), SPAN_NONE (nowhere: the
    reference's call returns ([], []) and its caller takes its fallback reward -- e.g. a
    candidate with leading whitespace the chat template trims), SPAN_ELSEWHERE (e.g. a
    one-word statement that also occurs in the system text: the text-compat path).
    An ASCII prompt's token strings join to the rendered text itself, so SPAN_NONE is
    decided by one string search there, without encoding."""
    api_user = user_prompt + MARKER if user_prompt.endswith(("\n", " ")) else user_prompt
    chat_text = _ascii_text_of(tok)
    if chat_text is not None:
        text = chat_text(system_prompt or None, api_user, True)
        if text.isascii() and text.find(user_prompt) == -1:
            return SPAN_NONE
    ids, (start, _) = tok.render_chat(system_prompt or None, api_user)
    text = "".join(tok.tokens(ids))
    lo = text.find(user_prompt)
    if lo == -1:
        return SPAN_NONE
    return SPAN_AT_USER if lo == len("".join(tok.tokens(ids[:start]))) else SPAN_ELSEWHERE


def span_found_at_user(tok, system_prompt, user_prompt) -> bool:
    """True when the reference's first-occurrence ``find`` of the user prompt lands on the
    user turn itself (src/utils.py:321-327).  False means the reference scores a span
    elsewhere in the prompt, or none; callers then take the text-compat path."""
    return span_check(tok, system_prompt, user_prompt) == SPAN_AT_USER


def text_compat_mean(model, system_prompt, user_prompt):
    """(mean log-prob, mean prob, count) of the reference's user-span log-probs."""
    _, lps = get_prompt_logprobs(model, system_prompt, user_prompt)
    vals = [v for v in lps if v is not None]
    if not vals:
        return float("nan"), float("nan"), 0
    import math as _m
    return sum(vals) / len(vals), sum(_m.exp(v) for v in vals) / len(vals), len(vals)


@torch.no_grad()
def user_span_sums(model, systems: Sequence[Optional[str]], users: Sequence[str],
                   *, device_out: bool = False):
    """``sum(get_prompt_logprobs(model, systems[i], users[i])[1])`` for every i, batched.

    The reference calls get_prompt_logprobs once per (agent, text) and sums the user-span
    log-probs (src/methods/mcts.py:270-320, 343-368).  Here every pair whose user span is
    where the reference's ``find`` lands (span_found_at_user) is scored in ONE engine pass
    (prefill of the distinct chat prefixes, one logits block, cs_logsoftmax_gather,
    cs_segment_reduce); the rest take the text-compat path.  Returns a float64 tensor
    [n] (on the device when ``device_out`` and every pair took the batched path) with NaN
    where the reference's call yields no usable log-probs (empty span, a None entry).
    """
    engine, tok = runtime.get_engine(model)
    with runtime.device_lock(engine.device):
        return _user_span_sums(engine, tok, systems, users, device_out)


def _user_span_sums(engine, tok, systems, users, device_out):
    n = len(users)
    out = torch.full((n,), float("nan"), dtype=torch.float64)
    where = [span_check(tok, systems[i], users[i]) if users[i] else SPAN_NONE for i in range(n)]
    fast = [i for i in range(n) if where[i] == SPAN_AT_USER]
    if fast:
        keys, owner, uniq = {}, [], []
        for i in fast:
            s = systems[i] or None
            if s not in keys:
                keys[s] = len(uniq)
                uniq.append(tok.chat_prefix(s, ""))
            owner.append(keys[s])
        conts = [tok.encode(users[i]) for i in fast]
        cache = engine.prefill(uniq)
        lp = engine.score(cache, owner, conts)
        seg = ops.segment_reduce(lp, engine.offsets(conts, engine.device))
        ok = seg["count"] == torch.as_tensor([len(c) for c in conts], dtype=torch.int32,
                                             device=engine.device)
        sums = torch.where(ok & (seg["count"] > 0), seg["sum_lp"].double(),
                           torch.full_like(seg["sum_lp"], float("nan"), dtype=torch.float64))
        if device_out and len(fast) == n:
            return sums
        out[torch.as_tensor(fast)] = sums.cpu()
    # SPAN_NONE pairs stay NaN: the reference's call returns ([], [])
    slow = [i for i in range(n) if where[i] == SPAN_ELSEWHERE]
    if slow:
        vals = text_compat_span_sums(engine, tok, [systems[i] for i in slow],
                                     [users[i] for i in slow])
        out[torch.as_tensor(slow)] = torch.as_tensor(vals, dtype=torch.float64)
    return out.to(engine.device) if device_out else out


@torch.no_grad()
def text_compat_span_sums(engine, tok, systems: Sequence[Optional[str]],
                          users: Sequence[str]) -> List[float]:
    """``sum(get_prompt_logprobs(.., systems[i], users[i])[1])`` (NaN where that call gives
    no usable log-probs) for many pairs in ONE batched prefill: the reference's span
    (first-occurrence ``find``, char overlap; src/utils.py:284-373) depends only on the
    token strings, so only the kept positions' rows go through the LM head."""
    n = len(users)
    res = [float("nan")] * n
    idss, keeps = [], []
    for s, u in zip(systems, users):
        try:
            api_user = u + MARKER if u.endswith(("\n", " ")) else u
            ids, _ = tok.render_chat(s or None, api_user)
            data = SimpleNamespace(tokens=tok.tokens(ids), token_logprobs=list(range(len(ids))))
            _, keep = extract_user_prompt_logprobs(data, u)
        except Exception as e:       # get_prompt_logprobs would return ([], [])
            logger.error("get_prompt_logprobs failed: %s", e)
            ids, keep = [], []
        idss.append(list(ids))
        keeps.append(keep)
    # position 0 has no log-prob (None in the reference's list -> no usable sum)
    todo = [j for j in range(n) if keeps[j] and keeps[j][0] > 0]
    if not todo:
        return res
    dev = engine.device
    cache = engine.prefill([idss[j] for j in todo])
    r_idx = [r for r, j in enumerate(todo) for _ in keeps[j]]
    p_idx = [i - 1 for j in todo for i in keeps[j]]
    tgt = [idss[j][i] for j in todo for i in keeps[j]]
    rows = cache.hidden[torch.as_tensor(r_idx, device=dev), torch.as_tensor(p_idx, device=dev)]
    lp = engine.rows_logprobs(rows, torch.as_tensor(tgt, dtype=torch.int32, device=dev)[:, None])
    lp = lp.view(-1).double().cpu().tolist()
    o = 0
    for j in todo:                   # the reference's Python sum, in span order
        k = len(keeps[j])
        res[j] = float(sum(lp[o:o + k]))
        o += k
    return res


@torch.no_grad()
def text_compat_last(engine, tok, systems: Sequence[Optional[str]],
                     users: Sequence[str], fallback: float = -10.0) -> List[float]:
    """The LAST log-prob of the reference's user span, ``sum(get_prompt_logprobs(..)[1][-1:])``
    (src/methods/beam_search.py:370-395), for many pairs in one batched prefill;
    ``fallback`` where the reference's call gives nothing usable (empty span, None), as
    its except branch does (:397-404)."""
    n = len(users)
    res = [float(fallback)] * n
    idss, last = [[] for _ in range(n)], [-1] * n
    apis = [u + MARKER if u.endswith(("\n", " ")) else u for u in users]
    # an ASCII prompt's token strings join to the rendered text itself: a user prompt that
    # text does not contain is found nowhere (the reference's call gives ([], []) and the
    # fallback), decided without encoding -- the common case of re-scored beam candidates
    # whose statement begins with whitespace the chat template trims
    live = list(range(n))
    chat_text = _ascii_text_of(tok)
    texts = None
    if chat_text is not None:
        try:
            texts = [chat_text(s or None, a, True) for s, a in zip(systems, apis)]
            live = [j for j in range(n)
                    if not (texts[j].isascii() and texts[j].find(users[j]) == -1)]
        except Exception:   # noqa: BLE001 -- per-call path below reports the failure
            texts, live = None, list(range(n))
    rendered = None
    many = getattr(tok, "encode_many", None) if texts is not None else None
    if live and many is not None:
        try:    # one batched (multi-threaded) encode of the prompts left
            rendered = dict(zip(live, many([texts[j] for j in live])))
        except Exception:   # noqa: BLE001
            rendered = None
    for j in live:
        try:
            ids = (rendered[j] if rendered is not None
                   else tok.render_chat(systems[j] or None, apis[j])[0])
            k = last_user_span_index(tok.tokens(ids), users[j])
        except Exception as e:       # get_prompt_logprobs would return ([], [])
            logger.error("get_prompt_logprobs failed: %s", e)
            ids, k = [], -1
        idss[j] = list(ids)
        last[j] = k
    _last_logprobs(engine, idss, last, res)
    return res


def _last_logprobs(engine, idss, last, res) -> None:
    """res[j] = log p(idss[j][last[j]] | idss[j][:last[j]]) for every j with last[j] > 0
    (position 0 has no log-prob: None in the reference's list), in one batched prefill."""
    todo = [j for j in range(len(idss)) if last[j] > 0]
    if not todo:
        return
    dev = engine.device
    cache = engine.prefill([idss[j][:last[j]] for j in todo])
    rows = cache.last_hidden
    tgt = torch.as_tensor([idss[j][last[j]] for j in todo], dtype=torch.int32, device=dev)
    lp = engine.rows_logprobs(rows, tgt[:, None]).view(-1).double().cpu().tolist()
    for j, v in zip(todo, lp):
        res[j] = float(v)


_PERIODS: Dict[str, int] = {}


def _min_period(u: str) -> int:
    """The smallest period of ``u`` (prefix function); two occurrences of u in a text that
    overlap start at least this far apart."""
    p = _PERIODS.get(u)
    if p is None:
        pi = [0] * len(u)
        k = 0
        for i in range(1, len(u)):
            while k and u[i] != u[k]:
                k = pi[k - 1]
            if u[i] == u[k]:
                k += 1
            pi[i] = k
        p = len(u) - (pi[-1] if u else 0)
        if len(_PERIODS) > 256:
            _PERIODS.clear()
        _PERIODS[u] = p
    return p


@torch.no_grad()
def text_compat_last_stems(engine, tok, system: Optional[str], agent_users: Sequence[str],
                           stems: Sequence[str], stem_of: Sequence[int], pieces: Sequence[str],
                           fallback: float = -10.0) -> List[float]:
    """text_compat_last for the users ``agent_users[a] + stems[stem_of[i]] + pieces[i]``
    (a-major: entry a * n + i) under one system prompt -- a beam step's re-tokenized texts,
    where every (agent, beam) shares its prompt up to the beam's statement and candidates
    differ in one token (src/methods/beam_search.py:358-395 via src/utils.py:201-373).

    Re-tokenized incrementally: each agent's chat prompt is rendered once around its user
    text (BPETokenizer.chat_frame) and encoded once up to a pre-token boundary a few
    pre-tokens before its end (cut_point: BPE merges never cross a pre-token, and appended
    text changes no pre-token before the last one); the short text from there to a boundary
    before the beam statement's end is encoded once per distinct string, each distinct
    candidate tail (statement end + token + marker) once, the template's closing part once.
    The reference's first-occurrence ``find`` of the user text in the joined token strings
    is decided from the head's joined strings (the agent text's first occurrence there, and
    its smallest period bounding any later occurrence) plus a short prefix test of the
    tail's -- exactly the full-prompt search, without building ~A * B * K prompts.  Falls
    back to text_compat_last for tokenizers or templates without these properties, and
    checks one prompt per call against a full encode."""
    A, n = len(agent_users), len(pieces)

    def full_path():
        users = [agent_users[a] + stems[stem_of[i]] + pieces[i] for a in range(A) for i in range(n)]
        return text_compat_last(engine, tok, [system] * len(users), users, fallback)

    ok = getattr(tok, "incremental_ok", None)
    if ok is None or not ok() or getattr(tok, "_inc_disabled", False) or not n or not A:
        return full_path()
    cache = tok.__dict__.setdefault("_inc_cache", {})
    if len(cache) > 4096:
        cache.clear()
    enc_later: Dict[str, Optional[List[int]]] = {}     # strings to encode in one batch

    def frame_of(u):
        key = ("frame", system, u)
        fr = cache.get(key)
        if fr is None:
            fr = tok.chat_frame(system or None, u)
            if fr is not None:
                pre, post, seg = fr
                y = tok.cut_point(pre, seg)
                fr = (pre[:y], pre[y:], post)
                enc_later.setdefault(fr[0], None)
                enc_later.setdefault(post, None)
            cache[key] = fr or False
        return fr or None

    frames = [frame_of(u) for u in agent_users]
    if any(f is None for f in frames) or any(not u or u[0].isspace() for u in agent_users):
        return full_path()
    bad_chars = tok.added_token_chars
    res = [float(fallback)] * (A * n)
    conts = [stems[stem_of[i]] + pieces[i] for i in range(n)]
    marks = [MARKER if c.endswith(("\n", " ")) else "" for c in conts]
    # items whose rendering is not pre + api + post (api ends in other whitespace the template
    # trims) or whose text could hold an added token: the full path
    def holds_added(text):
        return any(c in text for c in bad_chars)

    slow = [i for i in range(n) if (conts[i] + marks[i])[-1:].isspace() or holds_added(conts[i])]
    slow_agents = {a for a in range(A) if holds_added(agent_users[a])}
    slow_set = set(slow)
    groups: Dict[int, List[int]] = {}
    for i in range(n):
        if i not in slow_set:
            groups.setdefault(stem_of[i], []).append(i)
    # (mid + stem) -> (head part, tail part) at a pre-token boundary before the stem's end
    split: Dict[str, Tuple[str, str]] = {}
    for a in range(A):
        if a in slow_agents:
            continue
        mid = frames[a][1]
        for g in groups:
            s_ = mid + stems[g]
            if s_ not in split:
                x = tok.cut_point(s_, 0)
                split[s_] = (s_[:x], s_[x:])
                enc_later.setdefault(s_[:x], None)
                for i in groups[g]:
                    enc_later.setdefault(s_[x:] + pieces[i] + marks[i], None)
    todo_enc = [t for t, v in enc_later.items() if ("ids", t) not in cache]
    for t, ids in zip(todo_enc, tok.encode_many(todo_enc) if todo_enc else []):
        cache[("ids", t)] = ids
    ids_of = lambda t: cache[("ids", t)]                                 # noqa: E731
    jcache: Dict[str, str] = {}

    def joined(t):
        j = jcache.get(t)
        if j is None:
            ids = ids_of(t)
            j = jcache[t] = "".join(tok.tokens(ids)) if ids else ""
        return j

    # prompts checked against a full encode (a tokenizer outside the assumptions disables
    # the incremental path for good): the first item of every call, and one item of each
    # agent frame the first time that frame is seen -- every agent's own chat frame and cut
    # point (its user text, e.g. non-ASCII) is verified once, at the cost of one full encode
    # per distinct agent prompt
    fast_i = next((i for i in range(n) if i not in slow_set), None)
    probes = []
    if fast_i is not None:
        for a in range(A):
            if a in slow_agents:
                continue
            pkey = ("probed", system, agent_users[a])
            if not probes or pkey not in cache:
                probes.append(a)
                cache[pkey] = True
    for a in probes:
        i = fast_i
        base, mid, post = frames[a]
        hm, tp = split[mid + stems[stem_of[i]]]
        want = tok.encode(tok.chat_text(system or None, agent_users[a] + conts[i] + marks[i], True))
        if want != ids_of(base) + ids_of(hm) + ids_of(tp + pieces[i] + marks[i]) + ids_of(post):
            logger.warning("incremental re-tokenization disagrees with a full encode; "
                           "re-tokenizing whole prompts from now on")
            tok._inc_disabled = True
            return full_path()
    found: Dict[int, Tuple[List[int], int]] = {}      # a * n + i -> (prompt ids, last index)
    slow_items = []
    ginfo: Dict[str, tuple] = {}           # per (mid + stem): the candidates' tails, joined
    decided: Dict[tuple, List[int]] = {}   # per (mid + stem, head rest, post): the hits
    for a in range(A):
        if a in slow_agents:
            slow_items += [(a, i) for i in range(n)]
            continue
        slow_items += [(a, i) for i in slow]
        u = agent_users[a]
        base, mid, post = frames[a]
        jb, jq = joined(base), joined(post)
        per = min(_min_period(u), len(u))
        for g, items in groups.items():
            key_s = mid + stems[g]
            info = ginfo.get(key_s)
            if info is None:
                hm, tp = split[key_s]
                tkeys = [tp + pieces[i] + marks[i] for i in items]
                jts = [joined(t) for t in tkeys]
                info = ginfo[key_s] = (hm, tkeys, jts, max(map(len, jts)), joined(hm))
            hm, tkeys, jts, longest, jhm = info
            jh = jb + jhm
            f = jh.find(u)
            # u occurs first at f; any other occurrence overlapping the search region starts
            # at least min(period(u), len(u)) after f, and there is none when the text after
            # f is shorter than that plus len(u)
            if f >= 0 and len(jh) + longest + len(jq) - f - len(u) < per:
                rest_h = jh[f + len(u):]
                dkey = (key_s, rest_h, jq)
                hits = decided.get(dkey)
                if hits is None:
                    hits = decided[dkey] = [x for x, (i, jt) in enumerate(zip(items, jts))
                                            if (rest_h + jt + jq).startswith(conts[i])]
                los = [(x, f) for x in hits]
            else:
                los = []
                for x, (i, jt) in enumerate(zip(items, jts)):
                    lo = (jh + jt + jq).find(u + conts[i])
                    if lo >= 0:
                        los.append((x, lo))
            if not los:
                continue
            hid = ids_of(base) + ids_of(hm)
            hends = list(itertools.accumulate(map(len, tok.tokens(hid)))) if hid else []
            for x, lo in los:
                i, t = items[x], tkeys[x]
                ids = hid + ids_of(t) + ids_of(post)
                end = lo + len(u) + len(conts[i])
                if end <= len(jh):
                    k = bisect.bisect_left(hends, end)
                elif end <= len(jh) + len(jts[x]):
                    tends = list(itertools.accumulate(map(len, tok.tokens(ids_of(t)))))
                    k = len(hid) + bisect.bisect_left(tends, end - len(jh))
                else:
                    k = bisect.bisect_left(list(itertools.accumulate(map(len, tok.tokens(ids)))), end)
                found[a * n + i] = (ids, k)
    if slow_items:
        vals = text_compat_last(engine, tok, [system] * len(slow_items),
                                [agent_users[a] + conts[i] for a, i in slow_items], fallback)
        for (a, i), v in zip(slow_items, vals):
            res[a * n + i] = v
    if found:
        js = list(found)
        sub = [float(fallback)] * len(js)
        _last_logprobs(engine, [found[j][0] for j in js], [found[j][1] for j in js], sub)
        for j, v in zip(js, sub):
            res[j] = v
    return res


def get_token_ids(model, text) -> Dict[str, int]:
    """{token string: id} of the chat-rendered single-message prompt (src/utils.py:466-525)."""
    try:
        _, tok = runtime.get_engine(model)
        ids, _ = tok.render_chat(None, text)
        return {tok.token_str(i): i for i in ids}
    except Exception as e:
        logger.error("get_token_ids failed: %s", e)
        return {}


def generate_text(model, user_prompt, system_prompt=None, max_tokens=4096, temperature=1,
                  terminators=(), seed=None, bias_against_tokens=None, bias_value=-1000000,
                  use_chat_completions=True, repetition_penalty=1.0) -> str:
    """Sample a completion locally (src/utils.py:77-198 contract; '[ERROR: ...]' on failure).

    Chat mode renders the chat template with the generation prompt; completions mode
    uses the raw ``system + "\\n\\n" + user`` prompt.  Token t is drawn with seed
    draw_seed(seed, t); stop tokens end the text and are not included."""
    try:
        engine, tok = runtime.get_engine(model)
        if use_chat_completions:
            ids, _ = tok.render_chat(system_prompt or None, user_prompt)
        else:
            full = f"{system_prompt}\n\n{user_prompt}" if system_prompt else f"{user_prompt}"
            ids = tok.render_raw(full)
        bias = runtime.bias_token_ids(tok, bias_against_tokens)
        with runtime.device_lock(engine.device):
            out = runtime.generate(engine, tok, ids, [seed], max_tokens, float(temperature),
                                   bias_ids=bias, bias_value=float(bias_value))[0]
        text = tok.decode(out)
        for term in terminators or ():
            cut = text.find(term)
            if cut != -1:
                text = text[:cut]
        return text
    except Exception as e:
        logger.error("generate_text failed: %s", e)
        return f"[ERROR: {type(e).__name__}]"
