"""Character-level tokenizer with Llama-3 / Gemma-2 special tokens and chat templates.

Why character-level: the reference scores the re-tokenized STRING ``prompt + token``
and reads the last token's log-prob (src/methods/beam_search.py:358-390), and
slices the user span by character overlap (src/utils.py:321-363).  With a
merge-free tokenizer, appending a token id is exactly appending its string, so
the batched id-level engine and the reference's text-level path agree token for
token ("Parity under BPE re-tokenization").  No pretrained
tokenizer files are available offline; model vocabularies may be larger than the
tokenizer's (extra ids simply never occur in text).

Token strings concatenate back to the rendered prompt, which is what the
reference's ``extract_user_prompt_logprobs`` relies on (``"".join(tokens)``).
"""
from __future__ import annotations

import operator
from typing import Dict, Iterable, List, Optional, Sequence

LLAMA3_SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>",
                   "<|end_header_id|>", "<|eot_id|>"]
GEMMA2_SPECIALS = ["<bos>", "<eos>", "<start_of_turn>", "<end_of_turn>", "<pad>"]
# common non-Latin-1 characters in the reference's scenario texts and the marker
EXTRA_CHARS = ["\u200b", "\u2018", "\u2019", "\u201c", "\u201d", "\u2013", "\u2014", "\u2026",
               "\u2022", "\u20ac"]
UNK = "\ufffd"


# ids past the character table map to single code points from here on (no surrogates in
# planes 1+), so a full-vocabulary tokenizer stays merge-free: every id is one distinct
# character.  BENCHMARK / FIXTURE USE ONLY: these planes hold real characters (emoji from
# U+1F300, CJK Ext-B from U+20000), so with vocab_size > the table an opinion containing
# one encodes to an arbitrary vocabulary id instead of <unk>, and sampled ids decode to such
# characters.  Only the random-init benchmark engines (runtime.random_engine) and the
# parity fixtures use a full-vocabulary CharTokenizer; real checkpoints bring their own
# tokenizer.json (tokenizer.BPETokenizer).  The base is kept because the committed parity
# traces (tests/golden/method_traces_c1.json) spell their statements in these characters.
SYNTH_BASE = 0x10000


class CharTokenizer:
    """Deterministic char tokenizer: specials, Latin-1, a few extra code points, <unk>.

    ``vocab_size`` > the character table (e.g. the model's 128,256 or 256,000) gives every
    further id a distinct single synthetic character (chr(SYNTH_BASE + id)), for
    random-initialised benchmark models whose proposals range over the whole vocabulary:
    candidates stay distinct strings and encode(decode(ids)) == ids still holds."""

    def __init__(self, family: str = "llama3", vocab_size: int = 0) -> None:
        self.family = family
        specials = LLAMA3_SPECIALS + GEMMA2_SPECIALS
        self.id_to_str: List[str] = list(specials)
        self.special_ids: Dict[str, int] = {s: i for i, s in enumerate(specials)}
        self.char_to_id: Dict[str, int] = {}
        for c in [chr(i) for i in range(256)] + EXTRA_CHARS:
            if c not in self.char_to_id:
                self.char_to_id[c] = len(self.id_to_str)
                self.id_to_str.append(c)
        self.unk_id = len(self.id_to_str)
        self.id_to_str.append(UNK)
        self.char_to_id[UNK] = self.unk_id
        if family == "llama3":
            self.bos, self.eos = "<|begin_of_text|>", "<|eot_id|>"
            self.eos_strings = ("<|eot_id|>", "<|end_of_text|>")
        else:
            self.bos, self.eos = "<bos>", "<end_of_turn>"
            self.eos_strings = ("<end_of_turn>", "<eos>")
        self.bos_id = self.special_ids[self.bos]
        self.eos_id = self.special_ids[self.eos]
        self.eos_ids = tuple(self.special_ids[s] for s in self.eos_strings)
        self._specials_by_len = sorted(specials, key=len, reverse=True)
        self.n_table = len(self.id_to_str)
        self.full_vocab = max(int(vocab_size), self.n_table)

    @property
    def vocab_size(self) -> int:
        return self.full_vocab

    # --- plain text ---------------------------------------------------------------
    def encode(self, text: str) -> List[int]:
        """Characters -> ids; special-token strings in the text map to their special id
        (so a sampled special token survives the reference's string round trip)."""
        cid = self.char_to_id
        get = cid.get if self.full_vocab == self.n_table else self._char_id
        if "<" not in text:
            return [get(c, self.unk_id) for c in text]
        out: List[int] = []
        i, n = 0, len(text)
        specials = self._specials_by_len
        while i < n:
            c = text[i]
            if c == "<":
                for sp in specials:
                    if text.startswith(sp, i):
                        out.append(self.special_ids[sp])
                        i += len(sp)
                        break
                else:
                    out.append(get(c, self.unk_id))
                    i += 1
            else:
                out.append(get(c, self.unk_id))
                i += 1
        return out

    def _char_id(self, c: str, default: int) -> int:
        i = self.char_to_id.get(c)
        if i is not None:
            return i
        j = ord(c) - SYNTH_BASE
        return j if self.n_table <= j < self.full_vocab else default

    def decode(self, ids: Iterable[int]) -> str:
        return "".join(self.token_str(i) for i in ids)

    def token_str(self, i: int) -> str:
        if 0 <= i < self.n_table:
            return self.id_to_str[i]
        return chr(SYNTH_BASE + i) if self.n_table <= i < self.full_vocab else UNK

    def tokens(self, ids: Sequence[int]) -> List[str]:
        return [self.token_str(i) for i in ids]

    # --- prompt layouts -----------------------------------------------------------
    def render_raw(self, text: str, add_bos: bool = True) -> List[int]:
        """Completions-endpoint prompt: BOS + characters (no chat template)."""
        return ([self.bos_id] if add_bos else []) + self.encode(text)

    def render_chat(self, system: str | None, user: str, add_generation_prompt: bool = True):
        """Chat-template prompt.  Returns (ids, user_span) where user_span = (start, end)
        token positions of the user content (chat completions with echo=True)."""
        sp = self.special_ids
        ids: List[int] = []
        if self.family == "llama3":
            ids.append(sp["<|begin_of_text|>"])
            if system:
                ids += [sp["<|start_header_id|>"]] + self.encode("system")
                ids += [sp["<|end_header_id|>"]] + self.encode("\n\n" + system)
                ids.append(sp["<|eot_id|>"])
            ids += [sp["<|start_header_id|>"]] + self.encode("user")
            ids += [sp["<|end_header_id|>"]] + self.encode("\n\n")
            start = len(ids)
            ids += self.encode(user)
            end = len(ids)
            ids.append(sp["<|eot_id|>"])
            if add_generation_prompt:
                ids += [sp["<|start_header_id|>"]] + self.encode("assistant")
                ids += [sp["<|end_header_id|>"]] + self.encode("\n\n")
        else:  # gemma-2: no system role; system text is prefixed to the user turn
            ids.append(sp["<bos>"])
            ids += [sp["<start_of_turn>"]] + self.encode("user\n")
            if system:
                ids += self.encode(system + "\n\n")
            start = len(ids)
            ids += self.encode(user)
            end = len(ids)
            ids += [sp["<end_of_turn>"]] + self.encode("\n")
            if add_generation_prompt:
                ids += [sp["<start_of_turn>"]] + self.encode("model\n")
        return ids, (start, end)

    def chat_prefix(self, system: str | None, user_prefix: str) -> List[int]:
        """Token ids of the chat prompt up to and including ``user_prefix`` (the part of
        the user turn shared by every candidate).  Continuation tokens appended to this
        prefix are exactly the tokens the text path would produce for user_prefix+cont."""
        ids, (start, end) = self.render_chat(system, user_prefix, add_generation_prompt=False)
        return ids[:end]


FAMILY_SPECIALS = {
    # family: (bos, eos, end-of-sequence strings)
    "llama3": ("<|begin_of_text|>", "<|eot_id|>", ("<|eot_id|>", "<|end_of_text|>")),
    "gemma2": ("<bos>", "<end_of_turn>", ("<end_of_turn>", "<eos>")),
}
_SENTINEL = "⁣⁣cs-prefix-end⁣⁣"   # never in prompt text; cut point of chat_prefix


class BPETokenizer:
    """A checkpoint's own tokenizer: ``tokenizer.json`` (Hugging Face `tokenizers` format,
    e.g. Llama-3's byte-level BPE or Gemma-2's) and, from ``tokenizer_config.json``, its
    chat template (jinja, rendered as transformers' apply_chat_template renders it) —
    the text the hosted API of the reference renders and tokenizes server side
    (src/utils.py:249-259).  Same interface as CharTokenizer.

    Unlike a character tokenizer a BPE is NOT merge-free: the ids of ``prompt + token``
    need not be the prompt's ids plus the token's (the reference re-tokenizes the string,
    src/methods/beam_search.py:358-390).  ``merge_free`` is False and ``append_stable``
    tells the callers when an id-level continuation equals the re-tokenized text."""

    merge_free = False

    def __init__(self, path: str, family: str = "llama3", vocab_size: int = 0,
                 chat_template: "str | None" = None, use_config: bool = True) -> None:
        import json
        import os

        from tokenizers import Tokenizer

        tdir = path if os.path.isdir(path) else os.path.dirname(path)
        tfile = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
        self.tk = Tokenizer.from_file(tfile)
        self.family = family
        conf = {}
        cpath = os.path.join(tdir, "tokenizer_config.json")
        if use_config and os.path.exists(cpath):
            with open(cpath) as f:
                conf = json.load(f)
        self.chat_template = chat_template if chat_template is not None else conf.get("chat_template")
        bos, eos, eos_strings = FAMILY_SPECIALS[family]

        def tok_text(v, default):
            if isinstance(v, dict):
                v = v.get("content")
            return v or default

        self.bos = tok_text(conf.get("bos_token"), bos)
        self.eos = tok_text(conf.get("eos_token"), eos)
        self.eos_strings = tuple(s for s in dict.fromkeys((self.eos,) + eos_strings))
        self.special_ids: Dict[str, int] = {}
        for s in LLAMA3_SPECIALS + GEMMA2_SPECIALS + [self.bos, self.eos]:
            i = self.tk.token_to_id(s)
            if i is not None:
                self.special_ids[s] = i
        if self.bos not in self.special_ids or self.eos not in self.special_ids:
            raise ValueError(f"tokenizer {tfile} lacks the {family} special tokens {self.bos!r} / "
                             f"{self.eos!r}")
        self.bos_id = self.special_ids[self.bos]
        self.eos_id = self.special_ids[self.eos]
        self.eos_ids = tuple(self.special_ids[s] for s in self.eos_strings if s in self.special_ids)
        self.n_table = self.tk.get_vocab_size(with_added_tokens=True)
        self.full_vocab = max(int(vocab_size), self.n_table)
        self._strs: Dict[int, str] = {}
        self._table: Optional[List[str]] = None
        self._jinja = None

    @property
    def vocab_size(self) -> int:
        return self.full_vocab

    # --- plain text ---------------------------------------------------------------
    def encode(self, text: str) -> List[int]:
        return self.tk.encode(text, add_special_tokens=False).ids

    def encode_offsets(self, text: str):
        e = self.tk.encode(text, add_special_tokens=False)
        return e.ids, e.offsets

    def token_str(self, i: int) -> str:
        s = self._strs.get(i)
        if s is None:
            if 0 <= i < self.n_table:
                s = self.tk.decode([i], skip_special_tokens=False)
            elif self.n_table <= i < self.full_vocab:
                s = chr(SYNTH_BASE + i)
            else:
                s = UNK
            self._strs[i] = s
        return s

    def tokens(self, ids: Sequence[int]) -> List[str]:
        table = self._table
        if table is None:     # every table id's string, decoded once (C-speed lookups after)
            table = self._table = [self.token_str(i) for i in range(self.n_table)]
        ids = list(ids)
        if len(ids) > 1 and 0 <= min(ids) and max(ids) < self.n_table:
            return list(operator.itemgetter(*ids)(table))
        return [self.token_str(i) for i in ids]

    def decode(self, ids: Iterable[int]) -> str:
        ids = list(ids)
        if all(0 <= i < self.n_table for i in ids):
            return self.tk.decode(ids, skip_special_tokens=False)
        return "".join(self.token_str(i) for i in ids)

    def append_stable(self, prefix_text: str, prefix_ids: Sequence[int], piece: str,
                      piece_ids: Sequence[int]) -> bool:
        """Whether encode(prefix_text + piece) == prefix_ids + piece_ids (the id-level
        continuation is what the reference's re-tokenized string gives)."""
        return self.encode(prefix_text + piece) == list(prefix_ids) + list(piece_ids)

    # --- prompt layouts -----------------------------------------------------------
    def render_raw(self, text: str, add_bos: bool = True) -> List[int]:
        return ([self.bos_id] if add_bos else []) + self.encode(text)

    def _messages(self, system, user):
        if self.family == "gemma2":          # no system role: prefixed to the user turn
            return [{"role": "user", "content": (system + "\n\n" + user) if system else user}]
        msgs = [{"role": "system", "content": system}] if system else []
        return msgs + [{"role": "user", "content": user}]

    def chat_text(self, system: "str | None", user: str, add_generation_prompt: bool = True) -> str:
        """The rendered chat prompt string (the checkpoint's template, or the family's
        standard layout when it has none)."""
        if self.chat_template:
            if self._jinja is None:
                from jinja2.sandbox import ImmutableSandboxedEnvironment

                def raise_exception(msg):
                    raise ValueError(msg)

                env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
                env.globals["raise_exception"] = raise_exception
                self._jinja = env.from_string(self.chat_template)
            return self._jinja.render(messages=self._messages(system, user), bos_token=self.bos,
                                      eos_token=self.eos,
                                      add_generation_prompt=add_generation_prompt)
        if self.family == "llama3":
            t = "<|begin_of_text|>"
            if system:
                t += f"<|start_header_id|>system<|end_header_id|>\n\n{system}<|eot_id|>"
            t += f"<|start_header_id|>user<|end_header_id|>\n\n{user}<|eot_id|>"
            if add_generation_prompt:
                t += "<|start_header_id|>assistant<|end_header_id|>\n\n"
            return t
        u = (system + "\n\n" + user) if system else user
        t = f"<bos><start_of_turn>user\n{u}<end_of_turn>\n"
        return t + ("<start_of_turn>model\n" if add_generation_prompt else "")

    def render_chat(self, system: "str | None", user: str, add_generation_prompt: bool = True):
        """(ids, (start, end)): the chat prompt's ids and the token span of the user content
        (tokens whose characters overlap it, src/utils.py:321-363)."""
        text = self.chat_text(system, user, add_generation_prompt)
        ids, offs = self.encode_offsets(text)
        key = user.strip()
        c0 = text.rfind(key) if key else -1
        if c0 < 0:
            return ids, (len(ids), len(ids))
        c1 = c0 + len(key)
        span = [i for i, (a, b) in enumerate(offs) if a < c1 and b > c0]
        return ids, ((span[0], span[-1] + 1) if span else (len(ids), len(ids)))

    def render_chat_ids_many(self, systems, users, add_generation_prompt: bool = True):
        """render_chat(system, user)[0] for many pairs: the prompts rendered one by one, then
        encoded in ONE multi-threaded `tokenizers` batch (the per-call encode is most of a
        text-compat scoring call's host time)."""
        texts = [self.chat_text(s, u, add_generation_prompt) for s, u in zip(systems, users)]
        return [e.ids for e in self.tk.encode_batch(texts, add_special_tokens=False)]

    def encode_many(self, texts) -> List[List[int]]:
        return [e.ids for e in self.tk.encode_batch(list(texts), add_special_tokens=False)]

    # ASCII probes for ascii_joins_text: spaces (leading, doubled, trailing), newlines,
    # tabs, digits, punctuation, a marker-free trailing newline
    _ASCII_PROBES = (("You are a fair judge.  Answer briefly.", " The  statement: 'fair', 42.\n"),
                     ("Issue:\tprivacy\n\nOpinions follow.", "A\tB  c -- d ... e?!\n\nend "),
                     (None, "  leading and trailing  "))

    def ascii_joins_text(self) -> bool:
        """Whether an ASCII chat prompt's token strings join to the rendered text itself --
        true of byte-level BPEs (Llama-3), not of every tokenizer (a normalizer or a
        Metaspace / Strip decoder changes the strings).  The callers' shortcut that decides
        "the user text is found nowhere" by one search of the rendered text relies on it;
        checked once per tokenizer on probe prompts."""
        ok = getattr(self, "_ascii_join", None)
        if ok is None:
            ok = True
            for system, user in self._ASCII_PROBES:
                text = self.chat_text(system, user, True)
                if "".join(self.tokens(self.encode(text))) != text:
                    ok = False
                    break
            self._ascii_join = ok
        return ok

    # --- incremental re-tokenization ---------------------------------------------------
    def incremental_ok(self) -> bool:
        """Whether prompts may be re-tokenized incrementally (chat_frame / cut_point): no
        normalizer (the pre-tokenizer's char offsets are the text's) and a pre-tokenizer
        whose pieces BPE merges never cross (byte-level BPEs such as Llama-3's)."""
        ok = getattr(self, "_inc_ok", None)
        if ok is None:
            ok = self.tk.normalizer is None and self.tk.pre_tokenizer is not None
            # added tokens are split out of the text before pre-tokenization: content that
            # holds one's first character is re-tokenized whole (added_token_chars)
            self.added_token_chars = frozenset(
                t.content[0] for t in self.tk.get_added_tokens_decoder().values() if t.content)
            self._inc_ok = ok
        return ok

    def chat_frame(self, system: "str | None", user_prefix: str):
        """(pre, post, seg): the rendered chat prompt around user content ``user_prefix + X``
        -- chat_text(system, user_prefix + X) == pre + X + post for any X that does not end in
        whitespace (the template trims only the content's ends) -- and seg, the offset in
        ``pre`` after its last special token (the start of the text segment the pre-tokenizer
        sees).  None when the template does not render content that way or ``post`` does not
        open with a special token (which guarantees a token boundary after X)."""
        text = self.chat_text(system, user_prefix + _SENTINEL, True)
        i = text.find(_SENTINEL)
        if i < 0:
            return None
        pre, post = text[:i], text[i + len(_SENTINEL):]
        probe = " a, b:\n c.d"
        if self.chat_text(system, user_prefix + probe, True) != pre + probe + post:
            return None
        specials = list(self.special_ids)
        if not any(post.startswith(sp) for sp in specials):
            return None
        seg = max((pre.rfind(sp) + len(sp) for sp in specials if sp in pre), default=0)
        return pre, post, seg

    def cut_point(self, text: str, seg: int) -> int:
        """A token boundary of ``text + X`` for every X: the start of the second-to-last
        pre-token of text[seg:] (seg: a special-token boundary).  Pre-token matches before
        it end at least one whole pre-token before the end of ``text``, so appended text
        changes none of them (the split pattern looks ahead at most one character and never
        behind), and BPE merges stay inside pre-tokens."""
        pieces = self.tk.pre_tokenizer.pre_tokenize_str(text[seg:])
        if len(pieces) < 2:
            return seg
        return seg + pieces[-2][1][0]

    def chat_prefix(self, system: "str | None", user_prefix: str) -> List[int]:
        """Ids of the chat prompt up to the end of ``user_prefix`` (the part of the user
        turn shared by every candidate), with nothing of the template after it: the
        prompt is rendered with a sentinel after the prefix (so the template's trim does
        not eat the prefix's trailing whitespace) and cut there."""
        text = self.chat_text(system, user_prefix + _SENTINEL, add_generation_prompt=False)
        return self.encode(text[:text.index(_SENTINEL)])


def load_tokenizer(path: str, family: str, vocab_size: int = 0) -> BPETokenizer:
    return BPETokenizer(path, family=family, vocab_size=vocab_size)
