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

from typing import Dict, Iterable, List, Sequence

LLAMA3_SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>",
                   "<|end_header_id|>", "<|eot_id|>"]
GEMMA2_SPECIALS = ["<bos>", "<eos>", "<start_of_turn>", "<end_of_turn>", "<pad>"]
# common non-Latin-1 characters in the reference's scenario texts and the marker
EXTRA_CHARS = ["\u200b", "\u2018", "\u2019", "\u201c", "\u201d", "\u2013", "\u2014", "\u2026",
               "\u2022", "\u20ac"]
UNK = "\ufffd"


# ids past the character table map to single code points from here on (planes 1-4 are
# outside every text the prompts contain and hold no surrogates), so a full-vocabulary
# tokenizer stays merge-free: every id is one distinct character
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
