"""utils.text_compat_last_stems (CPU): the incremental re-tokenization of a beam step's texts
(each agent's prompt rendered once, each (agent, beam) prompt encoded once up to a
pre-token boundary, each candidate tail once) equals text_compat_last over the full
prompts -- the reference's re-tokenized last log-prob (src/methods/beam_search.py:358-395,
src/utils.py:201-373) -- on the byte-level BPE fixture: the same (prefix ids, target)
requests reach the engine, and the same values and fallbacks come back.  The engine is a
stub whose "log-prob" is a hash of the request, so any difference in the prompt ids, the
span's last index or the fallback decision shows."""
import importlib
import os
import random
import zlib

import pytest
import torch

PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
HERE = os.path.dirname(os.path.abspath(__file__))


class _StubEngine:
    device = torch.device("cpu")

    def __init__(self):
        self.requests = []

    def prefill(self, idss):
        self._batch = [tuple(x) for x in idss]
        return type("C", (), {"last_hidden": torch.arange(len(idss), dtype=torch.float32)[:, None]})()

    def rows_logprobs(self, rows, tgt):
        out = []
        for r, t in zip(rows[:, 0].long().tolist(), tgt[:, 0].tolist()):
            key = self._batch[r] + (int(t),)
            self.requests.append(key)
            out.append(-(zlib.crc32(repr(key).encode()) % 100000) / 1000.0)
        return torch.tensor(out, dtype=torch.float32)


@pytest.fixture(scope="module")
def bpe():
    T = importlib.import_module(PKG + ".tokenizer")
    return T.BPETokenizer(os.path.join(HERE, "golden", "bpe_fixture"), "llama3", vocab_size=4096,
                          use_config=True)


def _case(bpe, seed):
    P = importlib.import_module(PKG + ".methods.prompts")
    rng = random.Random(seed)
    issue = "Should a person's genetic code be considered private information?"
    opinions = ["It is private and must stay so.", "Research needs data; share it anonymised.",
                "Café owners and <b>bold</b> people disagree.", "Only with consent.\n"]
    users = [P.BEAM["agent_user"].format(issue=issue, opinion=o) for o in opinions]
    words = [" the", " data", " private", "Genetic", " information", ",", ".", " should",
             " be", " consent", "\n", " ", "  ", "\t", "é", " naïve", "'s", " 123", "4"]
    frag = [bpe.token_str(i) for i in rng.sample(range(300, 4000), 60)]
    stems = ["", "Genetic", "Genetic data should", " The data", "It is 12", "Privacy matters. ",
             "ends with newline\n", "x\t", "Tok<en"]
    for _ in range(4):
        stems.append("".join(rng.choice(words + frag) for _ in range(rng.randint(1, 12))))
    pieces, stem_of = [], []
    for g in range(len(stems)):
        for _ in range(rng.randint(3, 9)):
            pieces.append(rng.choice(words + frag + ["<|eot_id|>", " <"]))
            stem_of.append(g)
    return users, stems, stem_of, pieces


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_incremental_equals_full_prompts(bpe, seed):
    U = importlib.import_module(PKG + ".utils")
    P = importlib.import_module(PKG + ".methods.prompts")
    users, stems, stem_of, pieces = _case(bpe, seed)
    system = P.BEAM["agent_system"]
    e_inc, e_full = _StubEngine(), _StubEngine()
    got = U.text_compat_last_stems(e_inc, bpe, system, users, stems, stem_of, pieces)
    full = [users[a] + stems[stem_of[i]] + pieces[i] for a in range(len(users))
            for i in range(len(pieces))]
    want = U.text_compat_last(e_full, bpe, [system] * len(full), full)
    assert not getattr(bpe, "_inc_disabled", False)
    assert got == want
    assert sorted(e_inc.requests) == sorted(e_full.requests)
    assert e_full.requests, "no case was found at the user span"


def test_incremental_disables_itself_on_a_disagreeing_tokenizer(bpe):
    """A tokenizer that breaks the assumptions (here: cut_point forced into the middle of a
    word) is caught by the per-call full-encode check, and the result is still exact."""
    T = importlib.import_module(PKG + ".tokenizer")
    U = importlib.import_module(PKG + ".utils")
    P = importlib.import_module(PKG + ".methods.prompts")
    bad = T.BPETokenizer(os.path.join(HERE, "golden", "bpe_fixture"), "llama3", vocab_size=4096,
                         use_config=True)
    bad.cut_point = lambda text, seg: len(text) - 1
    users = [P.BEAM["agent_user"].format(issue="Parks?", opinion="More parks.")]
    stems, stem_of, pieces = ["Genetic data sho"], [0, 0], ["uld", "w"]
    system = P.BEAM["agent_system"]
    got = U.text_compat_last_stems(_StubEngine(), bad, system, users, stems, stem_of, pieces)
    full = [users[0] + stems[0] + p for p in pieces]
    want = U.text_compat_last(_StubEngine(), bad, [system] * 2, full)
    assert bad._inc_disabled and got == want


def test_every_agent_frame_is_checked_once(bpe):
    """The full-encode check covers every agent's own chat frame and cut point:
    a tokenizer whose cut point breaks only for the SECOND agent's prompt is caught on the
    first call, and the result is still exact."""
    T = importlib.import_module(PKG + ".tokenizer")
    U = importlib.import_module(PKG + ".utils")
    P = importlib.import_module(PKG + ".methods.prompts")
    bad = T.BPETokenizer(os.path.join(HERE, "golden", "bpe_fixture"), "llama3", vocab_size=4096,
                         use_config=True)
    good_cut = bad.cut_point
    users = [P.BEAM["agent_user"].format(issue="Parks?", opinion=o)
             for o in ("More parks.", "Naïve café prices.")]
    # a mid-word cut (" pr|ices", one BPE token) only inside the second agent's opinion
    bad.cut_point = lambda text, seg: (text.index("prices") + 2 if "prices" in text[seg:] else
                                       good_cut(text, seg))
    stems, stem_of, pieces = ["Genetic data sho"], [0, 0], ["uld", "w"]
    system = P.BEAM["agent_system"]
    got = U.text_compat_last_stems(_StubEngine(), bad, system, users, stems, stem_of, pieces)
    full = [u + stems[0] + p for u in users for p in pieces]
    want = U.text_compat_last(_StubEngine(), bad, [system] * len(full), full)
    assert bad._inc_disabled and got == want
