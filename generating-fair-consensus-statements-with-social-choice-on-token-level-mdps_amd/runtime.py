"""Model-identifier -> scoring engine registry, and seeded generation on the engine.

The reference resolves a model identifier (e.g. "meta-llama/Meta-Llama-3.1-8B-Instruct-Turbo")
to a remote endpoint through the module-global Together ``client`` (src/utils.py:69-74).
Here the identifier resolves to a local ``ScoringEngine`` on the current HIP device:
  * one registered explicitly (``register_engine``; tests register the parity fixture
    model this way);
  * a local Hugging Face checkpoint directory (config.json + *.safetensors +
    tokenizer.json): the identifier itself when it is a directory, or
    ``$CS_MODEL_ROOT/<identifier>`` (``register_model_dir`` maps an id to a directory);
  * ``random:<preset>`` (e.g. ``random:llama-3.1-8b``): an architecture-exact,
    random-initialised bf16 model with a full-vocabulary synthetic tokenizer — for
    throughput benchmarks only, the statements it produces mean nothing.
A real model id with none of these raises: random weights are never substituted
silently (set CS_ALLOW_RANDOM_INIT=1 to get the random-init model with a warning).

Concurrency: the reference runs generators in threads against one process
(src/experiment.py:283-322).  Everything that launches work on a device takes
``device_lock(device)`` (re-entrant), so forward passes and the kernels' shared
workspaces are used by one thread at a time per device.

Seed semantics of the local samplers (the replacement for the remote API's
``seed`` argument) are defined here once and restated by the test fake client:
  * a one-token draw with seed s uses the counter-based Gumbel noise g(s, v)
    (cs_vocab_sample);
  * token t of a multi-token generation with seed s uses seed ``draw_seed(s, t)``.
"""
from __future__ import annotations

import logging
import os
import re
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import ops
from .engine import BeamState, ScoringEngine
from .model import Model, preset
from .tokenizer import CharTokenizer

_M64 = (1 << 64) - 1
_lock = threading.RLock()
_ENGINES: Dict[str, Tuple[ScoringEngine, CharTokenizer]] = {}
_MODEL_DIRS: Dict[str, str] = {}
_DEVICE_LOCKS: Dict[str, threading.RLock] = {}
logger = logging.getLogger(__name__)

_NAME_TO_PRESET = [
    (r"3\.3-70b|llama-3\.3-70b|70b", "llama-3.3-70b"),
    (r"3\.1-8b|llama-3\.1-8b|8b", "llama-3.1-8b"),
    (r"3\.2-1b|1b", "llama-3.2-1b"),
    (r"gemma-2-9b|gemma", "gemma-2-9b"),
    (r"tiny-gemma", "tiny-gemma"),
    (r"tiny", "tiny-llama"),
]


def draw_seed(seed: int, t: int) -> int:
    """Seed of token t of a seeded multi-token generation."""
    return (int(seed) * 1000003 + int(t)) & _M64


def to_i64(seed: int) -> int:
    """uint64 seed -> the int64 bit pattern torch stores."""
    seed &= _M64
    return seed - (1 << 64) if seed >= (1 << 63) else seed


def fresh_seed() -> int:
    return int.from_bytes(os.urandom(8), "little")


def device_lock(device) -> threading.RLock:
    """The re-entrant lock serialising work on one device (forward passes, workspaces)."""
    key = str(torch.device(device))
    with _lock:
        lk = _DEVICE_LOCKS.get(key)
        if lk is None:
            lk = _DEVICE_LOCKS[key] = threading.RLock()
        return lk


def serialized(attr: str = "model_identifier"):
    """Method decorator: run under the device lock of ``getattr(self, attr)``'s engine
    (the reference's runner calls generators from threads, src/experiment.py:283-322)."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def wrap(self, *a, **k):
            eng, _ = get_engine(getattr(self, attr))
            with device_lock(eng.device):
                return fn(self, *a, **k)
        return wrap
    return deco


def register_engine(model_identifier: str, engine: ScoringEngine, tokenizer: CharTokenizer) -> None:
    with _lock:
        _ENGINES[model_identifier] = (engine, tokenizer)


def register_model_dir(model_identifier: str, path: str) -> None:
    """Serve ``model_identifier`` from a local checkpoint directory (loaded on first use)."""
    with _lock:
        _MODEL_DIRS[model_identifier] = path


def random_engine(preset_name: str, device=None, dtype=torch.bfloat16, seed: int = 0,
                  tokenizer_dir: Optional[str] = None, **engine_kw):
    """Architecture-exact random-init model + a full-vocabulary tokenizer: the
    character tokenizer, or the BPE of ``tokenizer_dir`` (tokenizer.json; ids past its
    table are synthetic single characters) for realistic prompt token counts."""
    cfg = preset(preset_name)
    dev = torch.device(device) if device is not None else \
        torch.device("cuda", torch.cuda.current_device())
    model = Model(cfg, dev, dtype, seed=seed)
    fam = "gemma2" if cfg.family == "gemma2" else "llama3"
    if tokenizer_dir:
        from .tokenizer import BPETokenizer
        # the fixture's chat template is Llama-3's: other families use their own layout
        tok = BPETokenizer(tokenizer_dir, fam, vocab_size=cfg.vocab, use_config=fam == "llama3")
    else:
        tok = CharTokenizer(fam, vocab_size=cfg.vocab)
    return ScoringEngine(model, **engine_kw), tok


def clear_engines() -> None:
    with _lock:
        _ENGINES.clear()


def resolve_preset(model_identifier: str) -> str:
    name = model_identifier.lower()
    for pat, pre in _NAME_TO_PRESET[::-1] if name.startswith("tiny") else _NAME_TO_PRESET:
        if re.search(pat, name):
            return pre
    raise ValueError(f"no local architecture known for model identifier {model_identifier!r}")


def _model_dir(model_identifier: str) -> Optional[str]:
    if model_identifier in _MODEL_DIRS:
        return _MODEL_DIRS[model_identifier]
    if os.path.isdir(model_identifier) and os.path.exists(os.path.join(model_identifier, "config.json")):
        return model_identifier
    root = os.environ.get("CS_MODEL_ROOT")
    if root:
        cand = os.path.join(root, model_identifier)
        if os.path.exists(os.path.join(cand, "config.json")):
            return cand
    return None


# --- GEMM solution selection -------------------------------------------------------
GEMM_TUNING = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "gemm_mi355x.csv")
_gemm_tuning: Optional[str] = None
_gemm_tuning_tried = False


def use_gemm_tuning(path: Optional[str] = None) -> Optional[str]:
    """Pick each forward GEMM's hipBLASLt solution from a committed PyTorch TunableOp
    results file (measured on MI355X by tools/tune_gemms.py) instead of the library
    heuristic — read only, no tuning at run time; shapes not in the file keep the heuristic.
    Returns the file in use (None: not used).

    TunableOp is process-wide (every later matmul of the process, bf16 rounding included,
    follows the file), so this is OPT-IN: call it (bench.py does), or set CS_GEMM_TUNING=1
    (the committed file) / CS_GEMM_TUNING=<file> to have ``get_engine`` call it.  An
    explicit TunableOp session (PYTORCH_TUNABLEOP_ENABLED in the environment, e.g. while
    tuning) is left alone; CS_GEMM_TUNING=0 disables.  Nothing is written back on exit."""
    global _gemm_tuning, _gemm_tuning_tried
    with _lock:
        if _gemm_tuning_tried and path is None:
            return _gemm_tuning
        _gemm_tuning_tried = True
        env = os.environ.get("CS_GEMM_TUNING")
        if env == "0" or "PYTORCH_TUNABLEOP_ENABLED" in os.environ or not torch.cuda.is_available():
            return None
        if env == "1":
            env = None
        path = path or env or GEMM_TUNING
        if not os.path.exists(path):
            return None
        import tempfile

        import torch.cuda.tunable as tunable
        try:
            tunable.enable(True)
            tunable.tuning_enable(False)
            tunable.record_untuned_enable(False)
            # the committed file is read only: no write-back at exit (and none to it)
            if hasattr(tunable, "write_file_on_exit"):
                tunable.write_file_on_exit(False)
            tunable.set_filename(os.path.join(tempfile.gettempdir(), f"cs_tunableop_{os.getpid()}.csv"))
            ok = tunable.read_file(path)
        except Exception as e:   # no usable device / TunableOp unavailable: library heuristic
            logger.warning("GEMM tuning file %s not loaded: %s", path, e)
            return None
        if not ok:
            logger.warning("GEMM tuning file %s not usable here (versions differ?)", path)
            tunable.enable(False)
            return None
        _gemm_tuning = path
        logger.info("GEMM solutions from %s (PyTorch TunableOp, process-wide, read only)", path)
        return path


_LOADING: Dict[str, threading.Lock] = {}


def get_engine(model_identifier: str) -> Tuple[ScoringEngine, CharTokenizer]:
    """The engine serving ``model_identifier``; loaded on first use.  A load (minutes for a
    70B checkpoint) holds only that identifier's loading lock, not the registry lock, so
    threads working on already-loaded engines are not stalled by it."""
    with _lock:
        if model_identifier in _ENGINES:
            return _ENGINES[model_identifier]
        if not torch.cuda.is_available():
            raise ops.CSError("no HIP device: the scoring engine has no CPU path")
        ld = _LOADING.setdefault(model_identifier, threading.Lock())
    with ld:
        with _lock:
            if model_identifier in _ENGINES:     # loaded by another thread meanwhile
                return _ENGINES[model_identifier]
            path = _model_dir(model_identifier)
        ent = _load_engine(model_identifier, path)
        if os.environ.get("CS_GEMM_TUNING", "0") != "0":
            use_gemm_tuning()
        with _lock:
            _ENGINES[model_identifier] = ent
        return ent


def _load_engine(model_identifier: str, path: Optional[str]):
    """Construct the engine of an identifier (no registry lock held)."""
    if path is not None:
        from .checkpoint import load_engine
        ent = load_engine(path)
    elif model_identifier.startswith("random:"):
        ent = random_engine(model_identifier.split(":", 1)[1])
    elif os.environ.get("CS_ALLOW_RANDOM_INIT") == "1":
        name = resolve_preset(model_identifier)
        logger.warning("model %r: no checkpoint found; using RANDOM-INIT %s weights "
                       "(CS_ALLOW_RANDOM_INIT=1) -- statements will be meaningless",
                       model_identifier, name)
        ent = random_engine(name)
    else:
        raise ops.CSError(
            f"no weights for model {model_identifier!r}: register an engine "
            "(runtime.register_engine), give a local checkpoint directory (config.json, "
            "*.safetensors, tokenizer.json) as the id, via runtime.register_model_dir or "
            "under $CS_MODEL_ROOT, or use 'random:<preset>' for an architecture-exact "
            "random-init benchmark model")
    return ent


# --- logit bias -------------------------------------------------------------------
def bias_token_ids(tok: CharTokenizer, strings: Optional[Sequence[str]]) -> List[int]:
    """Ids the reference biases for ``strings``.

    Semantics of get_token_ids (src/utils.py:466-525: token map of the chat-rendered
    single-user-message prompt) followed by the containment filter
    ``{t: id for t, id in map.items() if s in t}`` (src/utils.py:124-136,
    src/methods/beam_search.py:240-251).
    """
    if not strings:
        return []
    if isinstance(strings, str):
        strings = [strings]
    out: List[int] = []
    for s in strings:
        ids, _ = tok.render_chat(None, s)
        tmap = {}
        for i in ids:
            tmap[tok.token_str(i)] = i
        for t, i in tmap.items():
            if s in t and i not in out:
                out.append(i)
    return out


def apply_bias(logits: torch.Tensor, ids: Sequence[int], value: float) -> torch.Tensor:
    if ids:
        idx = torch.as_tensor(list(ids), dtype=torch.long, device=logits.device)
        logits[:, idx] = logits[:, idx] + value
    return logits


# --- seeded generation on the engine ------------------------------------------------
@torch.no_grad()
def generate(engine: ScoringEngine, tok: CharTokenizer, prefix_ids: Sequence[int],
             seeds: Sequence[Optional[int]], max_tokens: int, temperature: float = 1.0,
             bias_ids: Sequence[int] = (), bias_value: float = -1e6,
             stop_ids: Optional[Sequence[int]] = None) -> List[List[int]]:
    """Sample len(seeds) continuations of one prefix in a batch (token t of stream i
    drawn with seed draw_seed(seeds[i], t)); a stream stops after a stop token (not
    included) or max_tokens tokens."""
    n = len(seeds)
    seeds = [fresh_seed() if s is None else int(s) for s in seeds]
    stop = set(tok.eos_ids if stop_ids is None else stop_ids)
    out: List[List[int]] = [[] for _ in range(n)]
    if n == 0 or max_tokens <= 0:
        return out
    cache = engine.prefill([list(prefix_ids)])
    st = BeamState(engine, cache, n_prefix=1)
    alive = list(range(n))          # stream ids, in beam order
    dev = engine.device
    for t in range(max_tokens):
        logits = st.next_logits(0).float() if st.n_beams == len(alive) else None
        if st.n_beams == 1 and len(alive) > 1:
            logits = engine.model.lm_head(st.next_hidden).float().expand(len(alive), -1).contiguous()
        logits = apply_bias(logits, bias_ids, bias_value)
        sd = torch.tensor([[to_i64(draw_seed(seeds[i], t))] for i in alive], dtype=torch.int64,
                          device=dev)
        ids, _ = ops.vocab_sample(logits, sd, temperature=temperature, softcap=engine.softcap)
        ids = ids[:, 0].tolist()
        parent, toks, nxt = [], [], []
        for j, (i, v) in enumerate(zip(alive, ids)):
            if v in stop:
                continue
            out[i].append(v)
            if t + 1 < max_tokens:
                parent.append(0 if st.n_beams == 1 else j)
                toks.append(v)
                nxt.append(i)
        if not nxt:
            break
        st.advance(parent, toks)
        alive = nxt
    return out
