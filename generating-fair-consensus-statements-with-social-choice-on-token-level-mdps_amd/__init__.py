"""MI355X-native agent x candidate scoring + welfare for token-level MDP decoding.

A drop-in for the hot path of
cartgr/Generating-Fair-Consensus-Statements-with-Social-Choice-on-Token-Level-MDPs:
per-agent log-probability utilities of candidate extensions and their
egalitarian / utilitarian / Nash welfare, computed by hand-written gfx950 HIP
kernels behind the C-ABI in ``include/consensus_scoring.h``.

The directory name is not a Python identifier; import it with
``importlib.import_module("generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd")``
(the test suite and entry points register the alias ``fair_consensus_amd``).
"""
from ._lib import CSError, load as load_library, version  # noqa: F401

__all__ = ["CSError", "load_library", "version", "ops"]


def __getattr__(name):
    import importlib

    if name in ("ops", "core", "engine", "model", "tokenizer", "utils", "methods", "evaluation",
                "parallel", "scoring", "build"):
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
