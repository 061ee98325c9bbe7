"""Method plugin registry (src/methods/__init__.py:11-44 contract).

GENERATOR_MAP / get_method_generator(method_name, method_config, generation_model)
-> generator_class(model_identifier, config).  The three scoring methods named by
the hot path and MCTS (the same agent-scoring primitive)
run on the local engine; the other reference methods (habermas_machine, zero_shot,
predefined) make no agent x candidate scoring calls, are outside this build's
scope and are not registered.
"""
from .base import BaseGenerator
from .beam_search import BeamSearchGenerator
from .best_of_n import BestOfNGenerator
from .finite_lookahead import FiniteLookaheadGenerator
from .mcts import MCTSGenerator

GENERATOR_MAP = {
    "mcts": MCTSGenerator,
    "beam_search": BeamSearchGenerator,
    "finite_lookahead": FiniteLookaheadGenerator,
    "best_of_n": BestOfNGenerator,
}


def get_method_generator(method_name: str, method_config: dict, generation_model: str) -> BaseGenerator:
    cls = GENERATOR_MAP.get(method_name)
    if cls is None:
        raise ValueError(f"Unknown method: {method_name}")
    return cls(generation_model, method_config)


__all__ = ["GENERATOR_MAP", "get_method_generator", "BaseGenerator", "BeamSearchGenerator",
           "BestOfNGenerator", "FiniteLookaheadGenerator", "MCTSGenerator"]
