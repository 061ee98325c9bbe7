"""BaseGenerator: the reference's method plugin contract (src/methods/base.py:4-45)."""
from __future__ import annotations

import logging
from abc import ABC, abstractmethod


class BaseGenerator(ABC):
    """generator_class(model_identifier, config).generate_statement(issue, agent_opinions) -> str"""

    def __init__(self, model_identifier: str, config: dict):
        self.model_identifier = model_identifier
        self.config = config
        self.pre_brushup_statement = None  # read by src/experiment.py:184-188
        logging.getLogger(__name__).info("Initializing %s with model '%s' and config: %s",
                                         self.__class__.__name__, model_identifier, config)

    @abstractmethod
    def generate_statement(self, issue: str, agent_opinions: dict) -> str:
        """Generate a statement for ``issue`` given {agent id: opinion} (ordered)."""
