import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def _pkg():
    mod = importlib.import_module(PKG_DIR)
    sys.modules.setdefault("fair_consensus_amd", mod)
    return mod


@pytest.fixture(scope="session")
def pkg():
    return _pkg()


@pytest.fixture(scope="session")
def ops(pkg):
    return importlib.import_module(PKG_DIR + ".ops")


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def dev():
    """A GPU test that runs without a GPU must fail, not silently pass."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
