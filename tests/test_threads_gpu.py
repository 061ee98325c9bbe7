"""Generators sharing one engine from concurrent threads (the reference's runner,
src/experiment.py:283-322, runs method configurations in a ThreadPoolExecutor against one
process) return exactly what the same calls return one after another: forward passes and
the kernels' shared workspaces are serialised per device (runtime.device_lock)."""
import importlib
from concurrent.futures import ThreadPoolExecutor

import pytest

import method_parity as mp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def traces(dev):
    t = mp.load_traces("method_traces.json")
    mp.register_fixture_engine(t, dev)
    yield t
    importlib.import_module(mp.PKG + ".runtime").clear_engines()


CALLS = [
    ("beam_search", {"beam_width": 3, "max_tokens": 6, "proposer": "topk", "top_k": 5, "seed": 1}),
    ("beam_search", {"beam_width": 2, "max_tokens": 5, "seed": 7}),
    ("best_of_n", {"n": 4, "max_tokens": 8, "seed": 3}),
    ("finite_lookahead", {"branching_factor": 2, "max_depth": 2, "max_tokens": 3, "seed": 5}),
    ("beam_search", {"beam_width": 3, "max_tokens": 6, "proposer": "topk", "top_k": 5, "seed": 1}),
]


def _run(traces, name, cfg):
    methods = importlib.import_module(mp.PKG + ".methods")
    gen = methods.get_method_generator(name, dict(cfg), traces["model_id"])
    return gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))


def test_concurrent_generators_equal_serial(traces):
    serial = [_run(traces, n, c) for n, c in CALLS]
    with ThreadPoolExecutor(max_workers=len(CALLS)) as ex:
        futs = [ex.submit(_run, traces, n, c) for n, c in CALLS]
        threaded = [f.result(timeout=300) for f in futs]
    assert threaded == serial
    assert serial[0] == serial[4]
