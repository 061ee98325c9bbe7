"""Method-level parity on the MI355X: the product's generators, evaluator and
text-compat scoring primitive, running through the HIP C-ABI library on the GPU,
replay the reference's golden traces (tests/golden/method_traces.json, recorded by
running the reference's own code, see make_method_traces.py)."""
import importlib

import pytest
import torch

import method_parity as mp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=mp.TRACE_FILES)
def traces(request, dev):
    t = mp.load_traces(request.param)
    mp.register_fixture_engine(t, dev)
    yield t
    importlib.import_module(mp.PKG + ".runtime").clear_engines()


def test_native_library_is_the_path(traces):
    ops = importlib.import_module(mp.PKG + ".ops")
    assert ops.logsoftmax_gather.__module__ == mp.PKG + ".ops"
    lib = importlib.import_module(mp.PKG + "._lib")
    assert lib._lib is not None or lib.load() is not None


def test_methods_match_reference_traces(traces):
    failures = mp.check_methods(traces)
    assert not failures, "\n".join(failures)


def test_evaluator_matches_reference(traces):
    failures = mp.check_evaluations(traces)
    assert not failures, "\n".join(failures)


def test_prompt_logprobs_match_reference(traces):
    failures = mp.check_prompt_logprobs(traces)
    assert not failures, "\n".join(failures)


def test_beam_topk_proposer_runs(traces):
    """The deterministic top-K proposer (BASELINE 'top-k tokens per beam') end to end."""
    methods = importlib.import_module(mp.PKG + ".methods")
    gen = methods.get_method_generator("beam_search", {"beam_width": 4, "max_tokens": 6,
                                                       "proposer": "topk", "top_k": 10,
                                                       "seed": 1}, traces["model_id"])
    s1 = gen.generate_statement(traces["issue"], traces["agent_opinions"])
    s2 = methods.get_method_generator("beam_search", {"beam_width": 4, "max_tokens": 6,
                                                      "proposer": "topk", "top_k": 10, "seed": 1},
                                      traces["model_id"]).generate_statement(
        traces["issue"], traces["agent_opinions"])
    assert s1 == s2 and isinstance(s1, str)
    assert all(len(st["candidates"]) <= 4 * 10 for st in gen.step_log)
