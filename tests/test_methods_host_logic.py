"""CPU tests of the methods' HOST logic against the reference's golden traces.

The HIP kernels are not available on this CPU-only host, so these tests replace the
package's C-ABI ops *explicitly, inside the test* with the CPU oracle (test
infrastructure).  This checks everything around the kernels — prompt layouts, seed
schedules, tree order, dedupe/EOS walks, reward folding, selection — on the same
fixture model the reference traces were recorded with.  The product itself has no
CPU path: tests/test_methods_gpu.py replays the same traces through the real HIP
library on an MI355X.
"""
import importlib

import pytest
import torch

import method_parity as mp

PKG = mp.PKG


@pytest.fixture(scope="module", params=mp.TRACE_FILES)
def emulated(request, orc):
    import cpu_emulation
    R = importlib.import_module(PKG + ".runtime")
    saved = cpu_emulation.install()
    traces = mp.load_traces(request.param)
    mp.register_fixture_engine(traces, torch.device("cpu"))
    yield traces
    cpu_emulation.uninstall(saved)
    R.clear_engines()


def test_methods_match_reference_traces(emulated):
    failures = mp.check_methods(emulated)
    assert not failures, "\n".join(failures)


def test_beam_candidate_logprobs_match_reference_calls(emulated):
    failures, n = mp.check_beam_increments(emulated)
    assert n > 0 or not any(r["method"] == "beam_search" for r in emulated["runs"])
    assert not failures, "\n".join(failures[:20])


def test_evaluator_matches_reference(emulated):
    failures = mp.check_evaluations(emulated)
    assert not failures, "\n".join(failures)


def test_prompt_logprobs_match_reference(emulated):
    failures = mp.check_prompt_logprobs(emulated)
    assert not failures, "\n".join(failures)


def test_mcts_strict_mode_raises_the_reference_nameerror(emulated):
    """reference_rollout_nameerror reproduces mcts.py:615 (undefined name in the rollout's
    debug f-string): the first non-empty rollout raises NameError."""
    methods = importlib.import_module(PKG + ".methods")
    cfg = {"num_simulations": 2, "max_tokens": 2, "expansion_sample_width": 2, "rollout_depth": 3,
           "seed": 13, "reference_rollout_nameerror": True}
    gen = methods.get_method_generator("mcts", cfg, emulated["model_id"])
    with pytest.raises(NameError, match="final_statement"):
        gen.generate_statement(emulated["issue"], dict(emulated["agent_opinions"]))
