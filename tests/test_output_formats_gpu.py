"""§8(f) row 4 on the MI355X: the evaluator's file-level path (src/evaluation.py:1072-1428)
through the HIP library -- every statement of the committed results.csv scored under
every agent on the device (fp32 fixture model: the eager path; its bf16 rounding: the
stream kernels), evaluation_results.csv written in the published layout, the reference's
welfare identities (src/evaluation.py:329-381) holding on every row."""
import importlib
import math
import os
import shutil

import pandas as pd
import pytest
import torch

import method_parity as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "results_fixture")
MODEL = "google/gemma-2-9b-it"


@pytest.fixture(scope="module", params=["float32", "bfloat16"])
def evaluated(request, tmp_path_factory, dev):
    R = importlib.import_module(mp.PKG + ".runtime")
    L = importlib.import_module(mp.PKG + "._lib")
    traces = mp.load_traces("method_traces_wide.json")   # head_dim 64: bf16 -> stream kernels
    dtype = getattr(torch, request.param)
    eng, _ = mp.register_fixture_engine(traces, dev, dtype=dtype, model_id=MODEL)
    run = tmp_path_factory.mktemp("run_" + request.param)
    shutil.copy(os.path.join(FIX, "results.csv"), run / "results.csv")
    shutil.copy(os.path.join(FIX, "config.yaml"), run / "config.yaml")
    ev_mod = importlib.import_module(mp.PKG + ".evaluation")
    ev = ev_mod.StatementEvaluator(MODEL, include_comparative_ranking=False, verbose=False)
    out = run / "evaluation" / "google_gemma-2-9b-it" / "seed_0"
    combined = ev.evaluate_results_file(run / "results.csv", output_dir=out, is_seed_specific=True)
    assert L._lib is not None, "the HIP library must be the path"
    yield run, out, combined, eng
    R.clear_engines()


def test_evaluation_csv_schema_matches_published_on_gpu(evaluated):
    run, out, combined, eng = evaluated
    ours = pd.read_csv(out / "evaluation_results.csv")
    published = open(os.path.join(FIX, "published_evaluation_header.csv")).readline().strip().split(",")
    assert list(ours.columns) == published
    assert len(ours) == len(pd.read_csv(os.path.join(FIX, "results.csv")))
    assert (combined["evaluation_status"] == "completed").all()
    assert (out / "evaluation_config.yaml").exists()


def test_evaluation_csv_welfare_identities_on_gpu(evaluated):
    run, out, _, eng = evaluated
    df = pd.read_csv(out / "evaluation_results.csv")
    agents = [c[len("avg_logprob_"):] for c in df.columns if c.startswith("avg_logprob_")]
    assert agents
    for _, r in df.iterrows():
        lps = [r[f"avg_logprob_{a}"] for a in agents]
        assert all(math.isfinite(v) and v < 0 for v in lps)
        ppl = [math.exp(-v) for v in lps]
        assert abs(r["egalitarian_welfare_perplexity"] - max(ppl)) <= 1e-3 * max(ppl)
        assert abs(r["utilitarian_welfare_perplexity"] - sum(ppl)) <= 1e-3 * sum(ppl)
        assert abs(r["log_nash_welfare_perplexity"] - sum(lps)) < 1e-3
        for a, v in zip(agents, lps):
            assert abs(r[f"perplexity_{a}"] - math.exp(-v)) <= 1e-3 * math.exp(-v)


def test_evaluation_csv_rows_equal_single_statement_scoring(evaluated):
    """Each row's per-agent utilities equal evaluate_statement of that statement alone (the
    batched file path and the per-statement API agree on the device)."""
    run, out, _, eng = evaluated
    ev_mod = importlib.import_module(mp.PKG + ".evaluation")
    import yaml
    cfg = yaml.safe_load(open(run / "config.yaml"))["scenario"]
    ev = ev_mod.StatementEvaluator(MODEL, include_comparative_ranking=False, verbose=False)
    df = pd.read_csv(out / "evaluation_results.csv")
    tol = 1e-3 if eng.model.dtype == torch.float32 else 0.06
    for _, r in df.head(3).iterrows():
        one = ev.evaluate_statement(r["statement"], cfg["issue"], dict(cfg["agent_opinions"]))
        for k, v in one.items():
            if k.startswith("avg_logprob_"):
                assert abs(float(v) - r[k]) <= tol, (k, v, r[k])
