"""The bf16 rounding floor of a method trace (GPU diagnostic, not a test).

Replays a trace's beam search (free-running, as tests/method_parity.py check_beam_increments
does) three ways on the same seeded fixture weights and reports max / mean |delta| of every
per-agent candidate increment whose text the reference also scored:

  fp32-eager   fp32 weights, torch path (the fp32 parity route: should be ~1e-5)
  bf16-eager   the weights rounded once to bf16, torch path (torch matmuls + torch attention,
               fp32 accumulation): the error bf16 rounding itself costs at this model shape
  bf16-fused   the same bf16 weights on the shipped stream-kernel path (DecodeState,
               cs_prefix_attention, cs_gemm / hipBLASLt)

so a bf16 tolerance for a trace can be set against the measured floor rather than guessed.
Usage: python tools/bf16_floor.py method_traces_main128.json.gz
"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))

import importlib  # noqa: E402

import method_parity as mp  # noqa: E402


def beam_errors(traces):
    methods = importlib.import_module(mp.PKG + ".methods")
    prompts = importlib.import_module(mp.PKG + ".methods.prompts")
    users = [prompts.BEAM["agent_user"].format(issue=traces["issue"], opinion=op)
             for op in traces["agent_opinions"].values()]
    errs = []
    for run in traces["runs"]:
        if run["method"] != "beam_search":
            continue
        ref = {(c["system"], c["user"]): c["tail"][-1] for c in run["calls"] if c["tail"]}
        gen = methods.get_method_generator("beam_search", dict(run["config"]), traces["model_id"])
        gen.generate_statement(traces["issue"], dict(traces["agent_opinions"]))
        for step in gen.step_log:
            inc = step.get("increments")
            if inc is None:
                continue
            for i, cand in enumerate(step["candidates"]):
                for a, u in enumerate(users):
                    r = ref.get((prompts.BEAM["agent_system"], u + cand))
                    if r is not None:
                        errs.append(float(inc[a][i]) - r)
    return errs


def main():
    fname = sys.argv[1] if len(sys.argv) > 1 else "method_traces_main128.json.gz"
    dev = torch.device("cuda:0")
    t = mp.load_traces(fname)
    for tag, dtype, fused in (("fp32-eager", torch.float32, False),
                              ("bf16-eager", torch.bfloat16, False),
                              ("bf16-fused", torch.bfloat16, True)):
        t0 = time.time()
        eng, _ = mp.register_fixture_engine(t, dev, dtype=dtype)
        if not fused:
            eng.model.fused_ok = lambda *a, **k: False
        e = torch.tensor(beam_errors(t), dtype=torch.float64)
        a = e.abs()
        q = torch.quantile(a, torch.tensor([0.5, 0.99, 0.999], dtype=torch.float64)).tolist()
        print(f"{fname} beam {tag}: n={e.numel()} max_abs={a.max().item():.5f} "
              f"mean_abs={a.mean().item():.5f} mean_signed={e.mean().item():+.5f} "
              f"p50={q[0]:.5f} p99={q[1]:.5f} p99.9={q[2]:.5f} "
              f"over_0.06={(a > 0.06).sum().item()} ({time.time() - t0:.0f} s)", flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
