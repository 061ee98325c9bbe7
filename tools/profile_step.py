"""Steady-state decode steps of a BASELINE beam config for rocprofv3: the method's step
graph (parents' history gather, forward of the new tokens, LM head, cs_beam_decode_step)
replayed N times after the setup, so the kernel stats are dominated by decode steps:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o c3 -f csv -- \
        python tools/profile_step.py c3 100
"""
import importlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main(name="c3", reps=100):
    R = importlib.import_module(bench.PKG_DIR + ".runtime")
    R.use_gemm_tuning()
    mc = bench.METHOD_CONFIGS[name]
    dev = torch.device("cuda:0")
    eng, tok = R.random_engine(mc["preset"], dev, reuse_caches=0, tokenizer_dir=bench.BPE_FIXTURE)
    ms = bench._graph_step_ms(eng, tok, bench.synthetic_opinions(mc["agents"]), mc, dev, reps=reps)
    print(f"{name}: graph step {ms:.3f} ms over {reps} replays", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c3", int(sys.argv[2]) if len(sys.argv) > 2 else 100)
