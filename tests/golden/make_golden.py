"""Generate the committed golden vectors under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container, where /root/reference exists (read-only).  The
reference is imported with two stub modules standing in for its network-only
dependencies (``together`` — an HTTPS client, ``dotenv``); nothing from the
reference is copied: only input/output DATA is written here.  The GPU box never
runs this script and never reads /root/reference.

Outputs
  core_golden.npz               core.py generate_params / compute_utilities / F_val /
                                log_softmax_rows / FW_nash_welfare / argmax selections
  eval_welfare_published.csv    per-agent avg_logprob + perplexity + perplexity-welfare
                                columns of every complete row of the reference's
                                results/appendix/*/evaluation/*/seed_*/evaluation_results.csv
  (method traces: see make_method_traces.py)

Usage:  python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import glob
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def install_stubs() -> str:
    """Write stub `together` / `dotenv` packages to a temp dir and put it on sys.path."""
    d = tempfile.mkdtemp(prefix="ref_stubs_")
    os.makedirs(os.path.join(d, "together"))
    os.makedirs(os.path.join(d, "dotenv"))
    with open(os.path.join(d, "together", "__init__.py"), "w") as f:
        f.write("class Together:\n    def __init__(self, *a, **k):\n        pass\n")
    with open(os.path.join(d, "dotenv", "__init__.py"), "w") as f:
        f.write("def load_dotenv(*a, **k):\n    return False\n")
    sys.path.insert(0, d)
    return d


def import_reference(ref: str):
    sys.dont_write_bytecode = True  # never write __pycache__ into the reference tree
    install_stubs()
    if ref not in sys.path:
        sys.path.insert(0, ref)
    import core  # noqa: E402

    return core


def make_core(core) -> None:
    B, L, d, n = 3, 4, 8, 6          # core.py:342-344
    rho_grid = np.linspace(0.6, 5.0, 20)  # core.py:348
    rho_idx = [0, 9, 19]
    seeds = [42, 43, 44]             # base_seed + run, core.py:345-359
    out = {"B": B, "L": L, "d": d, "n": n, "seeds": np.array(seeds), "rho": rho_grid[rho_idx]}
    for s in seeds:
        v, w = core.generate_params(B, L, d, n, seed=s)
        out[f"v_{s}"] = v
        out[f"w_{s}"] = w
        for ri, rho in zip(rho_idx, rho_grid[rho_idx]):
            U, leaves = core.compute_utilities(v, w, rho)
            m = U.shape[1]
            fvals = np.array([core.F_val(U, np.eye(m)[j]) for j in range(m)])
            out[f"U_{s}_{ri}"] = U
            out[f"Fpoint_{s}_{ri}"] = fvals                       # core.py:108-113 at p = e_j
            out[f"jutil_{s}_{ri}"] = int(np.argmax(U.sum(axis=0)))  # core.py:374
            out[f"jegal_{s}_{ri}"] = int(np.argmax(U.min(axis=0)))  # max-min point mass
            out[f"jnash_{s}_{ri}"] = int(np.argmax(fvals))
        out["leaves"] = np.array(leaves, dtype=np.int32)
    # Nash-welfare lottery for one case (core.py:116-168), used by the lottery API
    v, w = core.generate_params(B, L, d, n, seed=42)
    U, _ = core.compute_utilities(v, w, rho_grid[9])
    out["p_nw_42_9"] = core.FW_nash_welfare(U, max_iters=1500, tol=1e-11)
    # raw log_softmax_rows vectors (core.py:64-68)
    rng = np.random.default_rng(7)
    for name, shape, scale in (("ls_small", (5, 7), 1.0), ("ls_wide", (3, 1000), 3.0),
                               ("ls_big", (4, 4099), 8.0)):
        M = rng.normal(size=shape) * scale
        out[f"{name}_in"] = M
        out[f"{name}_out"] = core.log_softmax_rows(M)
    np.savez_compressed(os.path.join(HERE, "core_golden.npz"), **out)
    print("wrote core_golden.npz")


def make_eval(ref: str) -> None:
    import pandas as pd

    rows = []
    files = sorted(glob.glob(os.path.join(ref, "results", "appendix", "*", "evaluation", "*",
                                          "seed_*", "evaluation_results.csv")))
    for f in files:
        df = pd.read_csv(f)
        agents = [c[len("avg_logprob_"):] for c in df.columns if c.startswith("avg_logprob_")]
        for i, r in df.iterrows():
            lp = [r[f"avg_logprob_{a}"] for a in agents]
            cols = ["egalitarian_welfare_perplexity", "utilitarian_welfare_perplexity",
                    "log_nash_welfare_perplexity"]
            if any(pd.isna(x) for x in lp) or any(pd.isna(r[c]) for c in cols):
                continue
            rec = {"source": os.path.relpath(f, ref), "row": i, "n_agents": len(agents)}
            for j, a in enumerate(agents):
                rec[f"avg_logprob_{j}"] = lp[j]
                rec[f"perplexity_{j}"] = r[f"perplexity_{a}"]
            for c in cols:
                rec[c] = r[c]
            rows.append(rec)
    out = pd.DataFrame(rows)
    out.to_csv(os.path.join(HERE, "eval_welfare_published.csv"), index=False, float_format="%.17g")
    print(f"wrote eval_welfare_published.csv ({len(out)} rows from {len(files)} files)")


def make_results_fixture(ref: str) -> None:
    """A published run directory (results.csv + config.yaml) and the header of its published
    evaluation_results.csv: inputs + expected schema of the file-level evaluation path."""
    import shutil

    src = os.path.join(ref, "results", "appendix", "aamas_gemma_scenario1_beam_search_20250511_222741")
    dst = os.path.join(HERE, "results_fixture")
    os.makedirs(dst, exist_ok=True)
    shutil.copyfile(os.path.join(src, "results.csv"), os.path.join(dst, "results.csv"))
    shutil.copyfile(os.path.join(src, "config.yaml"), os.path.join(dst, "config.yaml"))
    pub = os.path.join(src, "evaluation", "google_gemma-2-9b-it", "seed_0", "evaluation_results.csv")
    with open(pub) as f, open(os.path.join(dst, "published_evaluation_header.csv"), "w") as g:
        g.write(f.readline())
    print("wrote results_fixture/")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    core = import_reference(args.reference)
    make_core(core)
    make_eval(args.reference)
    make_results_fixture(args.reference)


if __name__ == "__main__":
    main()
