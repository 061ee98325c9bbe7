"""Per-category kernel time of a method leg's rocprof by-grid table (scripts/trace_by_grid.py
output): total, per forward pass (= rope_place launches / layers) and share of the
non-initialisation kernel time, over the launches that repeat every forward (the prefills'
one-off launches are left out).

    python scripts/step_breakdown.py gpurun_out/prof_method_c3_r8/by_grid.csv --layers 42 [--steps N]
"""
import argparse
import collections
import csv


def category(k: str) -> str:
    if "Cijk" in k or "gemm_kernel" in k:
        return "GEMM"
    for key, name in (("splitk_reduce", "GEMM split-K fold"), ("attn_merge", "attention merge"),
                      ("attn", "attention"), ("rope", "rope_place"), ("add_rms", "add_rms_norm"),
                      ("gated_act", "gated_act"), ("hist_gather", "hist / tree gather"),
                      ("beam_decode", "beam_decode"), ("lsg", "logsoftmax_gather")):
        if key in k:
            return name
    if "distribution" in k or "MulFunctor" in k or "bfloat16_copy" in k:
        return "model init (randn)"
    return "other"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--layers", type=int, required=True)
    ap.add_argument("--skip-grid", default="78643200x1x1",
                    help="grids to leave out (the C2 kernel-only launch of the same bench run)")
    ap.add_argument("--min-forwards", type=int, default=10,
                    help="keep launches seen at least this many times per layer: the decode "
                         "steps' kernels, not the one-off prefill / initialisation launches")
    ap.add_argument("--steps", type=int, default=0,
                    help="report per method step (this many steps in the trace) instead of "
                         "per forward pass")
    a = ap.parse_args()
    per_step = ("beam_decode", "hist / tree gather", "logsoftmax_gather")
    rows = [r for r in csv.DictReader(open(a.csv))
            if int(r["launches"]) >= a.min_forwards * (1 if category(r["kernel"]) in per_step
                                                       else a.layers)]
    tot = collections.defaultdict(float)
    fwd = 0
    for r in rows:
        if r["grid"] in a.skip_grid.split(","):
            continue
        c = category(r["kernel"])
        tot[c] += float(r["total_ms"])
        if c == "rope_place":
            fwd += int(r["launches"])
    fwd /= a.layers
    unit = a.steps if a.steps else fwd
    work = sum(v for k, v in tot.items() if k != "model init (randn)")
    print(f"forward passes: {fwd:.0f}" + (f", method steps: {a.steps}" if a.steps else ""))
    print("category,total_ms,us_per_" + ("step" if a.steps else "forward") + ",share")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        if k == "model init (randn)":
            continue
        print(f"{k},{v:.1f},{v / unit * 1e3:.1f},{v / work:.3f}")
    print(f"total,{work:.1f},{work / unit * 1e3:.1f},1.000")


if __name__ == "__main__":
    main()
