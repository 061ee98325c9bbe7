"""Merge tools/tune_gemm_dispatch.py outputs (--merge 0 runs, one per config) into the
installed selection: entries and measurements of the shapes a newer file measured replace
the older ones.

    python tools/merge_gemm_dispatch.py gpurun_out/a.json gpurun_out/b.json [--install]
"""
import argparse
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
INSTALLED = os.path.join(REPO, PKG, "tuned", "gemm_dispatch_mi355x.json")


def key(r):
    return f"{r['M']},{r['N']},{r['K']},{r['gated']}"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--install", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    with open(INSTALLED) as f:
        base = json.load(f)
    table, measured = dict(base.get("table", {})), list(base.get("measured", []))
    for fn in a.files:
        with open(fn) as f:
            new = json.load(f)
        seen = {key(r) for r in new["measured"]}
        table = {k: v for k, v in table.items() if k not in seen}
        table.update(new["table"])
        measured = [r for r in measured if key(r) not in seen] + new["measured"]
        for k in ("device", "torch", "hip", "library"):
            base[k] = new.get(k, base.get(k))
    base["table"], base["measured"] = table, measured
    out = INSTALLED if a.install else (a.out or os.path.join(REPO, "gpurun_out", "gemm_dispatch_merged.json"))
    with open(out, "w") as f:
        json.dump(base, f, indent=1)
    print(out, len(table), "entries,", sum("packed" in v for v in table.values()), "packed")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
