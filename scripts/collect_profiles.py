#!/usr/bin/env python3
"""Copy one gpu_check.sh round trip (gpurun_out/) into profiles/<prefix>_*: test summary +
smoke line, bench JSON line, rocprofv3 kernel stats, the lsg_stream_kernel PMC rows and the
per-launch HBM traffic (profiles/pmc_traffic.json, read by bench.py).
python scripts/collect_profiles.py r01h"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")
prefix = sys.argv[1]


def lines(path):
    with open(path, errors="replace") as f:
        return f.read().splitlines()


tests = [l for l in lines(os.path.join(OUT, "gpu_tests.log")) if "::" in l or "passed" in l]
smoke = [l for l in lines(os.path.join(OUT, "smoke.log")) if l.startswith("smoke")]
with open(os.path.join(PROF, f"{prefix}_gpu_tests_summary.txt"), "w") as f:
    f.write("\n".join(tests + smoke) + "\n")
bench = [l for l in lines(os.path.join(OUT, "bench.log")) if l.startswith("{")]
with open(os.path.join(PROF, f"{prefix}_bench.jsonl"), "w") as f:
    f.write("\n".join(bench) + "\n")
shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"),
            os.path.join(PROF, f"{prefix}_kernel_stats.csv"))

kb = {}
for name in ("fetch", "write"):
    src = os.path.join(OUT, f"pmc_{name}", "run_counter_collection.csv")
    with open(src) as f:
        rows = list(csv.DictReader(f))
    lsg = [r for r in rows if "lsg_stream_kernel" in r["Kernel_Name"]]
    with open(os.path.join(PROF, f"{prefix}_pmc_{name}_lsg.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(lsg)
    vals = [float(r["Counter_Value"]) for r in lsg]
    kb[name] = sum(vals) / len(vals)

line = json.loads(bench[0])
rows, vocab = 76800, 128256
alg = line["roofline"]["alg_bytes_per_launch"]
traffic = {"c2": {
    "rows": rows, "vocab": vocab,
    "fetch_size_kb": kb["fetch"], "write_size_kb": kb["write"],
    "hbm_bytes_per_launch": (2 * kb["fetch"] + kb["write"]) * 1024.0,
    "correction": "FETCH_SIZE x2: gfx950 reports half the bytes of a wide coalesced streaming "
                  "read (MI355X_MICROARCH.md, HBM section); WRITE_SIZE as reported",
    "alg_bytes_per_launch": alg,
    "source": f"profiles/{prefix}_pmc_fetch_lsg.csv, profiles/{prefix}_pmc_write_lsg.csv "
              "(rocprofv3 --pmc, separate passes)",
    "kernel_config": "lsg_stream_kernel<bf16, 1024 threads, 2 x 16 B in flight, nt>"}}
try:   # keep the other entries (beam_*: scripts/collect_pmc_beam.py)
    with open(os.path.join(PROF, "pmc_traffic.json")) as f:
        traffic = {**json.load(f), **traffic}
except (OSError, ValueError):
    pass
with open(os.path.join(PROF, "pmc_traffic.json"), "w") as f:
    json.dump(traffic, f, indent=1)
print(json.dumps({"tests": tests[-1] if tests else None, "value": line["value"],
                  "frac": line["roofline"]["frac"],
                  "traffic_over_alg": traffic["c2"]["hbm_bytes_per_launch"] / alg}))
