#!/usr/bin/env python3
"""Per-launch HBM traffic of the beam decode launches from a scripts/pmc_beam.sh round trip
(gpurun_out/pmc_beam_{FETCH,WRITE}_SIZE) -> profiles/<prefix>_pmc_beam.csv and the
beam_c1 / beam_c3 / beam_c5 entries of profiles/pmc_traffic.json (read by bench.py).
python scripts/collect_pmc_beam.py r01j"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")
prefix = sys.argv[1]
# decode kernel instantiation of each bench beam config at N = 1 -> (agent rows + ref rows, V, bytes/elt)
CONFIGS = {"beam_c1": ("beam_decode_kernel<0, false, false, 256, 8, 16>", 4 * 4 + 4, 128256, 4),
           "beam_c3": ("beam_decode_kernel<1, true, true, 1024, 2, 8>", 16 * 16 + 16, 256000, 2),
           "beam_c5": ("beam_decode_kernel<1, false, false, 1024, 2, 8>", 64 * 8 + 8, 128256, 2)}
kb, rows_out = {}, []
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    with open(os.path.join(OUT, f"pmc_beam_{counter}", "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            for name, (kern, *_rest) in CONFIGS.items():
                if kern in r["Kernel_Name"]:
                    kb.setdefault((name, counter), []).append(float(r["Counter_Value"]))
                    rows_out.append({"config": name, "counter": counter,
                                     "kernel": kern, "value_kb": r["Counter_Value"]})
with open(os.path.join(PROF, f"{prefix}_pmc_beam.csv"), "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=["config", "counter", "kernel", "value_kb"])
    w.writeheader()
    w.writerows(rows_out)
path = os.path.join(PROF, "pmc_traffic.json")
with open(path) as f:
    traffic = json.load(f)
for name, (kern, rows, vocab, esz) in CONFIGS.items():
    fetch = sum(kb[(name, "FETCH_SIZE")]) / len(kb[(name, "FETCH_SIZE")])
    write = sum(kb[(name, "WRITE_SIZE")]) / len(kb[(name, "WRITE_SIZE")])
    alg = rows * vocab * esz
    traffic[name] = {"rows": rows, "vocab": vocab, "fetch_size_kb": fetch, "write_size_kb": write,
                     "hbm_bytes_per_launch": (2 * fetch + write) * 1024.0,
                     "alg_bytes_per_launch": alg, "kernel_config": kern,
                     "correction": traffic["c2"]["correction"],
                     "source": f"profiles/{prefix}_pmc_beam.csv (rocprofv3 --pmc, separate passes)"}
    print(name, round(traffic[name]["hbm_bytes_per_launch"] / alg, 4))
with open(path, "w") as f:
    json.dump(traffic, f, indent=1)
