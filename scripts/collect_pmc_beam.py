#!/usr/bin/env python3
"""Per-launch HBM traffic of the beam decode launches from a scripts/pmc_beam.sh round trip
(gpurun_out/pmc_beam_<cfg>_{FETCH,WRITE}_SIZE, one bench beam config per run) ->
profiles/<prefix>_pmc_beam.csv and the beam_<cfg> entries of profiles/pmc_traffic.json
(read by bench.py).  python scripts/collect_pmc_beam.py r05h"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")
sys.path.insert(0, REPO)
prefix = sys.argv[1]
import bench  # noqa: E402  (BEAM_CONFIGS: agents, beams, top-k, vocab, cap, dtype)

kb, rows_out, meta = {}, [], {}
for cfg, (A, B, K, V, cap, dt, desc) in bench.BEAM_CONFIGS.items():
    esz = 4 if "float32" in str(dt) else 2
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(OUT, f"pmc_beam_{cfg}_{counter}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            for r in csv.DictReader(f):
                if "beam_decode_kernel" not in r["Kernel_Name"]:
                    continue
                kern = r["Kernel_Name"][r["Kernel_Name"].index("beam_decode_kernel"):].split("(")[0]
                kb.setdefault((cfg, counter), []).append(float(r["Counter_Value"]))
                meta[cfg] = (kern, A * B + B, V, esz)
                rows_out.append({"config": "beam_" + cfg, "counter": counter, "kernel": kern,
                                 "value_kb": r["Counter_Value"]})
with open(os.path.join(PROF, f"{prefix}_pmc_beam.csv"), "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=["config", "counter", "kernel", "value_kb"])
    w.writeheader()
    w.writerows(rows_out)
path = os.path.join(PROF, "pmc_traffic.json")
with open(path) as f:
    traffic = json.load(f)
for cfg, (kern, rows, vocab, esz) in meta.items():
    if (cfg, "FETCH_SIZE") not in kb or (cfg, "WRITE_SIZE") not in kb:
        continue
    fetch = sum(kb[(cfg, "FETCH_SIZE")]) / len(kb[(cfg, "FETCH_SIZE")])
    write = sum(kb[(cfg, "WRITE_SIZE")]) / len(kb[(cfg, "WRITE_SIZE")])
    alg = rows * vocab * esz
    name = "beam_" + cfg
    traffic[name] = {"rows": rows, "vocab": vocab, "fetch_size_kb": fetch, "write_size_kb": write,
                     "hbm_bytes_per_launch": (2 * fetch + write) * 1024.0,
                     "alg_bytes_per_launch": alg, "kernel_config": kern,
                     "launches": len(kb[(cfg, "FETCH_SIZE")]),
                     "correction": traffic["c2"]["correction"],
                     "source": f"profiles/{prefix}_pmc_beam.csv (rocprofv3 --pmc, separate passes)"}
    print(name, kern, round(traffic[name]["hbm_bytes_per_launch"] / alg, 4))
with open(path, "w") as f:
    json.dump(traffic, f, indent=1)
