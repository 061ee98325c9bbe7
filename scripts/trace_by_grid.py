#!/usr/bin/env python3
"""Aggregate a rocprofv3 kernel-trace CSV by (kernel, grid, workgroup): launches, mean and
total duration -- separates a decode step's launches from the prefill's launches of the same
kernel.  python3 scripts/trace_by_grid.py run_kernel_trace.csv > by_grid.csv"""
import csv
import sys


def main(path):
    agg = {}
    with open(path, newline="") as f:
        rd = csv.DictReader(f)
        cols = rd.fieldnames or []
        name = next(c for c in cols if c.lower() in ("kernel_name", "kernel-name", "name"))
        t0 = next(c for c in cols if "start" in c.lower())
        t1 = next(c for c in cols if "end" in c.lower())
        grid = [c for c in cols if c.lower().startswith("grid_size")]
        wg = [c for c in cols if c.lower().startswith("workgroup_size")]
        for r in rd:
            key = (r[name], "x".join(r[c] for c in grid), "x".join(r[c] for c in wg))
            d = int(r[t1]) - int(r[t0])
            n, tot = agg.get(key, (0, 0))
            agg[key] = (n + 1, tot + d)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "workgroup", "launches", "mean_us", "total_ms"])
    for (k, g, b), (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([k[:160], g, b, n, round(tot / n / 1e3, 2), round(tot / 1e6, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
