#!/usr/bin/env bash
# rocprofv3 kernel stats of the C2 end-to-end leg alone (the headline value's pass):
# bash scripts/prof_e2e.sh TAG -> gpurun_out/prof_e2e_TAG/run_kernel_stats.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT="$R/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-e2e}
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_e2e_$TAG" -o run -f csv -- \
   python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --beam "" --method "" --method-bon 0 \
   > "$OUT/prof_e2e_$TAG.log" 2>&1) && \
  python3 "$R/scripts/trace_by_grid.py" "$OUT/prof_e2e_$TAG/run_kernel_trace.csv" > "$OUT/prof_e2e_$TAG/by_grid.csv" && \
  rm -f "$OUT/prof_e2e_$TAG/run_kernel_trace.csv"
