#!/usr/bin/env bash
# Kernel-time breakdown of one method-level decode leg (bench --method <cfg> only):
# rocprofv3 --kernel-trace --stats, summary under gpurun_out/prof_method_<cfg>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
for c in "$@"; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_method_$c" -o run -f csv -- \
     python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --e2e 0 --beam "" --method "$c" \
       --method-bon 0 --method-text-steps 0 > "$R/gpurun_out/prof_method_$c.log" 2>&1) || exit $?
  python3 "$R/scripts/trace_by_grid.py" "$R/gpurun_out/prof_method_$c/run_kernel_trace.csv" \
    > "$R/gpurun_out/prof_method_$c/by_grid.csv" || exit $?
  rm -f "$R/gpurun_out/prof_method_$c/run_kernel_trace.csv"
  echo "prof $c done"
done
