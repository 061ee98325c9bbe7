#!/usr/bin/env bash
# Kernel-time breakdown of one method-level decode leg (bench --method <cfg> only):
# rocprofv3 --kernel-trace --stats, summary under gpurun_out/prof_method_<cfg>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
# EMULATE=N: the legs as rank 0 of an N-rank job (bench --emulate-ranks), output *_r<N>
TAG=""
EXTRA=""
if [ -n "${EMULATE:-}" ]; then TAG="_r$EMULATE"; EXTRA="--emulate-ranks $EMULATE"; fi
# SUFFIX: appended to the output name (A/B runs of one config)
TAG="$TAG${SUFFIX:-}"
for c in "$@"; do
  D="$R/gpurun_out/prof_method_$c$TAG"
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$D" -o run -f csv -- \
     python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-seconds 0 --e2e 0 --beam "" --method "$c" \
       --method-bon 0 --method-text-steps 0 $EXTRA > "$D.log" 2>&1) || exit $?
  python3 "$R/scripts/trace_by_grid.py" "$D/run_kernel_trace.csv" > "$D/by_grid.csv" || exit $?
  rm -f "$D/run_kernel_trace.csv"
  echo "prof $c$TAG done"
done
