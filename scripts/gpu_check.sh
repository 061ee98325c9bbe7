#!/usr/bin/env bash
# One GPU round-trip: parity tests, smoke, bench, kernel-trace profile.  Every GPU
# step has its own time limit and the chain stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT="$R/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEP="${1:-all}"
run_tests() { timeout -k 10 420 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread --capture=tee-sys ${PYTEST_ARGS:-} > "$OUT/gpu_tests.log" 2>&1; }
run_smoke() { timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; }
run_bench() { timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; }
run_prof() {
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -f csv -- \
     python3 "$R/bench.py" --cpu-seconds 0 > "$OUT/prof.log" 2>&1) && \
  python3 "$R/scripts/trace_by_grid.py" "$OUT/prof/run_kernel_trace.csv" > "$OUT/prof/run_kernel_by_grid.csv" && \
  rm -f "$OUT/prof/run_kernel_trace.csv"   # the per-dispatch trace exceeds gpurun's copy-back cap
}
run_pmc() {
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -f csv -- \
     python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --beam "" --e2e 0 --method "" > "$OUT/pmc_fetch.log" 2>&1) && \
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -f csv -- \
     python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --beam "" --e2e 0 --method "" > "$OUT/pmc_write.log" 2>&1)
}
case "$STEP" in
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  pmc) run_pmc ;;
  all) run_tests; rc=$?; echo "tests rc=$rc" ; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
       run_smoke && run_bench && run_prof && run_pmc ;;
esac
