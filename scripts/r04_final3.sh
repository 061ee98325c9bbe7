#!/bin/bash
# after the 4-wave gated form + re-tuned gated entries: GPU tests, smoke, bench, per-rank steps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
echo "smoke ok"
bash scripts/gpu_check.sh bench || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r04final3_bench_r8.jsonl 2>/dev/null || exit 5
