set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests; echo "tests rc=$?"; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
bash scripts/gpu_check.sh bench || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
echo "bench ok"
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r04n_bench_r8.jsonl 2> gpurun_out/r04n_bench_r8.err || exit 5
echo done
