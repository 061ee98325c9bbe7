set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1; grep FAILED gpurun_out/gpu_tests.log | head -5
[ $rc -eq 0 ] || exit 2
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c1,c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r04r_bench_methods.jsonl 2> gpurun_out/r04r_bench_methods.err || exit 3
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r04r_bench_r8.jsonl 2> gpurun_out/r04r_bench_r8.err || exit 4
echo done
