set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05k_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r05k_gpu_tests.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r05k_bench_r8.jsonl 2> gpurun_out/r05k_bench_r8.err || exit 3
EMULATE=8 bash scripts/prof_method.sh c3 c5 || exit 4
bash scripts/prof_method.sh c3 c5 c4 || exit 5
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r05k_bench_1g.jsonl 2> gpurun_out/r05k_bench_1g.err || exit 6
