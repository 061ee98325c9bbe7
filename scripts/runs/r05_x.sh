set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05x_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -12 gpurun_out/r05x_gpu_tests.log
[ $rc -eq 0 ] || exit 2
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05x_prof" -o run -f csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --beam "" --method "" --cpu-seconds 0 > "$R/gpurun_out/r05x_prof.log" 2>&1) || exit 3
python3 scripts/trace_by_grid.py gpurun_out/r05x_prof/run_kernel_trace.csv > gpurun_out/r05x_prof/by_grid.csv && rm -f gpurun_out/r05x_prof/run_kernel_trace.csv
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --beam "" --method c3,c4,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r05x_bench.jsonl 2> gpurun_out/r05x_bench.err || exit 4
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r05x_bench_r8.jsonl 2> gpurun_out/r05x_bench_r8.err || exit 5
