set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hist_rows_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05m_rows_tests.log 2>&1; rc=$?
echo "rows tests rc=$rc"; tail -15 gpurun_out/r05m_rows_tests.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05m_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r05m_gpu_tests.log
[ $rc -eq 0 ] || exit 3
B="python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam '' --method c3,c5,c1 --method-bon 0 --method-text-steps 0 --cpu-seconds 0"
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c1 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r05m_bench_rows.jsonl 2> gpurun_out/r05m_bench_rows.err || exit 4
CS_HIST_COPY=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c1 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r05m_bench_copy.jsonl 2> gpurun_out/r05m_bench_copy.err || exit 5
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r05m_bench_rows_r8.jsonl 2> gpurun_out/r05m_bench_rows_r8.err || exit 6
