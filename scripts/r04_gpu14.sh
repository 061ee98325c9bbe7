set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_gemm_gpu.py tests/test_bf16_traces_gpu.py tests/test_methods_gpu.py tests/test_sharded_fast_gpu.py tests/test_lookahead_stream_gpu.py -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r04m_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04m_tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c1,c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r04m_bench_methods.jsonl 2> gpurun_out/r04m_bench_methods.err || exit 3
echo "bench 1gpu ok"
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r04m_bench_r8.jsonl 2> gpurun_out/r04m_bench_r8.err || exit 4
echo done
