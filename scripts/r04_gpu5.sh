set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_gpu_tests.log 2>&1 || { echo "tests failed"; exit 2; }
echo "tests ok"
timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r04e_bench_c4_tunedcsv.jsonl 2> gpurun_out/r04e_bench_c4_tunedcsv.err || exit 3
echo "c4 bench (tuned csv) ok"
timeout -k 10 600 python -u tools/tune_gemm_dispatch.py --configs c4 --out gpurun_out/r04e_gemm_dispatch_c4.json --install > gpurun_out/r04e_gemm_dispatch_c4.log 2>&1 || exit 4
echo "dispatch c4 ok"
timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r04e_bench_c4_dispatch.jsonl 2> gpurun_out/r04e_bench_c4_dispatch.err || exit 5
echo done
