set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04g_gemm_tests.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/r04g_gemm_tests.log; exit 2; }
echo "gemm tests ok"
timeout -k 10 400 python -u tools/gemm_ab.py --shapes r8c3,r8c5,c1 --variants 5,6,7 --splits 0 > gpurun_out/r04g_gemm_thin_cold.jsonl 2> gpurun_out/r04g_gemm_thin_cold.err || exit 3
echo done
