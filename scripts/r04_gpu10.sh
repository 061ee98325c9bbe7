set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -q -k "pack" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k_pack_tests.log 2>&1 || { echo "pack tests failed"; tail -30 gpurun_out/r04k_pack_tests.log; exit 2; }
echo "pack tests ok"
timeout -k 10 500 python -u tools/gemm_ab.py --shapes r8c3,r8c5,c3,c5,c1 --variants 3,2,4 --splits 0 --packed --no-torch > gpurun_out/r04k_gemm_packed_ab.jsonl 2> gpurun_out/r04k_gemm_packed_ab.err || exit 3
echo done
