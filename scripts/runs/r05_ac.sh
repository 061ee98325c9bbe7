set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05ac_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r05ac_gemm_tests.log; exit 9; }
tail -2 gpurun_out/r05ac_gemm_tests.log
for i in 1 2; do
timeout -k 10 200 python -u tools/gemm_ab.py --shapes r8c5_gu_gated,r8c3_gu_gated --variants 2,4 --packed --no-torch > gpurun_out/r05ac_g7on_$i.jsonl 2> gpurun_out/r05ac_g7on_$i.err || exit 3
timeout -k 10 200 python -u tools/gemm_ab.py --shapes r8c5_gu_gated,r8c3_gu_gated --variants 2,4 --packed --no-torch --lib $R/tools/libcs_g7off.so > gpurun_out/r05ac_g7off_$i.jsonl 2> gpurun_out/r05ac_g7off_$i.err || exit 4
done
