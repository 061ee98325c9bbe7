set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_ab.py --shapes r8c3,r8c5 --variants 3,4 --splits 0 > gpurun_out/r04f_gemm_r8_cold.jsonl 2> gpurun_out/r04f_gemm_r8_cold.err || exit 2
timeout -k 10 300 python -u tools/gemm_ab.py --shapes r8c3,r8c5 --variants 3,4 --splits 0 --warm > gpurun_out/r04f_gemm_r8_warm.jsonl 2> gpurun_out/r04f_gemm_r8_warm.err || exit 3
echo "gemm ab ok"
EMULATE=8 bash scripts/prof_method.sh c3 c5 || exit 4
bash scripts/prof_method.sh c4 || exit 5
echo done
