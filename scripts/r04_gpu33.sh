set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_gemm_fetch" -o run -f csv -- python3 "$R/tools/gemm_ab.py" --shapes r8c5_gu_gated,r8c3_gu_gated --variants 3 --splits 0 --packed --no-torch > "$R/gpurun_out/pmc_gemm_fetch.log" 2>&1) || exit 2
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_gemm_write" -o run -f csv -- python3 "$R/tools/gemm_ab.py" --shapes r8c5_gu_gated,r8c3_gu_gated --variants 3 --splits 0 --packed --no-torch > "$R/gpurun_out/pmc_gemm_write.log" 2>&1) || exit 3
echo ok
