set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tune_gemm_dispatch.py --configs c5 --variants 2,3,4 --merge 0 --out gpurun_out/r04l_dispatch_c5.json > gpurun_out/r04l_dispatch_c5.log 2>&1 || exit 2
echo "c5 ok"
