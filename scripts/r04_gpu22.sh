set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/tune_gemm_dispatch.py --configs c4 --worlds 2,4 --variants 2,3,4 --merge 0 --out gpurun_out/r04w_dispatch_c4_w24.json > gpurun_out/r04w_dispatch_c4_w24.log 2>&1 || exit 2
echo "c4 w24 ok"
