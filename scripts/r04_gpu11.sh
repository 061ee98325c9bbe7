set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/tune_gemm_dispatch.py --configs c3 --variants 2,3,4 --merge 0 --out gpurun_out/r04l_dispatch_c3.json > gpurun_out/r04l_dispatch_c3.log 2>&1 || exit 2
echo "c3 ok"
timeout -k 10 300 python -u tools/tune_gemm_dispatch.py --configs c1 --variants 2,3,4,5,6,7 --merge 0 --out gpurun_out/r04l_dispatch_c1.json > gpurun_out/r04l_dispatch_c1.log 2>&1 || exit 3
echo "c1 ok"
