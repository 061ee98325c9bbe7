set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c3 c5 c1; do
  V=2,3,4; [ $c = c1 ] && V=2,3,4,5,6,7
  timeout -k 10 500 python -u tools/tune_gemm_dispatch.py --configs $c --gemms qkv,down --variants $V --merge 0 --out gpurun_out/r04aa_dispatch_fold_$c.json > gpurun_out/r04aa_dispatch_fold_$c.log 2>&1 || exit 2
  echo "$c ok"
done
timeout -k 10 500 python -u tools/tune_gemm_dispatch.py --configs c4 --gemms qkv,down --variants 2,3,4 --merge 0 --out gpurun_out/r04aa_dispatch_fold_c4.json > gpurun_out/r04aa_dispatch_fold_c4.log 2>&1 || exit 3
echo "c4 ok"
