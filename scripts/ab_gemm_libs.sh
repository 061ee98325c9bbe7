# A/B of cs_gemm_bf16 builds: bash scripts/ab_gemm_libs.sh TAG LIB [LIB...] (ablibs/<LIB>.so)
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
for L in "$@"; do
  extra="--no-torch"; [ $L = "$1" ] && extra=""
  timeout -k 10 400 python -u tools/gemm_ab.py --lib ablibs/$L.so --shapes ${SHAPES:-c3,c5,r8} --variants ${VARIANTS:-2,3,4} --splits ${SPLITS:-1,2,4,8} $extra > gpurun_out/${tag}_$L.jsonl 2> gpurun_out/${tag}_$L.err || { echo "FAIL $L"; tail -5 gpurun_out/${tag}_$L.err; exit 1; }
  echo "done $L $(wc -l < gpurun_out/${tag}_$L.jsonl)"
done
