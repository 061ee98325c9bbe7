set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 > gpurun_out/r04d_beam_ab_tree.jsonl 2> gpurun_out/r04d_beam_ab_tree.err || exit 3
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 --lib ablibs/lib_prev.so > gpurun_out/r04d_beam_ab_prev.jsonl 2> gpurun_out/r04d_beam_ab_prev.err || exit 4
timeout -k 10 300 python -u tools/gemm_ab.py --shapes c5_qkv,c5_gu,c5_lmhead --variants 2 --splits 0,-1 --no-torch > gpurun_out/r04d_gemm_sk_ab.jsonl 2> gpurun_out/r04d_gemm_sk_ab.err || exit 5
timeout -k 10 1800 python -u tools/tune_gemms.py --legs c4 --out gpurun_out/gemm_tuned_c4.csv > gpurun_out/r04d_tune_c4.log 2>&1 || exit 6
echo done
