set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/gemm_ab.py --shapes c5_qkv,c5_gu,c5_down,c5_o,c3_qkv,c3_gu,c3_down,c5_lmhead --variants 2 --splits 0,-1 > gpurun_out/r04c_gemm_sk_ab.jsonl 2> gpurun_out/r04c_gemm_sk_ab.err || exit 3
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 > gpurun_out/r04c_beam_ab_tree.jsonl 2> gpurun_out/r04c_beam_ab_tree.err || exit 4
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 --lib ablibs/lib_prio0.so > gpurun_out/r04c_beam_ab_prio0.jsonl 2> gpurun_out/r04c_beam_ab_prio0.err || exit 5
timeout -k 10 200 python -u tools/beam_trace.py > gpurun_out/r04c_beam_trace.jsonl 2> gpurun_out/r04c_beam_trace.err || exit 6
timeout -k 10 600 python -u bench.py --e2e 0 --beam "" --method c1,c3,c5 --cpu-seconds 0 --steps 3 --warmup 1 > gpurun_out/r04c_bench_text.log 2>&1 || exit 7
bash scripts/prof_method.sh c4 || exit 8
echo done
