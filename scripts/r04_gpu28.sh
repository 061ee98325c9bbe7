set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stream_attention_gpu.py tests/test_prefix_reuse.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04ac_attn_tests.log 2>&1 || { tail -20 gpurun_out/r04ac_attn_tests.log; exit 2; }
echo "attn tests ok"; tail -1 gpurun_out/r04ac_attn_tests.log
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r04ac_attn_pd2.jsonl 2> gpurun_out/r04ac_attn_pd2.err || exit 3
timeout -k 10 300 python -u tools/attn_bench.py --lib ablibs/lib_pd1.so > gpurun_out/r04ac_attn_pd1.jsonl 2> gpurun_out/r04ac_attn_pd1.err || exit 4
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r04ac_attn_pd2b.jsonl 2>/dev/null || exit 5
paste -d'\n' gpurun_out/r04ac_attn_pd1.jsonl gpurun_out/r04ac_attn_pd2.jsonl gpurun_out/r04ac_attn_pd2b.jsonl
