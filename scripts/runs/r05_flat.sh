set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
S="c1 c3 c5 c3r8=2,210,1700,16,1,16,8,256,25,50 c5r8=8,210,5500,8,1,64,8,128,25,0 c3r8np=2,210,0,16,1,16,8,256,25,50 c3g50=16,210,1700,16,1,16,8,256,50,50 c5r8g50=8,210,5500,8,1,64,8,128,50,0"
timeout -k 10 300 python -u -m pytest tests/test_stream_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05g_attn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05g_attn_tests.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 200 python -u tools/attn_bench.py $S > gpurun_out/r05g_attn_new.jsonl 2> gpurun_out/r05g_attn_new.err || exit 3
timeout -k 10 200 python -u tools/attn_bench.py --lib tools/libold.so $S > gpurun_out/r05g_attn_old.jsonl 2> gpurun_out/r05g_attn_old.err || exit 4
timeout -k 10 200 python -u tools/attn_trace.py tools/libattn_trace.so "c3r8=2,210,1700,16,1,16,8,256,25,50" "c5r8=8,210,5500,8,1,64,8,128,25,0" "c3r8np=2,210,0,16,1,16,8,256,25,50" > gpurun_out/r05g_attn_trace.jsonl 2> gpurun_out/r05g_attn_trace.err || exit 5
