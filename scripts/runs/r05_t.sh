set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stream_attention_gpu.py tests/test_hist_rows_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05t_attn_tests.log 2>&1 || { tail -30 gpurun_out/r05t_attn_tests.log; exit 2; }
tail -2 gpurun_out/r05t_attn_tests.log
for v in 1 0; do
CS_ATTN_LDS2=$v timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --beam "" --method "" --cpu-seconds 0 > gpurun_out/r05t_bench_lds2_$v.jsonl 2> gpurun_out/r05t_bench_lds2_$v.err || exit 3
done
