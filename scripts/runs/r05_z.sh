set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_stream_attention_gpu.py tests/test_hist_rows_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05z_attn_tests.log 2>&1 || { tail -30 gpurun_out/r05z_attn_tests.log; exit 9; }
for lib in tree merge0; do
  extra=""; [ $lib = merge0 ] && extra="--lib $R/tools/libcs_merge0.so"
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05z_$lib" -o run -f csv -- python3 "$R/tools/attn_bench.py" c3r8 c5r8 c3 c5 c1 $extra > "$R/gpurun_out/r05z_$lib.log" 2>&1) || exit 3
  rm -f "$R/gpurun_out/r05z_$lib"/*/run_kernel_trace.csv "$R/gpurun_out/r05z_$lib"/run_kernel_trace.csv
done
