set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/r05b_attn_prof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05b_attn_prof" -o run -f csv -- python3 "$R/tools/attn_bench.py" "c3r8=2,210,1700,16,1,16,8,256,25,50" "c5r8=8,210,5500,8,1,64,8,128,25,0" "c3r8np=2,210,0,16,1,16,8,256,25,50" > "$R/gpurun_out/r05b_attn_prof.log" 2>&1
cd "$R" && python3 scripts/trace_by_grid.py gpurun_out/r05b_attn_prof/run_kernel_trace.csv > gpurun_out/r05b_attn_prof/by_grid.csv && rm -f gpurun_out/r05b_attn_prof/run_kernel_trace.csv
