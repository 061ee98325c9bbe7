set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
for v in 1 0; do
  (cd /tmp && CS_ATTN_LDS2=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05u_prof_$v" -o run -f csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --beam "" --method "" --cpu-seconds 0 > "$R/gpurun_out/r05u_prof_$v.log" 2>&1) || exit 3
  python3 scripts/trace_by_grid.py gpurun_out/r05u_prof_$v/run_kernel_trace.csv > gpurun_out/r05u_prof_$v/by_grid.csv || exit 4
  rm -f gpurun_out/r05u_prof_$v/run_kernel_trace.csv
done
