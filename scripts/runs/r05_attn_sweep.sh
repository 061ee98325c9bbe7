set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out/r05c_attn_sweep
mkdir -p $OUT
for tw in 512 1024 2048; do for mi in 1 2 3; do
  d=$OUT/tw${tw}_mi${mi}
  (cd /tmp && CS_ATTN_TARGET_WGS=$tw CS_ATTN_MIN_ITEMS=$mi timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run -f csv -- python3 "$R/tools/attn_bench.py" "c3r8=2,210,1700,16,1,16,8,256,25,50" "c5r8=8,210,5500,8,1,64,8,128,25,0" "c3=16,210,1700,16,1,16,8,256,25,50" "c5=64,210,5500,8,1,64,8,128,25,0" > $d.log 2>&1) || exit 3
  python3 scripts/trace_by_grid.py $d/run_kernel_trace.csv | grep -i "attn" > $d.csv || exit 4
  rm -rf $d
done; done
