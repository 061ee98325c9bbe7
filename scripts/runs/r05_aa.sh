set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam '' --method c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0"
for res in default 16; do
  env=""; [ $res != default ] && env="CS_GEMM_PACK_RESERVE_GB=$res"
  eval "$env timeout -k 10 400 $B --emulate-ranks 8" > gpurun_out/r05aa_c5_r8_res$res.jsonl 2> gpurun_out/r05aa_c5_r8_res$res.err || exit 3
  echo "r8 $res done"
  eval "$env timeout -k 10 500 $B" > gpurun_out/r05aa_c5_1g_res$res.jsonl 2> gpurun_out/r05aa_c5_1g_res$res.err || exit 4
  echo "1g $res done"
done
