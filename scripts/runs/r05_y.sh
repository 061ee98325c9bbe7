set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "512 3" "256 3" "384 3" "512 5" "256 6"; do
  set -- $cfg
  CS_ATTN_TARGET_WGS=$1 CS_ATTN_MIN_ITEMS=$2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r05y_attn_t$1_m$2.jsonl 2> gpurun_out/r05y_attn_t$1_m$2.err || exit 3
  CS_ATTN_TARGET_WGS=$1 CS_ATTN_MIN_ITEMS=$2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r05y_attn_r8_t$1_m$2.jsonl 2> gpurun_out/r05y_attn_r8_t$1_m$2.err || exit 4
  echo "done $1 $2"
done
