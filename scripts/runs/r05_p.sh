set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 6 --warmup 2 --e2e 0 --beam '' --method-bon 0 --method-text-steps 0 --cpu-seconds 0"
for cfg in "512 3" "1024 3" "1024 2" "2048 2" "2048 1" "4096 1"; do
  set -- $cfg
  CS_ATTN_TARGET_WGS=$1 CS_ATTN_MIN_ITEMS=$2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r05p_attn_t$1_m$2.jsonl 2> gpurun_out/r05p_attn_t$1_m$2.err || exit 3
  echo "done $1 $2"
done
