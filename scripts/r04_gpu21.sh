set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "512 3" "256 3" "1024 3" "512 1" "512 6" "1024 1"; do set -- $cfg
  CS_ATTN_TARGET_WGS=$1 CS_ATTN_MIN_ITEMS=$2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r04v_attn_$1_$2.jsonl 2>/dev/null || exit 2
  echo "attn $1 $2 done"
done
