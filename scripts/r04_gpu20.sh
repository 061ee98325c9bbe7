set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--steps 6 --warmup 2 --e2e 0 --beam '' --method-bon 0 --method-text-steps 0 --cpu-seconds 0"
for cfg in "1 1" "0 0" "1 0" "0 1"; do set -- $cfg
  CS_FOLD_IN_ROPE=$1 CS_FOLD_IN_NORM=$2 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r04s_fold_$1$2_1gpu.jsonl 2>/dev/null || exit 2
  CS_FOLD_IN_ROPE=$1 CS_FOLD_IN_NORM=$2 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r04s_fold_$1$2_r8.jsonl 2>/dev/null || exit 3
  echo "fold $1$2 done"
done
