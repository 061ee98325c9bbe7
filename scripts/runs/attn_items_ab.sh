set -e
mkdir -p gpurun_out/attn_items
for mi in 3 12 24 4096; do
  CS_ATTN_MIN_ITEMS=$mi timeout -k 10 240 python bench.py --steps 20 --warmup 5 --e2e 0 --method c3,c5 --method-bon 0 --method-statements 0 --method-text-steps 0 --beam "" --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/attn_items/r8_mi$mi.json 2> gpurun_out/attn_items/r8_mi$mi.err
  CS_ATTN_MIN_ITEMS=$mi timeout -k 10 240 python bench.py --steps 20 --warmup 5 --e2e 0 --method c3 --method-bon 0 --method-statements 0 --method-text-steps 0 --beam "" --cpu-seconds 0 > gpurun_out/attn_items/r1_mi$mi.json 2> gpurun_out/attn_items/r1_mi$mi.err
done
