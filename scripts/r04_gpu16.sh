set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
CS_GEMM_PACK=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --beam "" --method "" --cpu-seconds 0 > gpurun_out/r04o_e2e_pack0_$r.jsonl 2>/dev/null || exit 2
CS_GEMM_PACK=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --beam "" --method "" --cpu-seconds 0 > gpurun_out/r04o_e2e_pack1_$r.jsonl 2>/dev/null || exit 3
done
for f in gpurun_out/r04o_e2e_pack*.jsonl; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), round(d['end_to_end']['model_tflops_per_s'],1))"; done
