set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r05r_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/r05r_gpu_tests.log
[ $rc -eq 0 ] || exit 2
for fm in 1 0; do
CS_ATTN_FUSED_MERGE=$fm timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r05r_bench_1g_fm$fm.jsonl 2> gpurun_out/r05r_bench_1g_fm$fm.err || exit 3
CS_ATTN_FUSED_MERGE=$fm timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r05r_bench_r8_fm$fm.jsonl 2> gpurun_out/r05r_bench_r8_fm$fm.err || exit 4
done
