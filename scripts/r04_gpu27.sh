set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_bf16_traces_gpu.py tests/test_methods_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04ab_tests.log 2>&1 || { tail -20 gpurun_out/r04ab_tests.log; exit 2; }
echo "tests ok"; tail -1 gpurun_out/r04ab_tests.log
for t in new old; do
  if [ $t = old ]; then export CS_GEMM_DISPATCH=ablibs/old_table.json; else unset CS_GEMM_DISPATCH; fi
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c4 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r04ab_r8_$t.jsonl 2>/dev/null || exit 3
  timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c1,c3,c5 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 > gpurun_out/r04ab_1gpu_$t.jsonl 2>/dev/null || exit 4
  echo "$t done"
done
