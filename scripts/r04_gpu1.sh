set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04a_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --e2e 0 --beam "" --method c1,c3,c5 --cpu-seconds 0 --steps 3 --warmup 1 > gpurun_out/r04a_bench_text.log 2>&1
echo "bench rc=$?"
