set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1; grep FAILED gpurun_out/gpu_tests.log | head
