set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh tests; echo "tests rc=$?"; tail -3 gpurun_out/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
echo "smoke ok"
bash scripts/gpu_check.sh bench || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log | cut -c1-300
