set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh prof || { echo "prof failed"; tail -5 gpurun_out/prof.log; exit 2; }
echo "prof ok"
bash scripts/gpu_check.sh pmc || { echo "pmc failed"; exit 3; }
echo "pmc ok"
