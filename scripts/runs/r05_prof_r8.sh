set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
EMULATE=8 bash scripts/prof_method.sh c3 c5 || exit 3
