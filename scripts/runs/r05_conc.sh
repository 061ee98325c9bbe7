set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/graph_concurrency.py > gpurun_out/r05j_conc.jsonl 2> gpurun_out/r05j_conc.err || exit 3
