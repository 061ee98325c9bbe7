# GPU tests + smoke + default bench (+ the beam A/B); every GPU step under its own limit
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/${T}_gpu_tests.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; exit 3; }
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.jsonl 2> gpurun_out/${T}_bench.err || { echo bench failed; exit 4; }
timeout -k 10 300 python -u tools/beam_ab.py > gpurun_out/${T}_beam_ab.jsonl 2> gpurun_out/${T}_beam_ab.err || exit 5
