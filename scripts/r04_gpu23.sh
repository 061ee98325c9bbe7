set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stream_attention_gpu.py -m gpu -q -k "gather" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x_gather_tests.log 2>&1 || { tail -20 gpurun_out/r04x_gather_tests.log; exit 2; }
echo "gather tests ok"
timeout -k 10 400 python -u tools/hist_gather_ab.py > gpurun_out/r04x_hist_gather_ab.jsonl 2> gpurun_out/r04x_hist_gather_ab.err || exit 3
cat gpurun_out/r04x_hist_gather_ab.jsonl
