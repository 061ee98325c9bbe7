set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/beam_ab.py --only r8c3,r8c5,c3,c5 --blocks > gpurun_out/r04h_decode_blocks_ab.jsonl 2> gpurun_out/r04h_decode_blocks_ab.err || exit 2
echo "ab ok"
CS_DECODE_BLOCK=1024 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k "decode" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04h_decode_block1024_tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/r04h_decode_block1024_tests.log
