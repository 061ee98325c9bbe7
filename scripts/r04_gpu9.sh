set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lsg_persist_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04i_lsg_persist_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r04i_lsg_persist_tests.log; exit 2; }
echo "tests ok"
timeout -k 10 400 python -u tools/lsg_variants.py 76800 128256 8 > gpurun_out/r04i_lsg_variants_c2.jsonl 2> gpurun_out/r04i_lsg_variants_c2.err || exit 3
cat gpurun_out/r04i_lsg_variants_c2.jsonl
