set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 > gpurun_out/r04c_beam_ab_tree.jsonl 2> gpurun_out/r04c_beam_ab_tree.err || exit 3
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 --lib ablibs/lib_prio0.so > gpurun_out/r04c_beam_ab_prio0.jsonl 2> gpurun_out/r04c_beam_ab_prio0.err || exit 4
timeout -k 10 600 python -u bench.py --e2e 0 --beam "" --method c1,c3,c5 --cpu-seconds 0 --steps 3 --warmup 1 > gpurun_out/r04c_bench_text.log 2>&1 || exit 5
bash scripts/prof_method.sh c4 || exit 6
echo done
