set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 --sweep > gpurun_out/r04b_beam_ab_tree.jsonl 2> gpurun_out/r04b_beam_ab_tree.err || exit 3
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5 --lib ablibs/lib_rawkeys0.so > gpurun_out/r04b_beam_ab_raw0.jsonl 2> gpurun_out/r04b_beam_ab_raw0.err || exit 4
timeout -k 10 600 python -u bench.py --e2e 0 --beam "" --method c3,c4,c5 --emulate-ranks 8 --cpu-seconds 0 --steps 3 --warmup 1 --method-text-steps 0 > gpurun_out/r04b_bench_emul8.log 2>&1 || exit 5
timeout -k 10 300 python -u tools/profile_method_host.py c1:text c3:text > gpurun_out/r04b_text_host_profile.txt 2>&1 || exit 6
echo done
