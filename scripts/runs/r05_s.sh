set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "" "--lib tools/libold.so"; do
  tag=new; [ -n "$lib" ] && tag=old
  timeout -k 10 400 python -u tools/gemm_ab.py --shapes r8c3,r8c5,c1 --splits 1,4,8 --variants 3,4 --packed --no-torch $lib > gpurun_out/r05s_gemm_$tag.jsonl 2> gpurun_out/r05s_gemm_$tag.err || exit 3
done
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam "" --method c3,c5,c1 --method-bon 0 --method-text-steps 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r05s_bench_r8.jsonl 2> gpurun_out/r05s_bench_r8.err || exit 4
