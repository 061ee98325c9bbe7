set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CS_GEMM_PACK_RESERVE_GB=16 timeout -k 10 600 python -u bench.py > gpurun_out/r05ab_bench_res16.jsonl 2> gpurun_out/r05ab_bench_res16.err || exit 3
echo "default bench done"
CS_GEMM_PACK_RESERVE_GB=16 timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --e2e 0 --beam '' --method c5,c3 --method-bon 0 --cpu-seconds 0 --emulate-ranks 8 > gpurun_out/r05ab_r8_res16.jsonl 2> gpurun_out/r05ab_r8_res16.err || exit 4
echo "r8 done"
