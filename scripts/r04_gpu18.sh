set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/prefetch_ab.py --shapes r8c3,r8c5 --idle-us 30 > gpurun_out/r04q_prefetch_ab.jsonl 2> gpurun_out/r04q_prefetch_ab.err || { tail -20 gpurun_out/r04q_prefetch_ab.err; exit 2; }
cat gpurun_out/r04q_prefetch_ab.jsonl
