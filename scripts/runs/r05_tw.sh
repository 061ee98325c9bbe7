set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for tw in 256 384 512 1024; do
  CS_TARGET_WGS=$tw timeout -k 10 200 python -u tools/beam_ab.py --only c3,c5,c3nocap > gpurun_out/r05i_tw$tw.jsonl 2> gpurun_out/r05i_tw$tw.err || exit 3
done
