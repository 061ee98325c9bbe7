set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/norm_block_ab.py > gpurun_out/r05l_norm_block.jsonl 2> gpurun_out/r05l_norm.err || exit 2
CS_NORM_VPT=1 timeout -k 10 200 python -u tools/norm_block_ab.py > gpurun_out/r05l_norm_vpt.jsonl 2>> gpurun_out/r05l_norm.err || exit 3
