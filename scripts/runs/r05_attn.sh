set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_bench.py c1 c3 c5 "c3r8=2,210,1700,16,1,16,8,256,25,50" "c5r8=8,210,5500,8,1,64,8,128,25,0" "c3r8g5=2,210,1700,16,1,16,8,256,5,50" "c5r8g5=8,210,5500,8,1,64,8,128,5,0" "c3r8np=2,210,0,16,1,16,8,256,25,50" > gpurun_out/r05a_attn.jsonl 2> gpurun_out/r05a_attn.err
