set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_trace.py tools/libattn_trace.so "c3r8=2,210,1700,16,1,16,8,256,25,50" "c5r8=8,210,5500,8,1,64,8,128,25,0" "c3r8np=2,210,0,16,1,16,8,256,25,50" "c5r8np=8,210,0,8,1,64,8,128,25,0" "c3=16,210,1700,16,1,16,8,256,25,50" > gpurun_out/r05d_attn_trace.jsonl 2> gpurun_out/r05d_attn_trace.err
