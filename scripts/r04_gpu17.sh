set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/beam_ab.py --only c3,c5,c3nocap --knobs "CS_TARGET_WGS=512,CS_DECODE_BLOCK=1024;CS_TARGET_WGS=768,CS_DECODE_BLOCK=1024;CS_TARGET_WGS=1024,CS_DECODE_BLOCK=1024;CS_TARGET_WGS=512;CS_TARGET_WGS=512,CS_DECODE_BLOCK=1024,CS_DECODE_ROWS_FIRST=0;CS_TARGET_WGS=512,CS_DECODE_BLOCK=1024,CS_DECODE_ROWS_FIRST=1" > gpurun_out/r04p_decode_knobs.jsonl 2> gpurun_out/r04p_decode_knobs.err || exit 2
python -c "
import json
for l in open('gpurun_out/r04p_decode_knobs.jsonl'):
    d=json.loads(l); print(d['config'], {k:round(v,1) for k,v in d.items() if k.startswith('decode') or k=='lsg_k0_us'})"
