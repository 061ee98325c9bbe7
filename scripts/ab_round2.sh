mkdir -p gpurun_out && rm -f gpurun_out/rope_ab.jsonl gpurun_out/attn_d256.jsonl gpurun_out/attn_plan.jsonl
for sw in 0 1; do for vt in 0 1; do CS_ROPE_SWIZZLE=$sw CS_ROPE_VTILE=$vt timeout -k 10 120 python -u tools/rope_bench.py >> gpurun_out/rope_ab.jsonl 2>>gpurun_out/rope.err || exit 1; done; done
for v in 0 1; do CS_ATTN_LDS=$v timeout -k 10 120 python -u tools/attn_bench.py "g3s=16,210,0,16,50,16,8,256,0,50" "g3p=1,0,0,17,256,16,8,256,0,50" "l8p=1,0,0,17,256,32,8,128,0,0" "l1s=4,210,0,4,50,32,8,64,0,0" >> gpurun_out/attn_d256.jsonl 2>>gpurun_out/attn.err || exit 1; done
for v in 0 1; do CS_ATTN_PLAN_LDS=$v timeout -k 10 120 python -u tools/attn_bench.py c1 c3 c5 >> gpurun_out/attn_plan.jsonl 2>>gpurun_out/attn.err || exit 1; done
CS_ATTN_PLAN_LDS=1 timeout -k 10 200 python -u -m pytest tests/test_stream_attention_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread --capture=tee-sys > gpurun_out/t_planlds.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_methods_gpu.py tests/test_stream_attention_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread --capture=tee-sys > gpurun_out/t_reuse.log 2>&1
