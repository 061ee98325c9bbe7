#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04_35
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_dispatch_host.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_35/tests.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/gemm_ab.py --shapes r8c5,r8c3 --variants 3 --splits 0 --packed --no-torch > gpurun_out/r04_35/tree.jsonl 2> gpurun_out/r04_35/tree.err
