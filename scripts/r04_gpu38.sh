#!/bin/bash
# A/B: variant 3 gated as 4 waves x 64 features per workgroup (tree) vs the 8-wave form (lib_g8)
set -o pipefail
mkdir -p gpurun_out/r04_38
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_38/tests.log 2>&1 || exit 2
for L in "" ablibs/lib_g8.so "" ablibs/lib_g8.so; do
  n=$(basename "${L:-tree}")
  timeout -k 10 240 python -u tools/gemm_ab.py --shapes c1_gu_gated,c3_gu_gated,c5_gu_gated,r8c3_gu_gated,r8c5_gu_gated --variants 2,3 --splits 0 --packed --no-torch ${L:+--lib $L} >> gpurun_out/r04_38/$n.jsonl 2> gpurun_out/r04_38/$n.err || exit 3
done
