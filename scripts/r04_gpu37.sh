#!/bin/bash
# A/B: four-stage ws2 pipeline for the <= 9-tile row blocks (tree) vs three stages (lib_d3)
set -o pipefail
mkdir -p gpurun_out/r04_37
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_37/tests.log 2>&1 || exit 2
for L in "" ablibs/lib_d3.so "" ablibs/lib_d3.so; do
  n=$(basename "${L:-tree}")
  timeout -k 10 240 python -u tools/gemm_ab.py --shapes c1,c3,c5,r8 --variants 2,3,4 --splits 0 --packed --no-torch ${L:+--lib $L} >> gpurun_out/r04_37/$n.jsonl 2> gpurun_out/r04_37/$n.err || exit 3
done
