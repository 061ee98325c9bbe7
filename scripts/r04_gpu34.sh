#!/bin/bash
# A/B: ws2 with 5-row-tile instantiation + two workgroups per CU (tree) vs HEAD vs MT5 at one WG/CU
set -o pipefail
mkdir -p gpurun_out/r04_34
for L in "" ablibs/lib_head.so ablibs/lib_occ1.so; do
  n=$(basename "${L:-tree}")
  timeout -k 10 240 python -u tools/gemm_ab.py --shapes r8c5,r8c3 --variants 2,3,4 --splits 0,2,4,8 --packed --no-torch ${L:+--lib $L} > gpurun_out/r04_34/$n.jsonl 2> gpurun_out/r04_34/$n.err || exit $?
done
