#!/usr/bin/env bash
# PMC passes over one GEMM shape (tools/gemm_one.py): cs_gemm variant(s) vs torch.
# usage: scripts/gemm_pmc.sh <shape> <splits> <variant|torch> [tag]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT="$R/gpurun_out/pmc_gemm"; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${4:-$1_$3}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVES TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P -d "$OUT/${TAG}_p$i" -o run -f csv -- \
     python3 "$R/tools/gemm_one.py" "$1" "$2" "$3" > "$OUT/${TAG}_p$i.log" 2>&1) || exit $?
done
