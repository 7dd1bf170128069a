#!/bin/bash
# PMC passes over one x3 GEMM tile on one x3bench shape (development aid).
# usage: bash tools/x3_pmc.sh <tag> <shape> <kernel-regex>
TAG=${1:-x3pmc}; SH=${2:-2}; RE=${3:-gemm_x3_kernel<128, 128, 2, 1, 16, 2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$R/tools/x3bench" $SH > "$OUT/x3bench.txt" 2>&1 || exit $?
i=0
for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "$RE" \
    -d "$OUT/pmc$i" -o p --output-format csv -- "$R/tools/x3bench" $SH \
    > "$OUT/pmc$i.log" 2>&1 || exit $?
done
