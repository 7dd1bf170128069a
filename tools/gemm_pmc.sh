#!/bin/bash
# GPU box: tiled-GEMM timing sweep (tools/gbench) + SQ counter passes on one shape/variant.
# usage: bash tools/gemm_pmc.sh <tag> [shape variant groups]
TAG=${1:-gpmc}
SH=${2:-2}; VA=${3:-0}; GR=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 "$R/tools/gbench" > "$R/$OUT/gbench.txt" 2>&1 || exit $?
i=0
for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc $c --kernel-include-regex "gemm_f32_kernel" \
    -d "$R/$OUT/pmc$i" -o p --output-format csv -- "$R/tools/gbench" $SH $VA $GR \
    > "$R/$OUT/pmc$i.log" 2>&1 || exit $?
done
