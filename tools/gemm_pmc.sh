#!/bin/bash
# PMC passes over one x3pbench shape / variant (tools/x3pbench.hip): SQ issue / wait / MFMA-busy
# counters, LDS and vector-memory instruction counts, the effective clock (GRBM_GUI_ACTIVE).
# usage: bash tools/gemm_pmc.sh <out dir> <shape substring> <variant substring> [launches]
OUT=$1; SH=$2; VAR=$3; N=${4:-500}
mkdir -p "$OUT"
export TMPDIR=/tmp
RE="gemm_x3p_kernel"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
P3="SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CU_CYCLES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "$RE" -d "$OUT/p$i" -o run \
    --output-format csv -- ./tools/x3pbench "$SH" "$VAR" "$N" > "$OUT/p$i.log" 2>&1 || exit 1
done
python3 tools/pmc_traffic.py --sum "$OUT" > "$OUT/summary.txt"
