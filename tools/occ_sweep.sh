#!/bin/bash
# GPU box: serving bench over GEMM LDS reservation (blocks per CU) x small-LDS decode GEMVs x
# decode group size.  Each run has its own time limit; the first failure ends the sweep.
# usage: bash tools/occ_sweep.sh <tag>   (CFGS="lds small group;..." overrides the list)
TAG=${1:-occ}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
IFS=';' read -r -a RUNS <<< "${CFGS:-0 0 4;41 0 4;0 1 4;41 1 4;41 1 2;0 1 2;41 0 2}"
for cfg in "${RUNS[@]}"; do
  set -- $cfg
  MPR_GEMM_LDS_KB=$1 MPR_SKINNY_SMALL=$2 MPR_DECODE_GROUP=$3 timeout -k 10 300 python bench.py \
    --no-cpu-baseline --no-c5 --no-index-build --no-probe \
    > "$OUT/b_$1_$2_$3.json" 2> "$OUT/b_$1_$2_$3.err" || exit $?
done
