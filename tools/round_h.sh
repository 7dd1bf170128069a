#!/bin/bash
# One GPU call: coarse-kernel and tower-graph checks and A/Bs.
#  1. coarse tests with 128-deep stages, timing of 64 vs 128 (tools/scan_ab.sh);
#  2. the tower-graph bit-identity test and the serving loop with / without tower graphs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_h
mkdir -p "$OUT"
MPR_COARSE_BK=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_kernels.py -q -m gpu \
  -k "coarse or c5 or scan_topk" -rf --timeout 200 --timeout-method thread > "$OUT/pytest_bk128.log" 2>&1
rc=$?; echo "pytest bk128 rc=$rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "tower_graphs or encode_towers" \
  -rf --timeout 200 --timeout-method thread > "$OUT/pytest_graphs.log" 2>&1
rc=$?; echo "pytest graphs rc=$rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
VARIANTS="MPR_COARSE_BK=128 DEFAULT=1" bash tools/scan_ab.sh r03_scan4 || exit $?
HOST_VARIANTS="DEFAULT=1 MPR_TOWER_GRAPHS=1 MPR_LOOKAHEAD_PASSES=2" bash tools/host_ab.sh r03_hostab2 || exit $?
echo done >> "$OUT/steps.log"
