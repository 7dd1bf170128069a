#!/bin/bash
# 128x128 split-bf16 tiles with / without the raised issue priority over the MFMA run
# (MPR_X3_WIDE_PRIO 1 / 0): serving bench at 40 steps with the GEMM replay, alternating.
mkdir -p gpurun_out/wprio
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-c5 --no-index-build"
for i in 1 2; do
  for p in 1 0; do
    MPR_X3_WIDE_PRIO=$p timeout -k 10 240 $B > gpurun_out/wprio/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/wprio/steps.log
  done
done
