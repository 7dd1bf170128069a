#!/bin/bash
# 64x128 split-bf16 launches with extra dynamic LDS (MPR_TALL_PAD bytes) so that no decode GEMV
# block fits beside one on a CU, vs none: serving bench, alternating (development aid).
mkdir -p gpurun_out/tp
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-c5 --no-index-build"
for i in 1 2; do
  for p in 0 36864; do
    MPR_TALL_PAD=$p timeout -k 10 240 $B > gpurun_out/tp/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/tp/steps.log
  done
done
