#!/bin/bash
# Decode GEMV row blocks of 16 (default) vs 32 (MPR_SKINNY_ROWS=32) at the bench's 80 steps,
# alternating (development aid).
mkdir -p gpurun_out/fk2
B="python bench.py --steps 80 --warmup 4 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2 3; do
  timeout -k 10 240 $B > gpurun_out/fk2/base_$i.json 2>/dev/null || exit $?
  MPR_SKINNY_ROWS=32 timeout -k 10 240 $B > gpurun_out/fk2/r32_$i.json 2>/dev/null || exit $?
  echo "round $i" >> gpurun_out/fk2/steps.log
done
