#!/bin/bash
# Serving-loop knobs at the bench's default 80 steps: default / MPR_SKINNY_ROWS=32 /
# MPR_DECODE_GROUP=6, alternating (development aid).
mkdir -p gpurun_out/fk
B="python bench.py --steps 80 --warmup 4 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2; do
  timeout -k 10 240 $B > gpurun_out/fk/base_$i.json 2>/dev/null || exit $?
  MPR_SKINNY_ROWS=32 timeout -k 10 240 $B > gpurun_out/fk/r32_$i.json 2>/dev/null || exit $?
  MPR_DECODE_GROUP=6 timeout -k 10 240 $B > gpurun_out/fk/g6_$i.json 2>/dev/null || exit $?
  echo "round $i" >> gpurun_out/fk/steps.log
done
