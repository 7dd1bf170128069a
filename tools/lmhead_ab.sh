#!/bin/bash
# Argmax head of grouped decodes as launches of <= MPR_LMHEAD_ROWS rows (0 = one launch), 20-step
# serving loop, alternating (development aid).
mkdir -p gpurun_out/lmab
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2; do
  for r in 0 64 32; do
    MPR_LMHEAD_ROWS=$r timeout -k 10 200 $B > gpurun_out/lmab/r${r}_$i.json 2>/dev/null || exit $?
    echo "r$r $i" >> gpurun_out/lmab/steps.log
  done
done
