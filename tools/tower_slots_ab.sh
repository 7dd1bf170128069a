#!/bin/bash
# Serving loop with 1 vs 2 tower passes in flight (MPR_TOWER_SLOTS), 20 steps, alternating
# (development aid).
mkdir -p gpurun_out/tsab
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2 3; do
  for t in 1 2; do
    MPR_TOWER_SLOTS=$t timeout -k 10 200 $B > gpurun_out/tsab/t${t}_$i.json 2>/dev/null || exit $?
    echo "t$t $i" >> gpurun_out/tsab/steps.log
  done
done
