#!/bin/bash
# Serving-loop knobs after the row-split GEMVs: decode group, calls in flight, argmax head launch
# rows; 40 steps, alternating (development aid).
mkdir -p gpurun_out/gab
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/gab/base_$i.json 2>/dev/null || exit $?
  MPR_LMHEAD_ROWS=0 timeout -k 10 200 $B > gpurun_out/gab/head0_$i.json 2>/dev/null || exit $?
  MPR_DECODE_GROUP=4 timeout -k 10 200 $B > gpurun_out/gab/g4_$i.json 2>/dev/null || exit $?
  MPR_DECODE_GROUP=6 timeout -k 10 200 $B > gpurun_out/gab/g6_$i.json 2>/dev/null || exit $?
  timeout -k 10 200 $B --inflight 3 > gpurun_out/gab/if3_$i.json 2>/dev/null || exit $?
  MPR_TOWER_SLOTS=2 timeout -k 10 200 $B > gpurun_out/gab/ts2_$i.json 2>/dev/null || exit $?
  echo "round $i" >> gpurun_out/gab/steps.log
done
