#!/bin/bash
# Stream priorities (MPR_STREAM_PRIO gen / none / enc) re-measured after the r02 kernel changes:
# serving bench at 40 steps, alternating (development aid).
mkdir -p gpurun_out/prio
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2; do
  for p in gen none enc; do
    MPR_STREAM_PRIO=$p timeout -k 10 240 $B > gpurun_out/prio/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/prio/steps.log
  done
done
