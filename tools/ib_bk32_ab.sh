#!/bin/bash
# Index build rows/s with and without the 32-deep 128x128 tiles (MPR_X3_BK32 0 / 1), alternating.
mkdir -p gpurun_out/ibk
for i in 1 2; do
  for p in 0 1; do
    MPR_X3_BK32=$p timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe --no-c5 \
      > gpurun_out/ibk/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/ibk/steps.log
  done
done
