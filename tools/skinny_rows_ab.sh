#!/bin/bash
# Grouped-decode GEMVs with rows split over blocks (MPR_SKINNY_ROWS 16 / 32; 0 = all rows in one
# block column): bit-identity tests under each split, then the 20-step serving loop, alternating.
mkdir -p gpurun_out/skr
T="python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_kernels.py tests/test_gpu_eos_stop.py -q -x --timeout 250 --timeout-method thread"
for r in 32 16; do
  MPR_SKINNY_ROWS=$r timeout -k 10 400 $T > gpurun_out/skr/pytest_$r.log 2>&1 || exit $?
done
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2; do
  for r in 0 32 16; do
    MPR_SKINNY_ROWS=$r timeout -k 10 200 $B > gpurun_out/skr/r${r}_$i.json 2>/dev/null || exit $?
    echo "r$r $i" >> gpurun_out/skr/steps.log
  done
done
