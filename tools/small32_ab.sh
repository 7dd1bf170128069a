#!/bin/bash
# 64x64 split-bf16 tiles with 32-deep K tiles (MPR_X3_SMALL_BK32 1: launches of <= 512 blocks, 2: all)
# vs 16-deep: bit-identity tests, then the serving bench with the GEMM replay, alternating.
mkdir -p gpurun_out/s32
MPR_X3_SMALL_BK32=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py -q -x \
  --timeout 250 --timeout-method thread > gpurun_out/s32/pytest.log 2>&1 || exit $?
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-c5 --no-index-build"
for i in 1 2; do
  for p in 0 1 2; do
    MPR_X3_SMALL_BK32=$p timeout -k 10 240 $B > gpurun_out/s32/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/s32/steps.log
  done
done
