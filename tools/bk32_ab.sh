#!/bin/bash
# 128x128 split-bf16 tiles with 32-deep K tiles for launches of <= 256 blocks (MPR_X3_BK32=1) vs
# 16-deep: bit-identity tests, then the serving bench with the GEMM replay, alternating.
mkdir -p gpurun_out/bk32b
MPR_X3_BK32=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py -q -x \
  --timeout 250 --timeout-method thread > gpurun_out/bk32b/pytest.log 2>&1 || exit $?
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-c5 --no-index-build"
for i in 1 2; do
  for p in 1 2; do
    MPR_X3_BK32=$p timeout -k 10 240 $B > gpurun_out/bk32b/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/bk32b/steps.log
  done
done
