#!/bin/bash
# Unhinted predict(): token-feature ViT deferred behind the retrieval towers (1) vs the paired
# pass (0): GPU tests, then bench sync_ms_per_step, alternating (development aid).
mkdir -p gpurun_out/defer
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 250 --timeout-method thread \
  > gpurun_out/defer/pytest.log 2>&1 || exit $?
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
for i in 1 2; do
  for p in 0 1; do
    MPR_PREDICT_DEFER_TOKENS=$p timeout -k 10 240 $B > gpurun_out/defer/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/defer/steps.log
  done
done
