#!/bin/bash
# Pooled last tower block (CLS / EOT rows only) vs the full block: GPU tests, then the serving
# loop and the index build, alternating (development aid).
mkdir -p gpurun_out/pool
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 250 --timeout-method thread \
  > gpurun_out/pool/pytest.log 2>&1 || exit $?
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-probe --no-c5"
for i in 1 2; do
  for p in 0 1; do
    MPR_POOL_LAST=$p timeout -k 10 240 $B > gpurun_out/pool/p${p}_$i.json 2>/dev/null || exit $?
    echo "p$p $i" >> gpurun_out/pool/steps.log
  done
done
