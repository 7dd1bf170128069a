#!/bin/bash
# Serving-loop A/B of host-side settings (alternating runs of the headline loop alone) and the
# C5 end-to-end leg with and without the two-slot decode of > 128-row batches.
# usage: bash tools/host_ab.sh <tag>
OUT=gpurun_out/${1:-host_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "t5_generate" -rf \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
LEAN="--no-cpu-baseline --no-probe --no-c5 --no-train-leg --no-eos-leg --no-index-build"
for i in 1 2; do
  for V in ${HOST_VARIANTS:-DEFAULT=1 MPR_LOOKAHEAD_PASSES=2}; do
    env "$V" timeout -k 10 300 python bench.py --steps 80 --warmup 4 $LEAN > "$OUT/bench_${V}_$i.json" 2> "$OUT/bench_${V}_$i.err" || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['sync_ms_per_step'], d['main_loop_ms_per_step'])" "$OUT/bench_${V}_$i.json" "$V" >> "$OUT/ab.txt"
  done
done
for V in ${C5_VARIANTS:-}; do
  env "$V" timeout -k 10 300 python -c "
import torch, bench, json
dev = torch.device('cuda:0'); torch.cuda.set_device(dev)
print('$V', json.dumps(bench.c5_serving(1, 0, dev, None, dev)))" >> "$OUT/ab.txt" 2> "$OUT/c5_$V.err" || exit $?
done
echo done >> "$OUT/steps.log"
