#!/bin/bash
# C5 coarse-scan probe (development aid): coarse-path tests, search timings (fused / unfused
# select+rerank, 1M and 131k rows, 128 and 256 queries), kernel stats, and one FETCH_SIZE pass
# over scan_bf_kernel.  usage: bash tools/c5_probe.sh <outdir under gpurun_out>
OUT=gpurun_out/${1:-c5p}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_configs.py -k "scan or coarse" tests/test_gpu_kernels.py tests/test_gpu_sharded.py \
  > "$OUT/tests.log" 2>&1 || exit $?
for a in "1 256" "8 256" "1 128"; do
  timeout -k 10 60 python tools/scan_c5.py $a >> "$OUT/t.log" 2>&1 || exit $?
done
for a in "1 256" "8 256"; do
  MPR_COARSE_UNFUSED=1 timeout -k 10 60 python tools/scan_c5.py $a >> "$OUT/t.log" 2>&1 || exit $?
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof1" -o run -- python tools/scan_c5.py 1 256 \
  > "$OUT/prof1.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof8" -o run -- python tools/scan_c5.py 8 256 \
  > "$OUT/prof8.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scan_bf_kernel" \
  -d "$OUT/pmc_fetch" -o run --output-format csv -- python tools/scan_c5.py 1 256 \
  > "$OUT/pmc_fetch.log" 2>&1 || exit $?
