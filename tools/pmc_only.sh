#!/bin/bash
# The two PMC passes of tools/gpu_round.sh alone (FETCH_SIZE, WRITE_SIZE over the GEMM replay of a
# <steps>-step bench), summarised on the box with the per (kernel, grid) breakdown.
TAG=${1:-pmc}
STEPS=${2:-80}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "gemm_x3_kernel|gemm_f32_kernel|probe_marker_kernel" \
    -d "$OUT/pmc_$c" -o run --output-format csv \
    -- python bench.py --steps "$STEPS" --warmup 4 --no-cpu-baseline --no-c5 --no-index-build \
    > "$OUT/pmc_$c.log" 2>&1 || exit $?
  echo "pmc_$c done" >> "$OUT/steps.log"
done
python tools/pmc_traffic.py "$OUT/pmc_FETCH_SIZE/run_counter_collection.csv" \
  "$OUT/pmc_WRITE_SIZE/run_counter_collection.csv" "$OUT/pmc_gemm.json" > "$OUT/pmc.log" 2>&1
rm -f "$OUT"/pmc_*/run_counter_collection.csv
