#!/bin/bash
# Coarse-scan A/B on the GPU box: the scan / coarse / merge tests (default kernel), then the C5
# search (1M x 512, 256 queries, k = 5) and its 1/8 shard timed per kernel variant (env settings
# in VARIANTS; ids checksums must agree), a rocprofv3 kernel-stats pass of the default at W = 1
# and 8, and a FETCH_SIZE pass of the coarse kernel.  Every GPU step has its own time limit;
# anything but a clean exit (or plain test failures, rc 1) ends the script.
# usage: bash tools/scan_ab.sh <tag>
TAG=${1:-scan}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-"DEFAULT=1"}
timeout -k 10 420 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -v -m gpu \
  -k "scan or coarse or c5 or merge" -rf --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
for W in 1 8; do
  for V in $VARIANTS; do
    env "$V" timeout -k 10 120 python tools/scan_c5.py $W >> "$OUT/c5.txt" 2>&1 || exit $?
  done
done
echo "c5 done" >> "$OUT/steps.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python tools/scan_c5.py 1 > "$OUT/prof.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof8" -o run --output-format csv \
  -- python tools/scan_c5.py 8 > "$OUT/prof8.log" 2>&1 || exit $?
rm -f "$OUT"/prof*/run_kernel_trace.csv
# HBM bytes of the coarse kernel (FETCH_SIZE x 2: the gfx950 half-count of 16-B streaming reads)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scan_bf" -d "$OUT/pmc" \
  -o run --output-format csv -- python tools/scan_c5.py 1 > "$OUT/pmc.log" 2>&1 || exit $?
python - "$OUT" >> "$OUT/c5.txt" 2>&1 <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)[0])))
v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"].startswith("FETCH_SIZE")]
print(f"scan_bf FETCH_SIZE: {len(v)} launches, {2 * sum(v) / len(v) * 1024 / 1e6:.1f} MB per launch (FETCH_SIZE KB x 2, gfx950 correction)")
PY
rm -f "$OUT"/pmc/*/*counter_collection.csv "$OUT"/pmc/*counter_collection.csv
echo done >> "$OUT/steps.log"
