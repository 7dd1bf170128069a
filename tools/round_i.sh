#!/bin/bash
# One GPU call: the coarse-scan A/B (tools/scan_ab.sh: tests, C5 timings, kernel stats), the C5
# end-to-end trace (tools/c5_trace.py under rocprofv3 + cProfile of one predict), then the
# driver's bench command.  Each GPU step has its own time limit; a failure ends the script.
# usage: bash tools/round_i.sh <tag>
TAG=${1:-r03_i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/scan_ab.sh "$TAG" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c5t" -o run \
  -- python tools/c5_trace.py --cprofile > "$OUT/c5_trace.txt" 2>&1 || exit $?
python tools/serving_trace.py --report "$OUT/c5t" >> "$OUT/c5_trace.txt" 2>&1
rm -f "$OUT"/c5t/*kernel_trace.csv "$OUT"/c5t/*/*kernel_trace.csv
echo "c5 trace done" >> "$OUT/steps.log"
timeout -k 10 600 python bench.py --steps 20 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo "bench done" >> "$OUT/steps.log"
