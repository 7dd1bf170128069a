#!/bin/bash
# One GPU call: the GPU test suite, the C5 end-to-end trace with the grouped-decode changes
# (tiled argmax head, wave-per-pair decode attention, 4-tile skinny blocks) against them off, the
# serving loop timed with each (alternating), then the driver's bench command.  Each GPU step
# has its own time limit; a failure ends the script.
# usage: bash tools/round_j.sh <tag>
TAG=${1:-r03_j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "$1 rc=$2" >> "$OUT/steps.log"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1
step pytest $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c5t" -o run \
  -- python tools/c5_trace.py > "$OUT/c5_trace.txt" 2>&1
step c5_trace $?
python tools/serving_trace.py --report "$OUT/c5t" >> "$OUT/c5_trace.txt" 2>&1
rm -f "$OUT"/c5t/*kernel_trace.csv "$OUT"/c5t/*/*kernel_trace.csv
for v in "MPR_TILED_HEAD=0 MPR_ATT_WAVE=0" "MPR_TILED_HEAD=1 MPR_ATT_WAVE=0" "MPR_TILED_HEAD=0 MPR_ATT_WAVE=1" "MPR_SKINNY_NT=4 MPR_TILED_HEAD=0 MPR_ATT_WAVE=0" "MPR_SKINNY_NT=4" "MPR_DEFAULTS=1"; do
  echo "[$v]" >> "$OUT/c5_ab.txt"
  env $v timeout -k 10 200 python tools/c5_trace.py >> "$OUT/c5_ab.txt" 2>&1
  step "c5 $v" $?
done
for r in 1 2; do
  for v in MPR_ATT_WAVE=0 MPR_DEFAULTS=1 MPR_SKINNY_NT=4; do
    echo "[$v]" >> "$OUT/serving_ab.txt"
    env $v timeout -k 10 200 python tools/serving_trace.py 40 >> "$OUT/serving_ab.txt" 2>&1
    step "serving $v" $?
  done
done
timeout -k 10 600 python bench.py --steps 20 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench $?
