#!/bin/bash
# One GPU call: C5 end to end (tools/c5_trace.py) and the serving loop (tools/serving_trace.py,
# 40 steps) timed per variant (env settings in VARIANTS, alternating, twice); TESTS=1 runs the
# grouped-decode GPU tests first.  Each GPU step has its own time limit; a failure ends the script.
# usage: VARIANTS="MPR_DEFAULTS=1 MPR_X=1" bash tools/decode_ab.sh <tag>
TAG=${1:-decode_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-"MPR_DEFAULTS=1"}
step() { echo "$1 rc=$2" >> "$OUT/steps.log"; [ "$2" -eq 0 ] || exit "$2"; }
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "t5 or decode or grouped" > "$OUT/pytest.log" 2>&1
  step pytest $?
fi
for r in 1 2; do
  for v in $VARIANTS; do
    echo "[$v]" >> "$OUT/c5_ab.txt"
    env $v timeout -k 10 200 python tools/c5_trace.py >> "$OUT/c5_ab.txt" 2>&1
    step "c5 $v" $?
    echo "[$v]" >> "$OUT/serving_ab.txt"
    env $v timeout -k 10 200 python tools/serving_trace.py 40 >> "$OUT/serving_ab.txt" 2>&1
    step "serving $v" $?
  done
done
