#!/bin/bash
# One GPU call: the grouped-decode tests, then C5 end to end and the serving loop timed with
# MPR_SKINNY_MAXC=4 against the default (alternating, twice).  Each GPU step has its own time
# limit; a failure ends the script.
# usage: bash tools/round_k.sh <tag>
TAG=${1:-r03_k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "$1 rc=$2" >> "$OUT/steps.log"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "t5 or decode or grouped" > "$OUT/pytest.log" 2>&1
step pytest $?
for r in 1 2; do
  for v in MPR_DEFAULTS=1 MPR_SKINNY_MAXC=4; do
    echo "[$v]" >> "$OUT/c5_ab.txt"
    env $v timeout -k 10 200 python tools/c5_trace.py >> "$OUT/c5_ab.txt" 2>&1
    step "c5 $v" $?
    echo "[$v]" >> "$OUT/serving_ab.txt"
    env $v timeout -k 10 200 python tools/serving_trace.py 40 >> "$OUT/serving_ab.txt" 2>&1
    step "serving $v" $?
  done
done
