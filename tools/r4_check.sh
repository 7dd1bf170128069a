#!/bin/bash
# Round-4 GPU check (development aid): GPU tests (optionally a -k filter), the bench, and the
# decode timing of a t5-base 256-row group.  Each GPU step time-limited; stops on a fault.
OUT=gpurun_out/${1:-r4chk}
FILTER=${2:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ -n "$FILTER" ]; then
  step pytest 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread -k "$FILTER"
else
  step pytest 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
fi
step bench 600 python bench.py --steps 20 --warmup 4
mv "$OUT/bench.log" "$OUT/bench.json"
step dec256 120 python tools/decode_rows.py base 256 40
step dec128 120 python tools/decode_rows.py base 128 40
echo done >> "$OUT/steps.log"
