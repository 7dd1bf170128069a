#!/bin/bash
# Decode loop A/B (development aid): tools/decode_rows.py over row counts, the round-3 skinny
# GEMVs vs gemm_rows (folded / unfolded chain), then rocprofv3 kernel stats of some shapes.
# usage: bash tools/r4_decode_ab.sh <tag> [ab|prof|both]
OUT=gpurun_out/${1:-r4dec}
WHAT=${2:-both}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # env... -- args
  timeout -k 10 120 env "$@" >> "$OUT/ab.txt" 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc ($*)" >> "$OUT/ab.txt"; exit $rc; fi
}
if [ "$WHAT" != prof ]; then
  for shape in "small 16" "small 128" "base 128" "base 256"; do
    [ "$shape" != "base 256" ] && run MPR_DECODE_GEMM=skinny python tools/decode_rows.py $shape
    run MPR_ROWS_FOLD=1 python tools/decode_rows.py $shape
    run MPR_ROWS_FOLD=0 python tools/decode_rows.py $shape
  done
fi
if [ "$WHAT" != ab ]; then
  for spec in "rows small 16" "rows small 128" "rows base 128" "skinny base 128" "skinny small 16"; do
    set -- $spec
    tag="$1_$2_$3"
    timeout -k 10 180 env MPR_DECODE_GEMM=$1 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run \
      --output-format csv -- python tools/decode_rows.py $2 $3 71 10 > "$OUT/prof_$tag.log" 2>&1 || exit $?
    find "$OUT/prof_$tag" -name "*kernel_trace.csv" -delete
  done
fi
echo done >> "$OUT/ab.txt"
