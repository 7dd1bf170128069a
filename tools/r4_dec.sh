#!/bin/bash
# Decode-projection A/B (development aid): skinny GEMVs vs the tiled GEMM (MPR_DEC_TILED=1).
OUT=gpurun_out/${1:-r4dec}
mkdir -p "$OUT"
for r in 128 256; do
  timeout -k 10 120 python tools/decode_rows.py base $r 40 > "$OUT/skinny$r.log" 2>&1 || exit $?
  MPR_DEC_TILED=1 timeout -k 10 120 python tools/decode_rows.py base $r 40 > "$OUT/tiled$r.log" 2>&1 || exit $?
done
timeout -k 10 120 python tools/decode_rows.py small 128 71 40 > "$OUT/skinny_s128.log" 2>&1 || exit $?
MPR_DEC_TILED=1 timeout -k 10 120 python tools/decode_rows.py small 128 71 40 > "$OUT/tiled_s128.log" 2>&1 || exit $?
timeout -k 10 200 python tools/c5_lens.py > "$OUT/lens.log" 2>&1 || exit $?
echo done
