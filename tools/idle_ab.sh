#!/bin/bash
# Serving-loop idle time under rocprofv3 (tools/serving_trace.py), default vs the image uploader
# thread (MPR_UPLOAD_THREAD=2: pageable -> pinned on a worker, the DMA on the consumer's stream).
# usage: bash tools/idle_ab.sh <tag>
OUT=gpurun_out/${1:-idle}
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in DEFAULT=1 MPR_UPLOAD_THREAD=2; do
  env "$V" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/st_$V" \
    -- python tools/serving_trace.py 20 > "$OUT/trace_$V.txt" 2>&1 || exit $?
  python tools/serving_trace.py --report "$OUT/st_$V" >> "$OUT/trace_$V.txt" 2>&1
  rm -rf "$OUT/st_$V"
done
echo done >> "$OUT/steps.log"
