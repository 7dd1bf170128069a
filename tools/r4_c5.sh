#!/bin/bash
# C5 serving-loop trace + sync predict() timeline (development aid).
OUT=gpurun_out/${1:-r4c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c5" -o run -- python tools/c5_trace.py > "$OUT/c5.log" 2>&1 || exit $?
python tools/serving_trace.py --report "$OUT/c5" > "$OUT/c5_report.txt" 2>&1
find "$OUT/c5" -name "*kernel_trace.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pt" -o run -- python tools/predict_timeline.py > "$OUT/pt.log" 2>&1 || exit $?
python tools/predict_timeline_report.py "$OUT/pt" > "$OUT/pt_report.txt" 2>&1
find "$OUT/pt" -name "*kernel_trace.csv" -delete
echo done
