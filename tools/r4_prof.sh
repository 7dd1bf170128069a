#!/bin/bash
# Host profiles (development aid): cProfile of the C5 serving loop and of sync predict().
OUT=gpurun_out/${1:-prof}
mkdir -p "$OUT"
timeout -k 10 300 python tools/c5_trace.py --cprofile > "$OUT/c5_cprofile.txt" 2>&1 || exit $?
timeout -k 10 300 python tools/predict_timeline.py --cprofile > "$OUT/pt_cprofile.txt" 2>&1 || exit $?
echo done
