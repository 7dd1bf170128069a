#!/bin/bash
# Training-step trace (development aid): timed steps, a rocprofv3 kernel trace, a cProfile.
OUT=gpurun_out/${1:-r4train}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/train_trace.py 6 > "$OUT/plain.log" 2>&1 || exit $?

timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tt" -o run -- python tools/train_trace.py 6 > "$OUT/trace.log" 2>&1 || exit $?
python tools/serving_trace.py --report "$OUT/tt" > "$OUT/report.txt" 2>&1
find "$OUT/tt" -name "*kernel_trace.csv" -delete
timeout -k 10 300 python tools/train_trace.py 3 --cprofile > "$OUT/cprofile.txt" 2>&1 || exit $?
echo done
