set -o pipefail
OUT=gpurun_out/${1:-r5h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5t -- python -u tools/c5_trace.py > $OUT/c5t.log 2>&1; echo "c5t rc=$?"
python tools/serving_trace.py --report $OUT/c5t > $OUT/c5_report.txt 2>&1
rm -rf $OUT/c5t
