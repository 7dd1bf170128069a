set -o pipefail
OUT=gpurun_out/${1:-r5j}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_dropin.py tests/test_gpu_train.py tests/test_gpu_eos_stop.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/train_trace.py 6 > $OUT/plain.log 2>&1; echo "train rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tt -o run -- python tools/train_trace.py 6 > $OUT/trace.log 2>&1; echo "trace rc=$?"
python tools/serving_trace.py --report $OUT/tt > $OUT/report.txt 2>&1
python tools/gap_list.py $OUT/tt > $OUT/gaps.txt 2>&1; find $OUT/tt -name "*kernel_trace.csv" -delete
