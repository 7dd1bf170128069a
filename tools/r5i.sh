set -o pipefail
OUT=gpurun_out/${1:-r5i}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_gemm_train.py -k "rows_x3p or packed" > $OUT/pytest.log 2>&1; echo "pytest rc=$?"
for V in 100000 128; do for W in 0 1; do
  MPR_DECODE_X3_ROWS=$V MPR_DECODE_X3_WO=$W timeout -k 10 200 python -u tools/c5_trace.py > $OUT/c5_${V}_${W}.txt 2>&1; echo "c5 $V $W rc=$?"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5t -- python -u tools/c5_trace.py > $OUT/c5t.log 2>&1; echo "c5t rc=$?"
python tools/serving_trace.py --report $OUT/c5t > $OUT/c5_report.txt 2>&1
rm -rf $OUT/c5t
