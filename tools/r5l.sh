set -o pipefail
OUT=gpurun_out/${1:-r5l}; mkdir -p $OUT
export TMPDIR=/tmp
MPR_BF2_GLDS=1 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_kernels.py tests/test_gpu_sharded.py -k "coarse or scan or c5 or sharded" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for W in 1 8; do for V in 0 1 0 1; do
  MPR_BF2_GLDS=$V timeout -k 10 120 python -u tools/scan_c5.py $W >> $OUT/c5.txt 2>&1 || exit $?
  echo "W=$W GLDS=$V" >> $OUT/c5.txt
done; done
MPR_BF2_GLDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u tools/scan_c5.py 8 > $OUT/prof.log 2>&1; echo "prof rc=$?"
