set -o pipefail
OUT=gpurun_out/${1:-r5m}; mkdir -p $OUT
export TMPDIR=/tmp
for V in 1 3; do
  MPR_BF2_QG2=$V timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_kernels.py -k "coarse or c5" > $OUT/pytest_$V.log 2>&1; rc=$?; echo "pytest $V rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
for W in 1 8; do for V in 0 1 2 3; do
  MPR_BF2_QG2=$V timeout -k 10 120 python -u tools/scan_c5.py $W >> $OUT/c5.txt 2>&1 || exit $?
  echo "W=$W QG2=$V" >> $OUT/c5.txt
done; done
