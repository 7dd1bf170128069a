set -o pipefail
OUT=gpurun_out/${1:-r5g}; mkdir -p $OUT
export TMPDIR=/tmp
for W in 1 8; do for V in 0 1 2; do
  MPR_BF2_VARIANT=$V timeout -k 10 120 python -u tools/scan_c5.py $W >> $OUT/c5.txt 2>&1 || exit $?
  echo "W=$W V=$V" >> $OUT/c5.txt
done; done
echo ok
