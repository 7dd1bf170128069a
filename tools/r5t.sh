set -o pipefail
OUT=gpurun_out/${1:-r5t}; mkdir -p $OUT
export TMPDIR=/tmp
LEAN="--no-c5 --no-eos-leg --no-index-build --no-cpu-baseline"
rm -f $OUT/summary.txt
for i in 1 2; do for P in 1 2; do
  MPR_X3_SB=$P timeout -k 10 400 python bench.py --steps 20 --warmup 4 $LEAN > $OUT/b_${P}_$i.json 2>/dev/null || exit $?
  python -c "import json,sys;d=json.loads(open('$OUT/b_${P}_$i.json').read().strip().splitlines()[-1]);t=d['train_step'];r=t['roofline'];print('X3_SB=$P', d['value'], t['ms_per_step'], r['gemm_ms_per_step'], r['frac'], r['gemm_share_of_wall'])" >> $OUT/summary.txt
done; done
cat $OUT/summary.txt
