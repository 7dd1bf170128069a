set -o pipefail
OUT=gpurun_out/${1:-r5p}; mkdir -p $OUT
export TMPDIR=/tmp
LEAN="--no-c5 --no-train-leg --no-eos-leg --no-index-build --no-cpu-baseline"
rm -f $OUT/summary.txt
for i in 1 2; do for P in gen none enc; do
  MPR_STREAM_PRIO=$P timeout -k 10 300 python bench.py --steps 20 --warmup 4 $LEAN > $OUT/b_${P}_$i.json 2>/dev/null || exit $?
  python -c "import json,sys;d=json.loads(open('$OUT/b_${P}_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('PRIO=$P', d['value'], d['sync_ms_per_step'], d['lookahead_ms_per_step'], d['main_loop_ms_per_step'], r['frac'], r['in_serving_loop']['frac'])" >> $OUT/summary.txt
done; done
cat $OUT/summary.txt
