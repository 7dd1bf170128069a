set -o pipefail
OUT=gpurun_out/${1:-r5t}; mkdir -p $OUT
export TMPDIR=/tmp
rm -f $OUT/summary.txt
LEAN="--no-c5 --no-index-build --no-cpu-baseline"
for i in 1 2; do for E in 1 0; do
  MPR_EAGER_STREAMS=$E timeout -k 10 400 python bench.py --steps 20 --warmup 4 $LEAN > $OUT/b_${E}_$i.json 2>/dev/null || exit $?
  python -c "import json,sys;d=json.loads(open('$OUT/b_${E}_$i.json').read().strip().splitlines()[-1]);t=d['train_step'];r=t['roofline'];print('EAGER=$E', d['value'], d['sync_ms_per_step'], d['lookahead_ms_per_step'], d['main_loop_ms_per_step'], t['ms_per_step'], r['gemm_ms_per_step'], d['eos_stop_leg']['eos_stop']['qa_pairs_per_s'], d['roofline']['frac'])" >> $OUT/summary.txt
done; done
cat $OUT/summary.txt
