set -o pipefail
OUT=gpurun_out/r5q; mkdir -p $OUT
export TMPDIR=/tmp
rm -f $OUT/summary.txt
LEAN="--no-c5 --no-index-build --no-train-leg --no-eos-leg --cpu-seconds 4"
for i in 1 2; do for E in 1 0; do
  MPR_EAGER_STREAMS=$E timeout -k 10 400 python bench.py --steps 20 --warmup 4 $LEAN > $OUT/b_${E}_$i.json 2>/dev/null || exit $?
  python -c "import json,sys;d=json.loads(open('$OUT/b_${E}_$i.json').read().strip().splitlines()[-1]);p=d['cpu_baseline']['parity'];print('EAGER=$E', d['value'], p['answers_equal'], p['serving_loop_answers_equal'], p['serving_loop_equal_predict'], p.get('mismatches'))" >> $OUT/summary.txt
done; done
cat $OUT/summary.txt
