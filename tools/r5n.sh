set -o pipefail
OUT=gpurun_out/${1:-r5n}; mkdir -p $OUT
export TMPDIR=/tmp
LEAN="--no-c5 --no-train-leg --no-eos-leg --no-index-build --no-cpu-baseline"
for i in 1 2 3; do for P in 0 1; do
  MPR_X3P_POLICY=$P timeout -k 10 300 python bench.py --steps 20 --warmup 4 $LEAN > $OUT/b_${P}_$i.json 2>/dev/null || exit $?
  python -c "import json,sys;d=json.loads(open('$OUT/b_${P}_$i.json').read().strip().splitlines()[-1]);print('P=$P', d['value'], d['roofline']['frac'], d['roofline']['in_serving_loop']['frac'], d['sync_ms_per_step'])" >> $OUT/summary.txt
done; done
cat $OUT/summary.txt
