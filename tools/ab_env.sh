#!/bin/bash
# A/B of environment settings on the serving headline (bench.py, 40 steps, no side legs).
# usage: bash tools/ab_env.sh <tag> "ENV=a ENV2=b" "ENV=c" ...   (each setting run twice, alternating)
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    env $setting timeout -k 10 300 python bench.py --steps 40 --warmup 4 --no-cpu-baseline \
      --no-index-build --no-eos-leg --no-train-leg --no-c5 --no-probe > "$OUT/ab_${i}_${rep}.json" 2>> "$OUT/ab.err" || exit $?
    python -c "import json,sys; d=json.load(open('$OUT/ab_${i}_${rep}.json')); print('$setting', d['value'], d['sync_ms_per_step'], d['main_loop_ms_per_step'], d['decode']['us_per_step'])" >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
