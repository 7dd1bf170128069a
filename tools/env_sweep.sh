#!/bin/bash
# GPU box: serving bench (bench.py, no CPU baseline / C5 / index build / probe) once per
# environment setting.  Each run has its own time limit; the first failure ends the sweep.
# usage: CFGS="MPR_STREAM_PRIO=enc;MPR_STREAM_PRIO=none INFLIGHT=1" bash tools/env_sweep.sh <tag>
# (INFLIGHT=n is passed as --inflight n; everything else is exported to the run.)
TAG=${1:-env}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
IFS=';' read -r -a RUNS <<< "${CFGS:-}"
i=0
for cfg in "${RUNS[@]}"; do
  i=$((i + 1))
  inflight=2
  envs=()
  for kv in $cfg; do
    case $kv in
      INFLIGHT=*) inflight=${kv#INFLIGHT=} ;;
      *) envs+=("$kv") ;;
    esac
  done
  echo "$i: $cfg" > "$OUT/cfg_$i.txt"
  env "${envs[@]}" timeout -k 10 300 python bench.py --inflight "$inflight" \
    --no-cpu-baseline --no-c5 --no-index-build --no-probe \
    > "$OUT/b_$i.json" 2> "$OUT/b_$i.err" || exit $?
done
