#!/bin/bash
# Which graphs the 20-step serving loop captures inside the timed region (development aid).
OUT=gpurun_out/${1:-graphlog}
mkdir -p "$OUT"
FAST="--steps 20 --no-c5 --no-train-leg --no-eos-leg --no-index-build --no-cpu-baseline --no-probe"
MPR_GRAPH_LOG=1 timeout -k 10 300 python bench.py $FAST --warmup 5 > "$OUT/w5.log" 2>&1
