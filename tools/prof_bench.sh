#!/bin/bash
# rocprofv3 kernel trace of a short bench run (dev aid): $1 = out tag, rest = env assignments
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pb}
mkdir -p $OUT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-c5 --no-index-build > $OUT/bench.log 2>&1
