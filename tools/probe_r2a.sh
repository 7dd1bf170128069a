#!/bin/bash
# r02 first probe: standalone decode split + kernel stats (t5-small 16 rows, t5-base 16 rows)
export TMPDIR=/tmp
OUT=gpurun_out/r02a
mkdir -p $OUT
timeout -k 10 200 python tools/decode_split.py 16 71 small > $OUT/split_small.txt 2>&1 || exit $?
timeout -k 10 200 python tools/decode_split.py 16 71 base > $OUT/split_base.txt 2>&1 || exit $?
timeout -k 10 200 python tools/decode_split.py 1 71 small > $OUT/split_small_b1.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/decode_split.py 16 71 small > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
