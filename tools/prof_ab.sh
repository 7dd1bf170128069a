#!/bin/bash
# A/B kernel traces of the bench: default vs MPR_GEMM=f32 (development aid).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/x3 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-index-build > $OUT/x3.log 2>&1 || exit $?
MPR_GEMM=f32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/f32 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c5 --no-index-build > $OUT/f32.log 2>&1
