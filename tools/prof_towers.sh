#!/bin/bash
# Kernel traces of the tower pass alone (towers_bench.py B), default vs MPR_GEMM=f32 (dev aid).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-tw}
B=${2:-32}
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/x3 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/towers_bench.py $B > $OUT/x3.log 2>&1 || exit $?
MPR_GEMM=f32 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/f32 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/towers_bench.py $B > $OUT/f32.log 2>&1
