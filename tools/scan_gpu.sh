#!/bin/bash
# Scan-only GPU check: scan/top-k parity tests, tools/scan_bench.py (events per search: scan +
# merge), and a rocprofv3 kernel trace of the same bench (kernel-only durations per shape:
# python tools/scan_prof.py <trace.csv>).   usage: bash tools/scan_gpu.sh <tag>
O=gpurun_out/${1:-scan}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "scan or topk" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python tools/scan_bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/scan_bench.py > $O/prof.log 2>&1 || exit $?
echo done
