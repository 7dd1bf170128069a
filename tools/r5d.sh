set -o pipefail
OUT=gpurun_out/${1:-r5d}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/proj_trace.py 8 40 > $OUT/proj.txt 2>&1; echo "proj rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u tools/proj_trace.py 8 40 > $OUT/prof.log 2>&1; echo "prof rc=$?"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py > $OUT/pytest.log 2>&1; echo "pytest rc=$?"
