set -o pipefail
OUT=gpurun_out/${1:-r5f}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_golden.py -k "sharded or rccl or merge or coarse or scan or c5 or search or golden" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/proj_trace.py 8 40 > $OUT/proj.txt 2>&1; echo "proj rc=$?"
timeout -k 10 200 python -u tools/proj_trace.py 1 20 > $OUT/proj1.txt 2>&1; echo "proj1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u tools/proj_trace.py 8 40 > $OUT/prof.log 2>&1; echo "prof rc=$?"
