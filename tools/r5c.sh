set -o pipefail
OUT=gpurun_out/${1:-r5c}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_decode_fuse.py tests/test_gpu_kernels.py -k "sharded or rccl or merge or fused" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/proj_diag.py > $OUT/diag.txt 2>&1; echo "diag rc=$?"
timeout -k 10 300 python -u tools/decode_fuse_ab.py 3 > $OUT/ab.txt 2>&1; echo "ab rc=$?"
