# round-5: fused decode attention check (bit-identity test + A/B timing)
set -o pipefail
OUT=gpurun_out/${1:-r5b}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_decode_fuse.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/decode_fuse_ab.py 3 > $OUT/ab.txt 2>&1; echo "ab rc=$?"
