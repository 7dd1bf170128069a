# round-5 GPU check: the whole -m gpu suite, then the default bench (driver's step counts)
set -o pipefail
OUT=gpurun_out/${1:-r5a}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests -rf > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
