set -o pipefail
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py "tests/test_gpu_configs.py::test_c2_full_size_end_to_end_vs_oracle" tests/test_gpu_kernels.py -k "sharded or rccl or c2_full or merge" -s > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
