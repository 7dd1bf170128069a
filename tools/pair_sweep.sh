#!/bin/bash
# GPU box: paired-decode parity tests, then the serving bench with decode pairing on/off and
# 1-3 generate calls in flight.  Each GPU step has its own time limit; the first failure ends it.
# usage: bash tools/pair_sweep.sh <tag> [steps]
TAG=${1:-pair}
STEPS=${2:-16}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py::test_t5_generate_pair_matches_single tests/test_gpu_kernels.py::test_encode_towers_slots_run_concurrently tests/test_gpu_golden.py \
  > "$OUT/pytest.log" 2>&1 || exit $?
# "pair in-flight lookahead" per run; CFGS (';'-separated) overrides
IFS=';' read -r -a RUNS <<< "${CFGS:-1 2 1;0 2 1;1 1 1;0 1 1;0 2 0}"
for cfg in "${RUNS[@]}"; do
  set -- $cfg
  MPR_PAIR_DECODE=$1 MPR_LOOKAHEAD=$3 timeout -k 10 200 python bench.py --steps "$STEPS" \
    --warmup 3 --no-cpu-baseline --no-c5 --inflight "$2" \
    > "$OUT/bench_p$1_if$2_la$3.json" 2> "$OUT/bench_p$1_if$2_la$3.err" || exit $?
done
