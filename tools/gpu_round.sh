#!/bin/bash
# GPU-box round: tests -> smoke -> bench -> rocprofv3 kernel stats -> two PMC passes (GEMM HBM
# traffic).  Each GPU step has its own time limit; anything but a clean exit (or plain test
# failures, rc 1) ends the script.
# usage: bash tools/gpu_round.sh <tag> [steps]   (bench, trace and PMC passes all at <steps>, so
# the trace's replay window and the PMC traffic describe the same launches as bench.json)
TAG=${1:-r}
STEPS=${2:-10}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# the profiled passes skip the side legs (C5, training, eos, index build): their kernels are not
# in the replay window or the GEMM counters
LEAN="--no-c5 --no-train-leg --no-eos-leg --no-index-build"

ok_or_stop() {  # $1 = rc, $2 = step name, $3 = allow-rc-1
  local rc=$1
  echo "$2 rc=$rc" >> "$OUT/steps.log"
  if [ "$rc" -eq 0 ]; then return 0; fi
  if [ "$3" = "1" ] && [ "$rc" -eq 1 ]; then return 0; fi
  echo "stopping after $2 (rc=$rc)" >> "$OUT/steps.log"
  exit "$rc"
}

if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -rf --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
  ok_or_stop $? pytest 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  ok_or_stop $? smoke 0
fi
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 4 > "$OUT/bench.json" 2> "$OUT/bench.err"
ok_or_stop $? bench 0
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python bench.py --steps "$STEPS" --warmup 4 --no-cpu-baseline $LEAN \
    > "$OUT/prof.log" 2>&1
  ok_or_stop $? rocprof 0
  python tools/prof_summary.py --replay "$OUT/prof/run_kernel_trace.csv" "$OUT/replay_window.json" >> "$OUT/prof.log" 2>&1
  rm -f "$OUT/prof/run_kernel_trace.csv"  # summarised; the full trace of 80 steps is > 64 MiB
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "gemm_x3_kernel|gemm_x3p_kernel|gemm_f32_kernel|probe_marker_kernel" \
      -d "$OUT/pmc_$c" -o run --output-format csv \
      -- python bench.py --steps "$STEPS" --warmup 4 --no-cpu-baseline $LEAN > "$OUT/pmc_$c.log" 2>&1
    ok_or_stop $? pmc_$c 0
  done
  python tools/pmc_traffic.py "$OUT/pmc_FETCH_SIZE/run_counter_collection.csv" \
    "$OUT/pmc_WRITE_SIZE/run_counter_collection.csv" "$OUT/pmc_gemm.json" >> "$OUT/prof.log" 2>&1
  rm -f "$OUT"/pmc_*/run_counter_collection.csv
fi
if [ -z "$SKIP_PROF" ]; then
  # the serving loop's and one predict()'s stream timelines from hipEvents, unprofiled (a
  # rocprofv3 kernel trace blocks the host in every graph launch: profiles/r05_profiler_block.txt)
  timeout -k 10 300 python tools/loop_events.py 40 > "$OUT/loop_events.txt" 2>&1
  ok_or_stop $? loop_events 0
  timeout -k 10 300 python tools/predict_events.py 12 > "$OUT/predict_events.txt" 2>&1
  ok_or_stop $? predict_events 0
fi
echo done >> "$OUT/steps.log"
