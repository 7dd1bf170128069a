#!/bin/bash
# GPU-box round: tests -> smoke -> bench -> rocprofv3 kernel stats.  Each GPU step has its own
# time limit; anything but a clean exit (or plain test failures, rc 1) ends the script.
# usage: bash tools/gpu_round.sh <tag> [steps]
TAG=${1:-r}
STEPS=${2:-10}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

ok_or_stop() {  # $1 = rc, $2 = step name, $3 = allow-rc-1
  local rc=$1
  echo "$2 rc=$rc" >> "$OUT/steps.log"
  if [ "$rc" -eq 0 ]; then return 0; fi
  if [ "$3" = "1" ] && [ "$rc" -eq 1 ]; then return 0; fi
  echo "stopping after $2 (rc=$rc)" >> "$OUT/steps.log"
  exit "$rc"
}

if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu -rf > "$OUT/pytest.log" 2>&1
  ok_or_stop $? pytest 1
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok_or_stop $? smoke 0
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
ok_or_stop $? bench 0
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe \
    > "$OUT/prof.log" 2>&1
  ok_or_stop $? rocprof 0
fi
echo done >> "$OUT/steps.log"
