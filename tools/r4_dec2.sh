#!/bin/bash
# gemm_dec round: kernel tests, launch sweep over MPR_DEC_BLOCKS, decode A/B at 16/128/256 rows,
# kernel stats of a t5-base 128-row decode.  Each GPU step time-limited; stops on a fault.
OUT=gpurun_out/${1:-r4dec3}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 300 python -u -m pytest tests/test_gpu_decode_gemm.py -q -x --timeout 120 --timeout-method thread
step sweep 400 python tools/rows_bench.py 128 192 256 384
for shape in "small 128" "base 128" "base 256"; do
  step "ab_$(echo $shape | tr ' ' _)" 120 python tools/decode_rows.py $shape
done
step ab_skinny_base_128 120 env MPR_DECODE_GEMM=skinny python tools/decode_rows.py base 128
step prof 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_base_128" -o run --output-format csv -- python tools/decode_rows.py base 128 71 10
find "$OUT" -name "*kernel_trace.csv" -delete
echo done >> "$OUT/steps.log"
