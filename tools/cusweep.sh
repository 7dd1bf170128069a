# Serving-loop stream priorities with two decodes in flight (bench c2).
set -e
mkdir -p gpurun_out/cus
for p in enc gen both none; do
  MPR_STREAM_PRIO=$p timeout -k 10 200 python bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-probe --no-c5 > gpurun_out/cus/bench_p$p.json 2> gpurun_out/cus/bench_p$p.err
done
