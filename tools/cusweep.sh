# Serving-loop stream priorities with two decodes in flight (bench c2).
set -e
mkdir -p gpurun_out/cus
for p in enc gen both none; do
  MPR_STREAM_PRIO=$p timeout -k 10 200 python bench.py --steps 16 --warmup 4 --no-cpu-baseline --no-probe --no-c5 > gpurun_out/cus/bench_p$p.json 2> gpurun_out/cus/bench_p$p.err
done
for n in 1 3; do
  timeout -k 10 200 python bench.py --steps 16 --warmup 4 --inflight $n --no-cpu-baseline --no-probe --no-c5 > gpurun_out/cus/bench_if$n.json 2> gpurun_out/cus/bench_if$n.err
done
