# Serving-pipeline stream policy sweep (bench c2, no cpu baseline / probe).
set -e
mkdir -p gpurun_out/cus
for p in enc dec none; do
  MPR_STREAM_PRIO=$p timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe > gpurun_out/cus/bench_$p.json 2> gpurun_out/cus/bench_$p.err
done
