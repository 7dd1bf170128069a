# Serving-pipeline sweep: decodes in flight (bench c2, no cpu baseline / probe).
# Measured (4 HW queues, the box default): 1 -> 1702, 2 -> 2105/2116, 3 -> 1216-1455 QA pairs/s;
# GPU_MAX_HW_QUEUES 8 / 16 with 2 in flight: 1651 / 1658.
set -e
mkdir -p gpurun_out/cus
for n in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 12 --warmup 4 --inflight $n --no-cpu-baseline --no-probe > gpurun_out/cus/bench_if$n.json 2> gpurun_out/cus/bench_if$n.err
done
