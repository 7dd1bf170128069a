# Rehearse the N-rank bench on one GPU: gloo backend, ranks share the device (collectives staged
# through host memory).  Checks the N>1 code path (sharded retrieval, barriers, max-over-ranks,
# C5 sharded scan ids checksum) before the driver's 8-GPU RCCL run.
set -e
mkdir -p gpurun_out/rehearse
for n in 2 4; do
  MPR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) \
    bench.py --gpus $n --steps 5 --warmup 2 --no-cpu-baseline --no-probe $EXTRA \
    > gpurun_out/rehearse/bench_n$n.json 2> gpurun_out/rehearse/bench_n$n.err
done
