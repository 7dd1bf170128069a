# Rehearse the N-rank bench on one GPU: gloo backend, ranks share the device (collectives staged
# through host memory).  Checks the N>1 code path (barriers, max-over-ranks, C5 sharded scan ids
# checksum, and with --index-sharding shard the row-sharded serving index through every bench
# leg) before the driver's 8-GPU RCCL run.
set -e
mkdir -p gpurun_out/rehearse
run() {  # name, nproc, extra args...
  local name=$1 n=$2; shift 2
  MPR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n + ${#name})) \
    bench.py --gpus $n --steps 5 --warmup 2 --no-cpu-baseline --no-probe --no-eos-leg "$@" \
    > gpurun_out/rehearse/$name.json 2> gpurun_out/rehearse/$name.err
  echo "$name done" >> gpurun_out/rehearse/steps.log
}
run bench_n2 2
[ -n "$WITH_N4" ] && run bench_n4 4
run shard_n2 2 --index-sharding shard --no-c5 --no-index-build
