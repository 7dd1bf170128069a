# Contention sweep: LDS residency of encoder GEMM blocks vs decode GEMV blocks (bench c2).
set -e
mkdir -p gpurun_out/cus
run() { timeout -k 10 200 env "$@" python bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-probe > gpurun_out/cus/bench_$TAG.json 2> gpurun_out/cus/bench_$TAG.err; }
TAG=base run X=0
TAG=sl run MPR_SKINNY_SMALL_LDS=1
TAG=cb3 run MPR_GEMM_CU_BLOCKS=3
TAG=cb3sl run MPR_GEMM_CU_BLOCKS=3 MPR_SKINNY_SMALL_LDS=1
TAG=cb2sl run MPR_GEMM_CU_BLOCKS=2 MPR_SKINNY_SMALL_LDS=1
