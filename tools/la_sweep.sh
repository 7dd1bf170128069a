set -e
mkdir -p gpurun_out/la3
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe --no-c5 --no-index-build"
timeout -k 10 200 $B > gpurun_out/la3/base.txt 2>&1
MPR_AHEAD_T5_STREAM=gen:1 timeout -k 10 200 $B > gpurun_out/la3/gen1.txt 2>&1
MPR_AHEAD_T5_STREAM=gen:2 timeout -k 10 200 $B > gpurun_out/la3/gen2.txt 2>&1
MPR_AHEAD_T5_STREAM=private timeout -k 10 200 $B > gpurun_out/la3/private.txt 2>&1
MPR_AHEAD_T5_STREAM=current timeout -k 10 200 $B > gpurun_out/la3/current.txt 2>&1
MPR_STREAM_PRIO=enc timeout -k 10 200 $B > gpurun_out/la3/prioenc.txt 2>&1
