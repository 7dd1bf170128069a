set -o pipefail
mkdir -p gpurun_out/r5t5
for T in gen:0; do for V in role; do for E in 1 0; do export MPR_EAGER_STREAMS=$E;
  export MPR_SPEC_STREAM=$V MPR_AHEAD_T5_STREAM=$T
  timeout -k 10 300 python tools/train_events.py > gpurun_out/r5t5/plain.txt 2>&1 || exit $?
  timeout -k 10 300 python tools/train_events.py --eos-first > gpurun_out/r5t5/eos.txt 2>&1 || exit $?
  echo "eager streams $E, predict on $T, spec $V | plain: $(grep 'per step' gpurun_out/r5t5/plain.txt) | eos-first: $(grep 'per step' gpurun_out/r5t5/eos.txt)" | tee -a gpurun_out/r5t5/summary.txt
done; done; done
