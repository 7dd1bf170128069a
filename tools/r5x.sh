set -o pipefail
for E in MPR_GEMM=f32 MPR_X3P_SB=1; do echo "== $E"; env $E STRESS_N=30 timeout -k 10 400 python tools/serving_stress2.py 24 2 2>&1 | grep -E "8-piece generate beside text|Error"; done
