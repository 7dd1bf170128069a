set -o pipefail
STRESS_N=24 timeout -k 10 400 python tools/serving_stress2.py 24 2 2>&1 | grep -E "pieces beside|Error" | tail -4
