set -o pipefail
STRESS_N=20 timeout -k 10 500 python tools/serving_stress2.py 24 2 2>&1 | grep -E "beside packed|beside text|Error|error"
