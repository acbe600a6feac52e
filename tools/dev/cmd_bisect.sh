# one reference vector: determinism (3 runs) and with the intra hand-off variants (env toggles)
set -o pipefail
V=${1:-test15549_5522_4902}
for i in 1 2 3; do timeout -k 10 120 python -u tools/dev/one_vector.py $V || exit 1; done
MI_IR_GRANULES=0 timeout -k 10 120 python -u tools/dev/one_vector.py $V || exit 1
MI_IR_STRIPS=1 timeout -k 10 120 python -u tools/dev/one_vector.py $V || exit 1
MI_IR_GRANULES=0 MI_IR_STRIPS=1 timeout -k 10 120 python -u tools/dev/one_vector.py $V || exit 1
