# the failing vector at several persistent-intra worker counts
set -o pipefail
for w in 64 128 192 256; do
  MI_IR_WORKERS=$w MI_VDIR=sweep_one timeout -k 10 120 python -u tools/dev/one_vector.py test15549_5522_4902 | sed "s/^/workers $w /" || exit 1
done
