# A/B of one stage: product library vs $VARIANT (graph-timed), alternating 3 times
set -o pipefail
for k in 1 2 3; do
  STAGE=$STAGE REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed 's/^/new /' || exit 1
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$VARIANT.so STAGE=$STAGE REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/$VARIANT /" || exit 1
done
