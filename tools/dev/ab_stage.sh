# A/B of one bench stage: product library vs the variant library librav1d_amd_$VARIANT.so
# (parity tests $TESTS against the variant first; graph-timed stage, alternating 3 times)
# usage: STAGE=cdef VARIANT=cdl TESTS=tests/test_cdef_gpu.py bash tools/dev/ab_stage.sh
set -o pipefail
if [ -n "$TESTS" ]; then
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$VARIANT.so timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_t.log 2>&1; rc=$?; tail -1 gpurun_out/ab_t.log; [ $rc -eq 0 ] || exit $rc
fi
for k in 1 2 3; do
  STAGE=$STAGE REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed 's/^/base /' || exit 1
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$VARIANT.so STAGE=$STAGE REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/$VARIANT /" || exit 1
done
