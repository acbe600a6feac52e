# MC hand-off with an agent acquire after the poll (variant librav1d_amd_acq.so) against the
# product's sc1-only consumer: parity, then the graph-timed one-grid MC stage alternating
set -o pipefail
mkdir -p gpurun_out
MI_LIB=$PWD/rav1d_amd/librav1d_amd_acq.so timeout -k 10 400 python -u -m pytest tests/test_mc_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_acq_t.log 2>&1; rc=$?; echo "acq tests: $(tail -1 gpurun_out/r5_acq_t.log)"; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  STAGE=mc_sync REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/base /" || exit 1
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_acq.so STAGE=mc_sync REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/acq /" || exit 1
done
