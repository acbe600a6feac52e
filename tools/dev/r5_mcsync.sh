# mi_mc_frame_sync: parity (MC GPU tests incl. the sync cases) then graph-timed MC stage
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mc_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_mcsync_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r5_mcsync_tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do for st in mc mc_sync mc_onegrid; do STAGE=$st REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1; done; done
