set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cdef_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_cdeford2.log 2>&1; rc=$?; tail -1 gpurun_out/r5_cdeford2.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do for st in cdef cdef_grid; do STAGE=$st TIME=1 REPS=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | grep " us" || exit 1; done; done
