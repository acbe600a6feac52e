set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cdef_lr_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5_cdeflr_dbg.log 2>&1; rc=$?; grep -E "differ|passed|failed" gpurun_out/r5_cdeflr_dbg.log | head -20; exit $rc
