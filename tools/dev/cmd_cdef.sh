# CDEF change: parity (cdef / stream / pipeline GPU tests) then bench timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cdef_gpu.py tests/test_streams_gpu.py tests/test_pipeline_gpu.py tests/test_inloop_filters.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_cdef.log 2>&1; rc=$?; tail -3 gpurun_out/pt_cdef.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 bash tools/dev/ab2.sh cdef base
