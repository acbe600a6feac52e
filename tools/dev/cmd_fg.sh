set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fg_gpu.py tests/test_dsp_calls_gpu.py tests/test_streams_gpu.py -k "fg or grain or filmgrain" -x -q --timeout 120 --timeout-method thread > gpurun_out/fg_t.log 2>&1; rc=$?; tail -3 gpurun_out/fg_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/dev/run_fg.py && MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so timeout -k 10 120 python -u tools/dev/ktl_fg.py
