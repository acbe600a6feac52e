set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lf_t.log 2>&1; rc=$?; tail -2 gpurun_out/lf_t.log; [ $rc -eq 0 ] || exit $rc
STAGE=deblock REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lf timeout -k 10 120 python -u tools/dev/ktl.py | grep -A9 "== lf"
