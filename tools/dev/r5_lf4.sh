set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lf_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_lf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5_lf_tests.log; [ $rc -eq 0 ] || exit $rc
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lf timeout -k 10 200 python tools/dev/ktl.py 2>&1 | grep -v amdgpu.ids | tail -10
bash tools/dev/ab2.sh deblock base tile sg64 || exit 1
