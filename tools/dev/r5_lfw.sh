set -o pipefail
mkdir -p gpurun_out
MI_LIB=$PWD/rav1d_amd/librav1d_amd_wagg.so timeout -k 10 600 python -u -m pytest tests/test_lf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_lf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5_lf_tests.log; [ $rc -eq 0 ] || exit $rc
STAGE=deblock VARIANT=wagg bash tools/dev/ab_stage.sh || exit 1
