# deblock 64x128 tiles (default) with 512-lane workgroups: parity with the variant library, then A/B
set -o pipefail
mkdir -p gpurun_out
MI_LIB=$PWD/rav1d_amd/librav1d_amd.so timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py tests/test_streams_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_lf128.log 2>&1; rc=$?; tail -2 gpurun_out/pt_lf128.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 bash tools/dev/ab2.sh deblock base th64
