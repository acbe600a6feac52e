set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py tests/test_streams_gpu.py tests/test_inloop_filters.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_lf.log 2>&1; rc=$?; tail -3 gpurun_out/pt_lf.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 bash tools/dev/ab2.sh deblock base latom nofilt nofnof
