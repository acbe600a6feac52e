set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_dsp_calls_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { tail -40 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
