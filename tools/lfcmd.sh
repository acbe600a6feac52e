set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "itx" > gpurun_out/pytest_q.log 2>&1 || { tail -40 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
timeout -k 10 300 python tools/exp_itx.py short
