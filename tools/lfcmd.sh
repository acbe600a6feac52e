set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "deblock" > gpurun_out/pytest_lf.log 2>&1 || { tail -30 gpurun_out/pytest_lf.log; exit 1; }
tail -1 gpurun_out/pytest_lf.log
timeout -k 10 120 python tools/exp_lf.py tiles && timeout -k 10 120 python tools/exp_lf.py tiles noedges
