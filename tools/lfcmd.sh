set -o pipefail
cd $GRAFT_REPO_ROOT
for v in tw32 tw64; do MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "deblock and tiles" > gpurun_out/pytest_lf.log 2>&1 || { tail -30 gpurun_out/pytest_lf.log; exit 1; }; tail -1 gpurun_out/pytest_lf.log; MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so timeout -k 10 120 python tools/exp_lf.py tiles; done
