set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lf_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_lf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5_lf_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/dev/ab2.sh deblock base tile || exit 1
bash tools/dev/r5_pmc_ab.sh base tile
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5_prof2 -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify > $GRAFT_REPO_ROOT/gpurun_out/r5_prof2.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r5_prof2 -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-4 | grep -E "lf_|itx|cdef|lr_"
