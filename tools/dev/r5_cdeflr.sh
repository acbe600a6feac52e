# round 5: fused CDEF + LR parity, stream vectors through the executor, stage timings, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cdef_lr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_cdeflr_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r5_cdeflr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_pipeline_gpu.py tests/test_cdef_gpu.py tests/test_lr_gpu.py tests/test_streams_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_cdeflr_suite.log 2>&1; rc=$?; tail -3 gpurun_out/r5_cdeflr_suite.log; [ $rc -eq 0 ] || exit $rc
for st in cdef lr cdef_lr; do STAGE=$st TIME=1 REPS=1 timeout -k 10 300 python tools/dev/run_stage.py 2>&1 | grep " us" || exit 1; done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5_cdeflr_bench.json 2> gpurun_out/r5_cdeflr_bench.err; rc=$?; tail -c 1500 gpurun_out/r5_cdeflr_bench.json; exit $rc
