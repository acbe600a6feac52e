# LR parity + timing + timelines (LR, CDEF), executor host-pass A/B (levels on / off)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_lr_gpu.py tests/test_cdef_gpu.py tests/test_pipeline_gpu.py tests/test_dsp_calls_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/combo_t.log 2>&1; rc=$?; tail -2 gpurun_out/combo_t.log; [ $rc -eq 0 ] || exit $rc
STAGE=lr REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1
STAGE=cdef REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lr,cdef timeout -k 10 120 python -u tools/dev/ktl.py > gpurun_out/combo_ktl.log 2>&1 || exit 1
grep -E "== |phase|type (0|2|3|13):" gpurun_out/combo_ktl.log
for v in 0 1; do
  echo "== MI_IR_NOLEVELS=$v"
  MI_IR_NOLEVELS=$v MI_FX_PROFILE=1 timeout -k 10 200 python -u tools/dev/run_rs.py itut_t35_10bit 3 2>gpurun_out/rs_$v.err || exit 1
  grep "frame_run" gpurun_out/rs_$v.err | tail -3
done
