# itx variants: parity (itx + pipeline GPU tests) then graph-timed itx stage of base and each, 3 passes
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so timeout -k 10 400 python -u -m pytest tests/test_itx_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_itx_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/r5_itx_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for k in 1 2 3; do
  STAGE=itx REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed 's/^/base /' || exit 1
  for v in "$@"; do
    MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so STAGE=itx REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/$v /" || exit 1
  done
done
