# deblock chroma tile height variants: parity of the product build and each variant, then the
# graph-timed deblock stage, alternating three times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_lf_base.log 2>&1; rc=$?; echo "base $(tail -1 gpurun_out/r5_lf_base.log)"; [ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so timeout -k 10 300 python -u -m pytest tests/test_lf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_lf_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/r5_lf_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for k in 1 2 3; do
  STAGE=deblock REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed 's/^/base /' || exit 1
  for v in "$@"; do
    MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so STAGE=deblock REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/$v /" || exit 1
  done
done
