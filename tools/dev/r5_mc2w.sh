# MC variant: parity (MC + pipeline GPU tests), then bench A/B of the mc stage (tools/dev/ab2.sh)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so timeout -k 10 400 python -u -m pytest tests/test_mc_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_mc_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/r5_mc_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/dev/ab2.sh mc base "$@" || exit 1
