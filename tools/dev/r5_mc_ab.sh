set -o pipefail
mkdir -p gpurun_out
for v in w8 w6 b4 b4w8; do
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_mc_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/r5_mc_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/dev/ab2.sh mc base w8 w6 b4 b4w8
