set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_itx_gpu.py -p no:cacheprovider > gpurun_out/r4d_itx_t.log 2>&1; rc=$?; tail -1 gpurun_out/r4d_itx_t.log; [ $rc -eq 0 ] || exit $rc
MI_LIB=$PWD/rav1d_amd/librav1d_amd_t64.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_itx_gpu.py -p no:cacheprovider > gpurun_out/r4d_itx_t64.log 2>&1; rc=$?; tail -1 gpurun_out/r4d_itx_t64.log; [ $rc -eq 0 ] || exit $rc
for o in 8 1; do
for v in old base r1 r4 t64 t64r1 t64r4; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  echo -n "order $o: "; MI_SYNTH_ITX_ROUNDS=$o NO64=0 MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
done
for v in base t64 r1; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  echo "traffic $v"; MI_LIB=$L timeout -k 10 300 bash tools/dev/pmc_traffic.sh tr_$v tools/dev/run_itx.py || exit 1
done
