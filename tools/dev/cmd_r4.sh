set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dev/itx_sizes.py > gpurun_out/r4_itx_sizes.log 2>&1 || exit 1
cat gpurun_out/r4_itx_sizes.log
for v in base no64 no64w6 no64w8; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
timeout -k 10 900 bash tools/dev/pmc_passes.sh pmc_itx tools/dev/run_itx.py || exit 1
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4_ktl.log 2>&1; echo "ktl rc=$?"; cat gpurun_out/r4_ktl.log
timeout -k 10 60 ./tools/dev/anyorder_test
