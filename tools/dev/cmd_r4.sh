set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fg_gpu.py tests/test_output_gpu.py tests/test_streams_gpu.py -k "grain or fg or film or output or 5606" -p no:cacheprovider > gpurun_out/r4_fg.log 2>&1; rc=$?; tail -3 gpurun_out/r4_fg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-intra --no-extra > gpurun_out/r4_fgbench.json 2> gpurun_out/r4_fgbench.err; python -c "import json;d=json.load(open('gpurun_out/r4_fgbench.json'));print(d.get('film_grain_8k10'))"
bash tools/dev/cmd_lfseg.sh || exit 1
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4_ktl.log 2>&1; echo "ktl rc=$?"; cat gpurun_out/r4_ktl.log
MI_LF_SEGH=128 MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lf timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4_ktl_seg.log 2>&1; echo "ktl seg rc=$?"; cat gpurun_out/r4_ktl_seg.log
timeout -k 10 60 ./tools/dev/anyorder_test
timeout -k 10 300 python -u tools/dev/itx_sizes.py > gpurun_out/r4_itx_sizes.log 2>&1 || exit 1
cat gpurun_out/r4_itx_sizes.log
for v in base no64 no64w6; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
timeout -k 10 900 bash tools/dev/pmc_passes.sh pmc_itx tools/dev/run_itx.py || exit 1
