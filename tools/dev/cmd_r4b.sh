set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lf_gpu.py tests/test_pipeline_gpu.py tests/test_inloop_filters.py -p no:cacheprovider > gpurun_out/r4b_lf_t.log 2>&1; rc=$?; tail -2 gpurun_out/r4b_lf_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --no-fg --no-intra --no-extra > gpurun_out/r4b_bench.json 2>/dev/null || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print('bench',d['value'],d['stage_ms'],d.get('verified'))" gpurun_out/r4b_bench.json
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lf,itx timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4b_ktl.log 2>&1; echo "ktl rc=$?"; grep -A12 "== lf" gpurun_out/r4b_ktl.log
bash tools/dev/cmd_lrband.sh 2>&1 | grep -i "lrband\|rc\|fail\|passed"
for v in base no64 no64w6 t64 t64no64 t128 p4 p8 t64p16 p4n skel new; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
for v in base t64 t128 p4 p8 t64p16 p4n skel new; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  NO64=0 MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
timeout -k 10 900 bash tools/dev/pmc_passes.sh pmc_itx tools/dev/run_itx.py || exit 1
