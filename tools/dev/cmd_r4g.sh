set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lf_gpu.py tests/test_pipeline_gpu.py tests/test_inloop_filters.py tests/test_itx_gpu.py -p no:cacheprovider > gpurun_out/r4g_t.log 2>&1; rc=$?; tail -1 gpurun_out/r4g_t.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base p96 p112; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify > gpurun_out/r4g_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['stage_ms'])" gpurun_out/r4g_$v.json $v
done; done
STAGE=deblock timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_lfpad -o p -- python3 tools/dev/run_stage.py > gpurun_out/pmc_lfpad.log 2>&1 && python3 tools/pmc_summary.py gpurun_out/pmc_lfpad | grep -A6 lf_tile
