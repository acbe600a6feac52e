set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_itx_gpu.py tests/test_pipeline_gpu.py -p no:cacheprovider > gpurun_out/r4c_itx_t.log 2>&1; rc=$?; tail -2 gpurun_out/r4c_itx_t.log; [ $rc -eq 0 ] || exit $rc
for v in base r1 r4 r16 t64 t64r1; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  NO64=0 MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
for v in base r1 t64; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  echo "traffic $v"; MI_LIB=$L timeout -k 10 300 bash tools/dev/pmc_traffic.sh tr_$v tools/dev/run_itx.py || exit 1
done
timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --no-fg --no-intra --no-extra > gpurun_out/r4c_bench.json 2>/dev/null || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print('bench',d['value'],d['stage_ms'],d.get('verified'))" gpurun_out/r4c_bench.json
