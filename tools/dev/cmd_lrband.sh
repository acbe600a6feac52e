# loop restoration over picture bands (diagnostic)
set -o pipefail
mkdir -p gpurun_out
MI_LR_BANDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lr_gpu.py tests/test_pipeline_gpu.py -p no:cacheprovider > gpurun_out/r4_lrband_t.log 2>&1; rc=$?; tail -2 gpurun_out/r4_lrband_t.log; [ $rc -eq 0 ] || exit $rc
for b in 0 1 0 1; do
  MI_LR_BANDS=$b timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify > gpurun_out/r4_lrband_$b.json 2>/dev/null || { echo "bench lr $b failed"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print('lrband',sys.argv[2],d['value'],d['stage_ms']['lr'])" gpurun_out/r4_lrband_$b.json $b
done
