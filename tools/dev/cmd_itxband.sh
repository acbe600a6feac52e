# banded itx: parity tests, then bench A/B (MI_ITX_BANDED=1 default vs 0), then CDEF per-phase PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_itx_gpu.py tests/test_streams_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_itx.log 2>&1; rc=$?; tail -3 gpurun_out/pt_itx.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
for b in 1 0; do
  MI_ITX_BANDED=$b timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify > gpurun_out/band_$b.json 2>/dev/null || { echo "band $b failed"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print('banded', sys.argv[2], d['value'], d['stage_ms'])" gpurun_out/band_$b.json $b
done
done
[ -n "$NOPMC" ] || timeout -k 10 600 bash tools/dev/cmd_cdef_pmc.sh base cd1 cd2 cd4 cd5
