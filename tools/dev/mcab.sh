# MC variants A/B on the bench (MC stage event time), each run twice
set -o pipefail
R=$PWD/rav1d_amd
for rep in 1 2; do
for v in base sb4 sb16 xc4 xc16 mu8; do
  if [ $v = base ]; then L=$R/librav1d_amd.so; else L=$R/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify > gpurun_out/mcab_$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['stage_ms']['mc'])" gpurun_out/mcab_$v.json $v
done
done
