# bench A/B of library variants: bash tools/dev/ab2.sh STAGE v1 v2 ... (base = librav1d_amd.so), two passes
set -o pipefail
R=$PWD/rav1d_amd
ST=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  if [ $v = base ]; then L=$R/librav1d_amd.so; else L=$R/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify > gpurun_out/ab2_$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['stage_ms'][sys.argv[3]], d['stage_ms'])" gpurun_out/ab2_$v.json $v $ST
done
done
