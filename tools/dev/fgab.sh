# film grain 8K10 apply A/B of library variants (bench's film_grain_8k10 entry), two passes
set -o pipefail
R=$PWD/rav1d_amd
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  if [ $v = base ]; then L=$R/librav1d_amd.so; else L=$R/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --no-intra --no-extra --no-verify > gpurun_out/fgab_$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['film_grain_8k10'])" gpurun_out/fgab_$v.json $v
done
done
