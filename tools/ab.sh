#!/bin/bash
# A/B timing of library variants on the GPU box: bash tools/ab.sh TESTS v1 v2 ...
# TESTS: pytest selector run against each variant first ("-" to skip); variant "base" is the
# product librav1d_amd.so, others librav1d_amd_<v>.so (rav1d_amd/build.py MI_BUILD_VARIANT).
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/ab
mkdir -p $OUT
T=$1; shift
for v in "$@"; do
  if [ $v = base ]; then L=$R/rav1d_amd/librav1d_amd.so; else L=$R/rav1d_amd/librav1d_amd_$v.so; fi
  if [ "$T" != "-" ]; then
    MI_LIB=$L timeout -k 10 300 python -m pytest $T -x -q > $OUT/test_$v.log 2>&1 || { echo "$v: tests failed"; tail -20 $OUT/test_$v.log; exit 1; }
    echo "$v: $(tail -1 $OUT/test_$v.log)"
  fi
done
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = base ]; then L=$R/rav1d_amd/librav1d_amd.so; else L=$R/rav1d_amd/librav1d_amd_$v.so; fi
    MI_LIB=$L timeout -k 10 200 python $R/bench.py --steps 50 --no-cpu-baseline --no-fg > $OUT/bench_${v}_$rep.json || { echo "$v bench failed"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['stage_ms'])" $OUT/bench_${v}_$rep.json $v
  done
done
