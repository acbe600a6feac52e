#!/bin/bash
# A/B of library variants on one stage, on the GPU box (replaces round 5's r5_*.sh one-offs):
#   STAGE=deblock TESTS="tests/test_lf_gpu.py" PASSES=3 bash tools/dev/ab_variants.sh v1 v2 ...
# Each variant librav1d_amd_<v>.so (rav1d_amd/build.py MI_BUILD_VARIANT=<v>) first passes
# TESTS ("-" skips), then the graph-timed STAGE (tools/dev/run_stage.py) runs for "base" (the
# product library) and every variant in turn, PASSES times, so drifts of the box hit all arms.
# BENCH=1 times the whole headline step (bench.py) instead of one stage. Every GPU step runs
# under its own time limit and the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/ab
mkdir -p $OUT
lib_of() { if [ "$1" = base ]; then echo $R/rav1d_amd/librav1d_amd.so; else echo $R/rav1d_amd/librav1d_amd_$1.so; fi; }
if [ "${TESTS:--}" != "-" ]; then
  for v in "$@"; do
    MI_LIB=$(lib_of $v) timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $OUT/test_$v.log 2>&1
    rc=$?; echo "$v tests: $(tail -1 $OUT/test_$v.log)"; [ $rc -eq 0 ] || exit $rc
  done
fi
for k in $(seq ${PASSES:-3}); do
  for v in base "$@"; do
    if [ "${BENCH:-0}" = 1 ]; then
      MI_LIB=$(lib_of $v) timeout -k 10 200 python $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-fg --no-intra --no-extra > $OUT/bench_${v}_$k.json || { echo "$v bench failed"; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d.get('verified'), d.get('stage_ms'))" $OUT/bench_${v}_$k.json $v
    else
      MI_LIB=$(lib_of $v) STAGE=${STAGE:?set STAGE} REPS=1 TIME=1 timeout -k 10 120 python -u $R/tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/$v /" || exit 1
    fi
  done
done
