#!/bin/bash
# quick GPU loop: selected tests (-k expr) + bench (no cpu baseline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "$1" > $OUT/pytest_quick.log 2>&1 || { tail -30 $OUT/pytest_quick.log; exit 1; }
tail -2 $OUT/pytest_quick.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_quick.json 2> $OUT/bench_quick.err || { tail -20 $OUT/bench_quick.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_quick.json')); print(d['value'], d['ms_per_step'], d['stage_ms'], d['stage_gbs'])"
