#!/bin/bash
# GPU-box check: full -m gpu suite, smoke, bench, rocprof kernel stats. Each GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-run}
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -3 $OUT/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o k -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || { tail -20 $OUT/prof_$TAG.log; exit 1; }
find $OUT/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \;
