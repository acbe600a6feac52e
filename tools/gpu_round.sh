#!/bin/bash
# One GPU-box pass: the -m gpu suite, smoke, the bench, then optional extra steps ($EXTRA, a
# command line run last). Every step under its own time limit; a step killed by its limit, a
# fault or an abort stops the script (nothing more runs on the GPU in this call).
# usage: bash tools/gpu_round.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r}
mkdir -p $OUT
stop() { case $1 in 124|137|134|139|132|135|136) echo "stopping after rc=$1 ($2)"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu_$TAG.log; stop $rc pytest
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
rc=$?; tail -1 $OUT/smoke_$TAG.log; stop $rc smoke
timeout -k 10 420 python -u $R/bench.py --steps 20 --warmup 5 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; tail -c 400 $OUT/bench_$TAG.err; stop $rc bench
if [ -n "$EXTRA" ]; then
  bash -c "$EXTRA"
  rc=$?; stop $rc extra
fi
exit 0
