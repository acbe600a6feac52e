#!/bin/bash
# itx stage (graph-timed) of the 4K10 bench frame: product library on the packed arena, the
# product library on the dense arena (DENSE=1), and a variant library ($1, dense arena), in turn.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
for k in 1 2 3; do
  STAGE=itx REPS=1 TIME=1 timeout -k 10 120 python -u $R/tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/packed /" || exit 1
  DENSE=1 STAGE=itx REPS=1 TIME=1 timeout -k 10 120 python -u $R/tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/dense /" || exit 1
  [ -n "$1" ] && { MI_LIB=$R/rav1d_amd/librav1d_amd_$1.so DENSE=1 STAGE=itx REPS=1 TIME=1 timeout -k 10 120 python -u $R/tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/$1-dense /" || exit 1; }
done
exit 0
