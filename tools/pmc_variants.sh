#!/bin/bash
# SQ counter pass over the bench for each library variant: bash tools/pmc_variants.sh TAG v1 v2 ...
# ("base" = librav1d_amd.so). Each rocprofv3 run has its own time limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then L=$R/rav1d_amd/librav1d_amd.so; else L=$R/rav1d_amd/librav1d_amd_$v.so; fi
  export MI_LIB=$L
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
      --kernel-trace --output-format csv -d $OUT/$v -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fg \
      > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -20 $OUT/$v.log; exit 1; }
  python3 $R/tools/pmc_summary.py $OUT/$v | grep -A12 '^mc_kernel' > $OUT/$v.txt
  echo "== $v"; cat $OUT/$v.txt
done
