#!/bin/bash
# GPU-box PMC passes over a short bench run (counters only with --kernel-trace, never with
# sys/runtime traces). Pass 1 FETCH_SIZE, pass 2 WRITE_SIZE (TCC slots cannot hold both),
# passes 3-4 SQ issue/stall counters. Each pass has its own time limit; stop at first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-pmc}
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
[ -n "$LIST" ] && { timeout -k 10 120 rocprofv3 -L > $OUT/$TAG/counters_list.txt 2>&1 || true; }
i=0
PASSES=("FETCH_SIZE" "WRITE_SIZE" \
        "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
        "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
# TRAFFIC_ONLY=1: just the two HBM byte passes
[ -n "$TRAFFIC_ONLY" ] && PASSES=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B")
# SQ_ONLY=1: just the two issue/stall passes
[ -n "$SQ_ONLY" ] && PASSES=("${PASSES[@]:2}") && i=2
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/$TAG/p$i -o p -- \
      python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify --no-two-in-flight $BENCH_ARGS > $OUT/$TAG/p$i.log 2>&1 \
      || { echo "pass $i failed"; tail -20 $OUT/$TAG/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT/$TAG > $OUT/$TAG/summary.txt && cat $OUT/$TAG/summary.txt
