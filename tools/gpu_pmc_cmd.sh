#!/bin/bash
# PMC passes over an arbitrary python command: bash tools/gpu_pmc_cmd.sh TAG "script.py args"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=$1; shift
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
         "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/$TAG/p$i -o p -- \
      python3 $R/$1 $2 > $OUT/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/$TAG/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT/$TAG > $OUT/$TAG/summary.txt && cat $OUT/$TAG/summary.txt
