#!/bin/bash
# LR order dealt to the XCDs (librav1d_amd_lrdeal.so) against the product: parity, graph-timed
# stage alternating, then HBM bytes of the LR stage under each (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
STAGE=lr TESTS="tests/test_lr_gpu.py" PASSES=3 bash $R/tools/dev/ab_variants.sh lrdeal || exit 1
for v in base lrdeal; do
  lib=$R/rav1d_amd/librav1d_amd.so; [ $v = base ] || lib=$R/rav1d_amd/librav1d_amd_$v.so
  MI_LIB=$lib STAGE=lr REPS=5 bash $R/tools/dev/pmc_traffic.sh lrpmc_$v tools/dev/run_stage.py > /dev/null 2>&1 || { echo "pmc $v failed"; exit 1; }
  echo "$v"; grep -A14 "^lr_kernel<unsigned short>" $R/gpurun_out/lrpmc_$v/summary.txt | grep -E "hbm_bytes|write_bytes|fetch_bytes|_dispatches"
done
