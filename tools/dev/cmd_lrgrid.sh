# LR grid order A/B: time (graph replay) and HBM traffic per MI_LR_BANDS mode
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
for m in ${MODES:-0 1 2}; do
  MI_LR_BANDS=$m STAGE=lr REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1
  MI_LR_BANDS=$m STAGE=lr REPS=5 bash tools/dev/pmc_traffic.sh lrgrid$m tools/dev/run_stage.py > /dev/null 2>&1
  grep -A40 "^lr_kernel" gpurun_out/lrgrid$m/summary.txt | grep -E "hbm_bytes|write_bytes|fetch_bytes" | head -3
done
