#!/bin/bash
# One GPU-box profiling pass for the round's evidence under gpurun_out/$TAG:
#   1. PMC calibration (tools/pmc_calib): FETCH_SIZE and WRITE_SIZE per access width
#   2. bench under rocprofv3 --kernel-trace --stats (kernel durations vs the bench's events)
#   3. FETCH_SIZE / WRITE_SIZE passes over the bench (tools/gpu_pmc.sh TRAFFIC_ONLY)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-prof}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -x $R/tools/pmc_calib ] || { echo "tools/pmc_calib not built"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; do
  D=${C%% *}
  timeout -k 10 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/calib_$D -o p -- \
      $R/tools/pmc_calib > $OUT/calib_$D.log 2>&1 || { echo "calib $D failed"; tail -20 $OUT/calib_$D.log; exit 1; }
done
echo "calibration done"
# the headline command alone (no real-stream / intra / grain legs), so that the per-kernel averages
# are the headline's launches, comparable with the bench's event-timed launch_us
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o p -- \
    python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fg --no-intra --no-extra --no-two-in-flight > $OUT/bench_stats.json 2> $OUT/bench_stats.err \
    || { echo "stats run failed"; tail -20 $OUT/bench_stats.err; exit 1; }
echo "kernel stats done"; cat $OUT/bench_stats.json
TRAFFIC_ONLY=1 bash $R/tools/gpu_pmc.sh $TAG/pmc > /dev/null || { echo "pmc failed"; exit 1; }
python3 $R/tools/traffic_json.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
# the same passes on the coherent motion field (bench --mv coherent): MC traffic beside the uniform one
BENCH_ARGS="--mv coherent" TRAFFIC_ONLY=1 bash $R/tools/gpu_pmc.sh $TAG/pmc_coh > /dev/null || { echo "pmc (coherent) failed"; exit 1; }
python3 $R/tools/traffic_json.py $OUT pmc_coh > $OUT/traffic_coherent.json && echo "coherent traffic done"
