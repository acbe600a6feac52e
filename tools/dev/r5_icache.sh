# instruction-cache counters of the itx stage (and deblock for comparison), one PMC pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for st in itx deblock; do
  STAGE=$st REPS=5 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d $R/gpurun_out/icache_$st -o p -- python3 $R/tools/dev/run_stage.py > $R/gpurun_out/icache_$st.log 2>&1 || { echo "pmc $st failed"; tail -5 $R/gpurun_out/icache_$st.log; exit 1; }
done
echo done
