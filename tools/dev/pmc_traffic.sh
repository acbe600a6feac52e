# HBM bytes of one python command under MI_LIB (diagnostic): bash tools/dev/pmc_traffic.sh TAG script.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=$1; shift
mkdir -p $OUT/$TAG
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/$TAG/p$i -o p -- \
      python3 $R/$1 > $OUT/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/$TAG/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT/$TAG > $OUT/$TAG/summary.txt && grep -A12 "itx_frame_kernel<unsigned short, int, short" $OUT/$TAG/summary.txt | grep -E "hbm_bytes|write_bytes|fetch_bytes"
