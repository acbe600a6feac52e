# SQ LDS counters of cdef_kernel per library variant: bash tools/dev/cmd_cdef_pmc.sh v1 v2 ... (base = product)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/cdef_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then L=$R/rav1d_amd/librav1d_amd.so; else L=$R/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES \
      --kernel-trace --output-format csv -d $OUT/$v -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify \
      > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -20 $OUT/$v.log; exit 1; }
  echo "== $v"; python3 $R/tools/pmc_summary.py $OUT/$v | grep -A8 '^cdef_kernel'
done
