# per-size itx kernel durations (rocprof kernel trace) for each library variant given (base = product)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/rav1d_amd/librav1d_amd.so; else L=$GRAFT_REPO_ROOT/rav1d_amd/librav1d_amd_$v.so; fi
  mkdir -p $GRAFT_REPO_ROOT/gpurun_out/itxs_$v
  MI_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/itxs_$v -o k -- python3 $GRAFT_REPO_ROOT/tools/dev/itx_sizes.py > $GRAFT_REPO_ROOT/gpurun_out/itxs_$v/log.txt 2>&1 || exit 1
done
