set -o pipefail
cd $GRAFT_REPO_ROOT
for v in base mc4 mc16 mc64; do
  L=$PWD/rav1d_amd/librav1d_amd_$v.so; [ $v = base ] && L=$PWD/rav1d_amd/librav1d_amd.so
  MI_LIB=$L timeout -k 10 200 python tools/exp_mc.py > gpurun_out/exp_mc_$v.log 2>&1 || { tail gpurun_out/exp_mc_$v.log; exit 1; }
  echo $v $(head -1 gpurun_out/exp_mc_$v.log)
done
