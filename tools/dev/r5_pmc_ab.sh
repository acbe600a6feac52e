# SQ counter passes (tools/gpu_pmc.sh SQ_ONLY) of the product library and variants: r5_pmc_ab.sh v1 v2 ...
set -o pipefail
for v in "$@"; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L SQ_ONLY=1 bash tools/gpu_pmc.sh pmc_$v > /dev/null 2>&1 || { echo "pmc $v failed"; exit 1; }
  echo "== $v"; grep -A40 "^lf_" gpurun_out/pmc_$v/summary.txt | grep -E "^lf_|SQ_INSTS|SQ_WAIT|SQ_WAVE|SQ_LDS|SQ_ACTIVE_INST_ANY|GRBM_GUI"
done
