set -o pipefail
mkdir -p gpurun_out
for st in deblock cdef lr; do
  STAGE=$st timeout -k 10 900 bash tools/dev/pmc_passes.sh pmc_$st tools/dev/run_stage.py > gpurun_out/pmc_$st.txt 2>&1 || { echo "pmc $st failed"; tail gpurun_out/pmc_$st.txt; exit 1; }
  grep -A40 -E "^(lf_tile|cdef_kernel|lr_kernel)" gpurun_out/pmc_$st/summary.txt | head -42
done
