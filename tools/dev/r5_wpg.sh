# MC with 2 / 4 independent waves per workgroup (MI_MC_WPG): parity against the oracle with each
# variant, then the graph-timed one-grid MC stage and the bench, alternating with the product
set -o pipefail
mkdir -p gpurun_out
for V in wpg2 wpg4; do
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_$V.so timeout -k 10 400 python -u -m pytest tests/test_mc_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_wpg_t_$V.log 2>&1; rc=$?; echo "$V tests: $(tail -1 gpurun_out/r5_wpg_t_$V.log)"; [ $rc -eq 0 ] || exit $rc
done
for k in 1 2 3; do
  for V in base wpg2 wpg4; do
    L=""; [ $V = base ] || L=$PWD/rav1d_amd/librav1d_amd_$V.so
    MI_LIB=$L STAGE=mc_sync REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed "s/^/$V /" || exit 1
  done
done
for k in 1 2; do
  for V in base wpg2 wpg4; do
    L=""; [ $V = base ] || L=$PWD/rav1d_amd/librav1d_amd_$V.so
    MI_LIB=$L timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-fg --no-intra --no-extra > gpurun_out/r5_wpg_b_$V.json 2>gpurun_out/r5_wpg_b_$V.err || { tail -5 gpurun_out/r5_wpg_b_$V.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/r5_wpg_b_$V.json').read().strip().splitlines()[-1]);print('$V bench',d['value'],d['ms_per_step'])"
  done
done
