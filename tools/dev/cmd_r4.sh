set -o pipefail
mkdir -p gpurun_out
NEW=$PWD/rav1d_amd/librav1d_amd_new.so
# 1. the candidate library (pair-split 64-point itx, barrier-free film-grain AR) through the GPU suite parts it touches
MI_LIB=$NEW timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_itx_gpu.py tests/test_fg_gpu.py tests/test_output_gpu.py tests/test_pipeline_gpu.py -p no:cacheprovider > gpurun_out/r4_new_t.log 2>&1; echo "new lib tests rc=$?"; tail -3 gpurun_out/r4_new_t.log
# 2. streaming deblock parity + A/B
bash tools/dev/cmd_lfseg.sh; echo "lfseg rc=$?"
# 3. timelines
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4_ktl.log 2>&1; echo "ktl rc=$?"; cat gpurun_out/r4_ktl.log
MI_LF_SEGH=128 MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lf timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4_ktl_seg.log 2>&1; echo "ktl seg rc=$?"; cat gpurun_out/r4_ktl_seg.log
timeout -k 10 60 ./tools/dev/anyorder_test
# 4. itx variants (64-class excluded, then all)
for v in base no64 no64w6 t64 t64no64 t128 new p4 p8 t64p16 p4n skel; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
for v in base t64 t128 new p4 p8 t64p16 p4n skel; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  NO64=0 MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
timeout -k 10 300 python -u tools/dev/itx_sizes.py > gpurun_out/r4_itx_sizes.log 2>&1 || exit 1
cat gpurun_out/r4_itx_sizes.log
MI_LIB=$NEW timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-intra --no-extra > gpurun_out/r4_fgbench.json 2> gpurun_out/r4_fgbench.err; python -c "import json;d=json.load(open('gpurun_out/r4_fgbench.json'));print(d.get('film_grain_8k10'), d['stage_ms'])"
timeout -k 10 900 bash tools/dev/pmc_passes.sh pmc_itx tools/dev/run_itx.py || exit 1
