# round-4 GPU step: intra + stream parity, the red check against the unfixed kernel, itx timing, quick bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_intra_frame_gpu.py tests/test_streams_gpu.py -p no:cacheprovider > gpurun_out/r4_t1.log 2>&1
rc=$?; tail -3 gpurun_out/r4_t1.log; [ $rc -eq 0 ] || exit $rc
MI_LIB=$PWD/rav1d_amd/librav1d_amd_wrap.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_intra_frame_gpu.py -k "saturates or test15549" tests/test_streams_gpu.py -p no:cacheprovider > gpurun_out/r4_t1_wrap.log 2>&1
echo "wrap rc=$?"; tail -5 gpurun_out/r4_t1_wrap.log
timeout -k 10 300 python -u tools/dev/itx_sizes.py > gpurun_out/r4_itx_sizes.log 2>&1 || exit 1
cat gpurun_out/r4_itx_sizes.log
for v in base no64 no64w6 no64w8; do
  if [ $v = base ]; then L=$PWD/rav1d_amd/librav1d_amd.so; else L=$PWD/rav1d_amd/librav1d_amd_$v.so; fi
  MI_LIB=$L timeout -k 10 120 python -u tools/dev/exp_itx_sub.py || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench0.json 2> gpurun_out/r4_bench0.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r4_bench0.json'));print(d['value'],d.get('stage_ms'),d.get('stage_roofline'))"
