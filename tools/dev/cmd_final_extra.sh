# extra steps of the round's last GPU pass: stage timings, LR / CDEF timelines, the executor's
# host pass with and without the level order, two frames in flight
set -o pipefail
STAGE=lr REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1
STAGE=cdef REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1
STAGE=deblock REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 || exit 1
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lr,cdef timeout -k 10 120 python -u tools/dev/ktl.py > gpurun_out/final_ktl.log 2>&1 || exit 1
grep -E "== |phase|type (0|2|3|13):" gpurun_out/final_ktl.log
for v in 0 1; do
  echo "== MI_IR_NOLEVELS=$v"
  MI_IR_NOLEVELS=$v MI_FX_PROFILE=1 timeout -k 10 200 python -u tools/dev/run_rs.py itut_t35_10bit 3 2>gpurun_out/rs_$v.err || exit 1
  grep "frame_run" gpurun_out/rs_$v.err | tail -4
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --two-in-flight --no-fg --no-intra --no-extra --no-cpu-baseline > gpurun_out/bench_two.json 2> gpurun_out/bench_two.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_two.json')); print('one', d['value'], 'two', d.get('two_frames_in_flight'))"
# LR with uniform-trip A/B loops (opt-in build): parity, then time against the product build
MI_LIB=$PWD/rav1d_amd/librav1d_amd_lru.so timeout -k 10 200 python -u -m pytest tests/test_lr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lru_t.log 2>&1; rc=$?; tail -1 gpurun_out/lru_t.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  STAGE=lr REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed 's/^/base /' || exit 1
  MI_LIB=$PWD/rav1d_amd/librav1d_amd_lru.so STAGE=lr REPS=1 TIME=1 timeout -k 10 120 python -u tools/dev/run_stage.py 2>&1 | tail -1 | sed 's/^/uniform /' || exit 1
done
