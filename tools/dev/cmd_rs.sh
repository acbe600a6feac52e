set -o pipefail
for v in 0 1; do
  echo "== MI_IR_NOLEVELS=$v"
  MI_IR_NOLEVELS=$v MI_FX_PROFILE=1 timeout -k 10 200 python -u tools/dev/run_rs.py itut_t35_10bit 3 2>gpurun_out/rs_$v.err || exit 1
  grep "frame_run" gpurun_out/rs_$v.err | tail -4
done
