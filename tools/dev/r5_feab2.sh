# front-end A/B on the GPU box's CPU share: the committed library (libmi_av1dec_base.so, built
# from HEAD) against the working tree's, one temporal unit at a time and pipelined; then the
# unpipelined trace of issue_295 and the bench's real-stream breakdown
set -o pipefail
R=$PWD/rav1d_amd
for la in 0 ""; do
  echo "LOOKAHEAD=${la:-pipelined}"
  LOOKAHEAD=$la timeout -k 10 400 python tools/dev/fe_ab.py $R/libmi_av1dec_base.so $R/libmi_av1dec.so issue_295,issue_318,00001141,itut_t35_10bit 7 8 || exit 1
done
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_fe.json 2> gpurun_out/bench_fe.err || { tail -5 gpurun_out/bench_fe.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_fe.json"))
print("value", d["value"], d["ms_per_step"])
for n, v in d.get("real_streams", {}).items():
    print(n, v["gpu_ms"], "fe", v["stages_ms"]["front_end_ms"], "fe_pipe", v["stages_pipelined_ms"]["front_end_ms"], "host", v["stages_ms"]["run_host_ms"], v["md5_verified"])
PY
