# round 5: stream vectors with the front-end's intra queue / the executor's own plan, real streams
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_streams_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_q_streams.log 2>&1; rc=$?; tail -3 gpurun_out/r5_q_streams.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -c "
import json,sys,torch
sys.path.insert(0,'.')
import bench
from rav1d_amd import frame as F
ctx=F.Context(0)
r=bench.real_streams(ctx)
json.dump(r,open('gpurun_out/r5_q_real_streams.json','w'),indent=1)
for k,v in r.items(): print(k, v['md5_verified'], v['gpu_ms'], v['stages_ms']['front_end_ms'], v['stages_ms']['run_host_ms'], v['front_end_only_ms'], v['front_end_8_threads_ms'])
"
