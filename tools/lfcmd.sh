set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_intra_frame_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
for N in 8 16 24; do timeout -k 10 300 python -c "
import bench, json
from rav1d_amd.frame import Context
r = bench.intra_1080p8(Context(0), nframes=$N, ndesc=2)
print($N, r['ms_per_frame'], r['batch_ms'], r['mpx_per_s'])
" || exit 1; done
