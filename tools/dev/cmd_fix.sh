# 12-bit intra row buffer in its own LDS: the failing vector, the intra / stream GPU tests, every vector
set -o pipefail
mkdir -p gpurun_out
MI_VDIR=sweep_one timeout -k 10 120 python -u tools/dev/one_vector.py test15549_5522_4902 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_streams_gpu.py tests/test_intra_frame_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_fix.log 2>&1; rc=$?; tail -1 gpurun_out/pt_fix.log; [ $rc = 0 ] || exit $rc
[ -d sweep_vectors ] || exit 0
timeout -k 10 800 python -u tools/gpu_sweep.py run sweep_vectors gpurun_out/sweep_s4.jsonl > gpurun_out/sweep_s4.log 2>&1; rc=$?; tail -1 gpurun_out/sweep_s4.log; exit $rc
