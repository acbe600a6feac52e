set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/dev/inflight.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5_inflight.txt
