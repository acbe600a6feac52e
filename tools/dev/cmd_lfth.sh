# occupancy / shape A/Bs: deblock tile height, MC waves per SIMD, itx rounds per workgroup
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bash tools/dev/ab2.sh deblock base th128 th32 || exit 1
timeout -k 10 300 bash tools/dev/ab2.sh mc base mcw6 mcw8 || exit 1
timeout -k 10 400 bash tools/dev/ab2.sh itx base r42 r48 r81 r84
