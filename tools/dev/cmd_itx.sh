set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 bash tools/dev/ab2.sh itx base w5 w6
