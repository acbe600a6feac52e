# LR tile->XCD mapping variants and CDEF store-width diagnostics (bench A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 bash tools/dev/ab2.sh lr base lr1 lr8 lr30 || exit 1
timeout -k 10 300 bash tools/dev/ab2.sh cdef base cd6 cd7
