set -o pipefail
mkdir -p gpurun_out
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=lf timeout -k 10 200 python tools/dev/ktl.py 2>&1 | tail -12
bash tools/dev/ab2.sh deblock base nof || exit 1
bash tools/dev/r5_pmc_ab.sh nof
