set -o pipefail
mkdir -p gpurun_out
for v in ktl lf64 lf96; do
  echo "== variant $v"; MI_LIB=$PWD/rav1d_amd/librav1d_amd_$v.so KTL_UNITS=lf timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4e_ktl_$v.log 2>&1 || { echo fail; cat gpurun_out/r4e_ktl_$v.log | tail; exit 1; }
  grep -A9 "== lf" gpurun_out/r4e_ktl_$v.log
done
MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=itx,cdef,lr timeout -k 10 300 python -u tools/dev/ktl.py > gpurun_out/r4e_ktl_all.log 2>&1; cat gpurun_out/r4e_ktl_all.log | grep -v "size "
