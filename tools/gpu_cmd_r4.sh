timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_intra_frame_gpu.py tests/test_streams_gpu.py -p no:cacheprovider > gpurun_out/r4_t1.log 2>&1
rc=$?; tail -3 gpurun_out/r4_t1.log; [ $rc -eq 0 ] || exit $rc
MI_LIB=$PWD/rav1d_amd/librav1d_amd_wrap.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_intra_frame_gpu.py -k "saturates or test15549" tests/test_streams_gpu.py -p no:cacheprovider > gpurun_out/r4_t1_wrap.log 2>&1
echo "wrap rc=$?"; tail -5 gpurun_out/r4_t1_wrap.log
