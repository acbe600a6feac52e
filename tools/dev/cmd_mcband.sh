# per-class XCD chunking of MC: parity tests, bench A/B (base vs mc0), then CDEF per-phase PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mc_gpu.py tests/test_mc_ext_gpu.py tests/test_streams_gpu.py tests/test_pipeline_gpu.py tests/test_sstream_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_mc.log 2>&1; rc=$?; tail -3 gpurun_out/pt_mc.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 bash tools/dev/ab2.sh mc base mc0 || exit 1
timeout -k 10 600 bash tools/dev/cmd_cdef_pmc.sh cd1 cd2 cd4 cd5
