set -o pipefail
R=$PWD/rav1d_amd
timeout -k 10 200 python -m pytest -x -q tests/test_itx_gpu.py 2>&1 | tail -2 || exit 1
for v in librav1d_amd.so librav1d_amd_nocap.so librav1d_amd_r1.so librav1d_amd_r8.so; do
  echo "== $v"; MI_LIB=$R/$v timeout -k 10 120 python tools/dev/exp_itx.py 2>&1 | grep -v amdgpu | head -8
done
