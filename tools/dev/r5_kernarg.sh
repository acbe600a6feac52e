# itx workgroup front (timeline build) with kernel arguments in device memory or not
set -o pipefail
for v in 0 1; do
  HIP_FORCE_DEV_KERNARG=$v MI_LIB=$PWD/rav1d_amd/librav1d_amd_ktl.so KTL_UNITS=itx timeout -k 10 300 python tools/dev/ktl.py > gpurun_out/ktl_itx_ka$v.txt 2>&1 || exit 1
  python -c "
import numpy as np
a=np.load('gpurun_out/ktl_itx.npy')
ok=(a[:,3]!=0)&(a[:,3]>=a[:,0])&(a[:,1]>=a[:,3])
print('HIP_FORCE_DEV_KERNARG=$v', 'start->karg %.2f' % np.mean((a[ok,3]-a[ok,0])/100.0), 'karg->desc %.2f' % np.mean((a[ok,1]-a[ok,3])/100.0))
"
  grep "== itx" gpurun_out/ktl_itx_ka$v.txt
done
for v in 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-fg --no-intra --no-extra > gpurun_out/ka_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ka_$v.json'));print('bench HIP_FORCE_DEV_KERNARG=$v', d['value'], d['ms_per_step'], d['stage_ms'])"
done
