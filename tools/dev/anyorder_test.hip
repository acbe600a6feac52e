// Does hipExtAnyOrderLaunch let two kernels of one stream overlap on gfx950? Kernel A: 8
// workgroups that sleep ~50 us; kernel B: 8 workgroups that sleep ~50 us. Serialized: ~100 us
// between the events; overlapped: ~50 us. (diagnostic)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>

__global__ void sleeper(int iters, unsigned long long *t) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) __builtin_amdgcn_s_sleep(127);
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main() {
    unsigned long long *ta, *tb;
    hipMalloc(&ta, 1024);
    hipMalloc(&tb, 1024);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 400;
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0, s);
            hipLaunchKernelGGL(sleeper, dim3(8), dim3(64), 0, s, iters, ta);
            if (mode == 0) hipLaunchKernelGGL(sleeper, dim3(8), dim3(64), 0, s, iters, tb);
            else {
                void *args[] = { (void *)&iters, (void *)&tb };
                hipExtLaunchKernel((const void *)sleeper, dim3(8), dim3(64), args, 0, s, nullptr, nullptr,
                                   mode == 1 ? hipExtAnyOrderLaunch : 0);
            }
            hipEventRecord(e1, s);
            hipStreamSynchronize(s);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long ha[2], hb[2];
            hipMemcpy(ha, ta, 16, hipMemcpyDeviceToHost);
            hipMemcpy(hb, tb, 16, hipMemcpyDeviceToHost);
            printf("mode %d (%s): %.1f us; A %llu-%llu B %llu-%llu (10 ns ticks, B start - A end = %lld)\n", mode,
                   mode == 0 ? "plain" : mode == 1 ? "ext any-order" : "ext ordered", ms * 1e3, 0ULL, ha[1] - ha[0],
                   (long long)(hb[0] - ha[0]), (long long)(hb[1] - ha[0]), (long long)hb[0] - (long long)ha[1]);
        }
    }
    return 0;
}
