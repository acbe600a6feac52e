// PMC calibration for FETCH_SIZE / WRITE_SIZE on gfx950 (MI355X_MICROARCH.md "HBM": only the
// 16-B-per-lane streaming read and write are calibrated there; "calibrate on a known byte count
// in your own access pattern"). Streams a 1 GiB buffer (past the 256 MiB Infinity Cache) with
// coalesced per-lane widths of 2, 4, 8 and 16 B, reading (rd_wN) or writing (wr_wN), so
// `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` of this binary gives counter / true bytes
// per width. Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T>
__global__ void rd(const T *__restrict__ src, size_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v = src[i];
        const uint32_t *p = reinterpret_cast<const uint32_t *>(&v);
        if constexpr (sizeof(T) >= 4) {
#pragma unroll
            for (int k = 0; k < (int)(sizeof(T) / 4); k++) acc = acc * 31u + p[k];
        } else {
            acc = acc * 31u + (uint32_t)v;     // not a plain xor: keeps the test below reachable
        }
    }
    if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;  // never true for the zero-filled input
}

template <typename T>
__global__ void wr(T *__restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v;
        uint8_t *b = reinterpret_cast<uint8_t *>(&v);
        for (int k = 0; k < (int)sizeof(T); k++) b[k] = (uint8_t)(i + k);
        dst[i] = v;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t bytes = size_t(1) << 30;
    void *buf; uint32_t *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(buf, 0, bytes));
    const int grid = 256 * 16, block = 256;
    hipLaunchKernelGGL(rd<uint16_t>, grid, block, 0, 0, (const uint16_t *)buf, bytes / 2, sink);
    hipLaunchKernelGGL(rd<uint32_t>, grid, block, 0, 0, (const uint32_t *)buf, bytes / 4, sink);
    hipLaunchKernelGGL(rd<uint2>, grid, block, 0, 0, (const uint2 *)buf, bytes / 8, sink);
    hipLaunchKernelGGL(rd<uint4>, grid, block, 0, 0, (const uint4 *)buf, bytes / 16, sink);
    hipLaunchKernelGGL(wr<uint16_t>, grid, block, 0, 0, (uint16_t *)buf, bytes / 2);
    hipLaunchKernelGGL(wr<uint32_t>, grid, block, 0, 0, (uint32_t *)buf, bytes / 4);
    hipLaunchKernelGGL(wr<uint2>, grid, block, 0, 0, (uint2 *)buf, bytes / 8);
    hipLaunchKernelGGL(wr<uint4>, grid, block, 0, 0, (uint4 *)buf, bytes / 16);
    CK(hipDeviceSynchronize());
    printf("pmc_calib: 8 kernels, %zu bytes each (rd/wr x 2,4,8,16 B per lane)\n", bytes);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
