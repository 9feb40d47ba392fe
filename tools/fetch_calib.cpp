// fetch_calib — what gfx950's FETCH_SIZE / WRITE_SIZE counters report for
// known byte counts in the access shapes the step kernels use (analysis
// tool; run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`, one
// pass each, and compare each kernel's counter with the bytes printed here).
//
//   k_read16  : 16 B per lane, coalesced (float4 streams: k_obs rows, lidar)
//   k_read4   : 4 B per lane, coalesced (SoA columns: k_sim, k_move)
//   k_gather4 : 4 B per lane at a random 128-B line (scattered state)
//   k_write4  : 4 B per lane, coalesced stores
//
// hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.cpp -o fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void k_read16(const float4 *__restrict__ src, float *out, int64_t n)
{
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) out[0] = acc; // keeps the loads
}

__global__ void k_read4(const float *__restrict__ src, float *out, int64_t n)
{
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc += src[i];
    if (acc == 12345.f) out[0] = acc;
}

__global__ void k_gather4(const float *__restrict__ src, float *out, int64_t n, int64_t lines)
{
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        // a multiplicative hash of i picks the line: distinct lines, no reuse
        const uint64_t l = ((uint64_t)i * 0x9E3779B97F4A7C15ull >> 20) % (uint64_t)lines;
        acc += src[l * 32];
    }
    if (acc == 12345.f) out[0] = acc;
}

__global__ void k_write4(float *__restrict__ dst, int64_t n)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = (float)i;
}

int main()
{
    const int64_t bytes = 1ll << 30; // 1 GiB
    float *a = nullptr, *out = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(a, 0, bytes) != hipSuccess) return 1;
    const dim3 grid(8192), block(256);
    const int64_t n4 = bytes / 4, n16 = bytes / 16, lines = bytes / 128;
    const int64_t gathers = lines / 4; // a quarter of the lines, one 4-B read each
    hipLaunchKernelGGL(k_read16, grid, block, 0, 0, reinterpret_cast<const float4 *>(a), out, n16);
    hipLaunchKernelGGL(k_read4, grid, block, 0, 0, a, out, n4);
    hipLaunchKernelGGL(k_gather4, grid, block, 0, 0, a, out, gathers, lines);
    hipLaunchKernelGGL(k_write4, grid, block, 0, 0, a, n4);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("k_read16 bytes %lld\nk_read4 bytes %lld\nk_gather4 reads %lld x 4 B from distinct 128-B lines (%lld line bytes)\n"
           "k_write4 bytes %lld\n", (long long)bytes, (long long)bytes, (long long)gathers, (long long)(gathers * 128),
           (long long)bytes);
    hipFree(a);
    hipFree(out);
    return 0;
}
