// calib_fetch.hip -- FETCH_SIZE calibration for the access patterns of the alignment kernels
// (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16-B/lane streaming reads; calibrate
// other widths on a known byte count).  Each kernel reads exactly 1 GiB:
//   k_stream   : coalesced 16 B per lane (the guide's reference pattern)
//   k_gather64 : one random 64-B block per lane, 4 x 16-B loads (the occ-block rank query)
//   k_gather16 : one random 16-B entry per lane (the k-mer interval table)
// over a 4 GiB table (beyond the 256 MiB Infinity Cache) and, for the gathers, over a 96 MiB table
// (resident, like the 100 Mbp occ array).  Run under: rocprofv3 --pmc FETCH_SIZE --kernel-trace.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

static __device__ __forceinline__ uint64_t mix(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

__global__ void k_stream(const uint4 *t, uint64_t n16, uint32_t *sink)
{
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = t[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_gather64(const uint4 *t, uint64_t nblocks, uint64_t nlanes, uint32_t *sink)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlanes) return;
    const uint4 *p = t + (mix(i) % nblocks) * 4;
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    const uint32_t acc = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ d.x;
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_gather16(const uint4 *t, uint64_t nent, uint64_t nlanes, uint32_t *sink)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlanes) return;
    const uint4 a = t[mix(i) % nent];
    const uint32_t acc = a.x ^ a.y ^ a.z ^ a.w;
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_copy(const uint4 *a, uint4 *b, uint64_t n16)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

// STREAM-like ceilings: 2 GiB read-only stream and a 2 GiB -> 2 GiB copy, best of 5
static void ceilings(uint4 *t, uint32_t *sink)
{
    const uint64_t bytes = 2ull << 30, n16 = bytes / 16;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float best_r = 1e30f, best_c = 1e30f;
    for (int it = 0; it < 5; ++it) {
        float ms = 0;
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, t, n16, sink);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
        best_r = ms < best_r ? ms : best_r;
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, t, t + n16, n16);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
        best_c = ms < best_c ? ms : best_c;
    }
    printf("ceiling: stream-read %.0f GB/s, copy %.0f GB/s (read+write bytes), 2 GiB each\n",
           bytes / (best_r * 1e-3) / 1e9, 2.0 * bytes / (best_c * 1e-3) / 1e9);
}

int main()
{
    const uint64_t big = 4ull << 30, small = 96ull << 20, bytes = 1ull << 30;
    uint4 *t = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc(&t, big) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(t, 0x5a, big);
    hipDeviceSynchronize();
    const uint64_t n64 = bytes / 64, n16 = bytes / 16;
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, t, n16, sink);
    hipLaunchKernelGGL(k_gather64, dim3((unsigned)(n64 / 256)), dim3(256), 0, 0, t, big / 64, n64, sink);
    hipLaunchKernelGGL(k_gather16, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, t, big / 16, n16, sink);
    // resident table: warm it, then measure
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, t, small / 16, sink);
    hipLaunchKernelGGL(k_gather64, dim3((unsigned)(n64 / 256)), dim3(256), 0, 0, t, small / 64, n64, sink);
    hipLaunchKernelGGL(k_gather16, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, t, small / 16, n16, sink);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    ceilings(t, sink);
    printf("dispatch order: stream(4G) gather64(4G) gather16(4G) stream(96M warm) gather64(96M) gather16(96M); "
           "each reads %llu bytes except the warm stream (%llu)\n", (unsigned long long)bytes, (unsigned long long)small);
    return 0;
}
