// gather_ceiling.hip -- the achievable rate of the seeding kernel's memory access pattern on this GPU.
//
// k_smem_lds spends its time on random 32-B rank-block loads (two 16-B loads each, k and l ends of an interval,
// DESIGN.md section 3) from a table that is Infinity-Cache resident at 100 Mbp (C2/C3: 100 MB of blocks) and far
// beyond every cache at 3 Gbp (C4: 3 GB).  This program measures, for a 100 MB and a 3 GB table:
//   * indep: every lane issues 8 independent random 32-B block loads per trip (all in flight): the gather throughput
//     ceiling of the memory system for this access size (blocks/s);
//   * chain: every lane follows a dependent chain of random 32-B block loads (the next address from the loaded
//     block), 16 one-wave blocks per CU: the latency-bound rate of a kernel shaped like the seeding kernel (one
//     dependent query per lane, two per paired step).
// Usage: gather_ceiling  -> one line per case: blocks/s, GB/s of 32-B blocks, ns per dependent load.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                                  \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

__device__ inline uint64_t mix(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

// 8 independent random 32-B blocks per lane per trip
__global__ void __launch_bounds__(256) k_indep(const uint4 *t, uint64_t nblk, int trips, uint32_t *sink)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    uint64_t s = mix(g + 1);
    for (int r = 0; r < trips; ++r) {
        uint4 a[8], b[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s = mix(s + k);
            const uint4 *p = t + 2 * (s % nblk);
            a[k] = p[0]; b[k] = p[1];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= a[k].x ^ b[k].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// one dependent chain of random 32-B blocks per lane (the next index from the loaded block)
__global__ void __launch_bounds__(64) k_chain(const uint4 *t, uint64_t nblk, int steps, uint32_t *sink)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t i = mix(g + 7) % nblk;
    uint32_t acc = 0;
    for (int r = 0; r < steps; ++r) {
        const uint4 *p = t + 2 * i;
        const uint4 x = p[0], y = p[1];
        acc ^= y.w;
        i = mix(((uint64_t)x.y << 32 | x.x) + r) % nblk;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// P dependent chains per lane, advanced together (P blocks in flight per lane, like the paired backward extensions)
template <int P>
__global__ void __launch_bounds__(64) k_chains(const uint4 *t, uint64_t nblk, int steps, uint32_t *sink)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t i[P];
#pragma unroll
    for (int k = 0; k < P; ++k) i[k] = mix(g * P + k + 7) % nblk;
    uint32_t acc = 0;
    for (int r = 0; r < steps; ++r) {
        uint4 x[P], y[P];
#pragma unroll
        for (int k = 0; k < P; ++k) { x[k] = t[2 * i[k]]; y[k] = t[2 * i[k] + 1]; }
#pragma unroll
        for (int k = 0; k < P; ++k) {
            acc ^= y[k].w;
            i[k] = mix(((uint64_t)x[k].y << 32 | x[k].x) + r) % nblk;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// MODE 1: one 16-B load per step (a 16-B block); MODE 2: 32-B blocks, but lanes 2j and 2j+1 load the two halves of
// the same block (two loads per lane per two chains, each instruction coalescing lane pairs onto one 32-B block) and
// swap them with a DPP quad permute
template <int P, int MODE>
__global__ void __launch_bounds__(64) k_chainsm(const uint4 *t, uint64_t nblk, int steps, uint32_t *sink)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int odd = threadIdx.x & 1;
    uint64_t i[P];
#pragma unroll
    for (int k = 0; k < P; ++k) i[k] = mix(g * P + k + 7) % nblk;
    uint32_t acc = 0;
    for (int r = 0; r < steps; ++r) {
        uint4 x[P], y[P];
        if constexpr (MODE == 1) {
#pragma unroll
            for (int k = 0; k < P; ++k) { x[k] = t[i[k]]; y[k] = x[k]; }
        } else {
#pragma unroll
            for (int k = 0; k < P; ++k) {
                // instruction A: both lanes of a pair read the even lane's block (even: half 0, odd: half 1);
                // instruction B: both read the odd lane's block; then each lane takes its missing half from the other
                const uint64_t pi = (uint64_t)__shfl_xor((long long)i[k], 1);
                const uint4 a = t[2 * (odd ? pi : i[k]) + odd];
                const uint4 b = t[2 * (odd ? i[k] : pi) + odd];
                uint4 sw;
                const uint4 give = odd ? a : b;
                sw.x = __shfl_xor((int)give.x, 1); sw.y = __shfl_xor((int)give.y, 1);
                sw.z = __shfl_xor((int)give.z, 1); sw.w = __shfl_xor((int)give.w, 1);
                x[k] = odd ? sw : a;   // h0
                y[k] = odd ? b : sw;   // h1
            }
        }
#pragma unroll
        for (int k = 0; k < P; ++k) {
            acc ^= y[k].w;
            i[k] = mix(((uint64_t)x[k].y << 32 | x[k].x) + r) % (MODE == 1 ? 2 * nblk : nblk);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int P, int MODE>
static void sweep_m(const uint4 *t, uint64_t nblk, uint64_t bytes, int cus, uint32_t *sink, hipEvent_t a, hipEvent_t b)
{
    for (int wpc : {4, 8, 12, 16}) {
        const int grid = cus * wpc, steps = 4096 / P;
        float ms = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            float m = 0;
            CHK(hipEventRecord(a));
            hipLaunchKernelGGL((k_chainsm<P, MODE>), dim3(grid), dim3(64), 0, 0, t, nblk, steps, sink);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            CHK(hipEventElapsedTime(&m, a, b));
            ms = m < ms ? m : ms;
        }
        const double loads = (double)grid * 64 * steps * P;
        printf("table %6.0f MB  %s %d chains/lane %2d waves/CU: %6.2f G blocks/s  %.0f ns per step\n", bytes / 1048576.0,
               MODE == 1 ? "16-B blocks      " : "32-B lane-paired ", P, wpc, loads / (ms * 1e-3) / 1e9, ms * 1e6 / steps);
    }
}

template <int P>
static void sweep_chains(const uint4 *t, uint64_t nblk, uint64_t bytes, int cus, uint32_t *sink, hipEvent_t a, hipEvent_t b)
{
    for (int wpc : {1, 2, 4, 6, 8, 10, 12, 14, 16}) {
        const int grid = cus * wpc, steps = 4096 / P;
        float ms = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            float m = 0;
            CHK(hipEventRecord(a));
            hipLaunchKernelGGL(k_chains<P>, dim3(grid), dim3(64), 0, 0, t, nblk, steps, sink);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            CHK(hipEventElapsedTime(&m, a, b));
            ms = m < ms ? m : ms;
        }
        const double loads = (double)grid * 64 * steps * P;
        printf("table %6.0f MB  %d chains/lane %2d waves/CU (%5d blocks in flight/CU): %6.2f G blocks/s  %.0f ns per step\n",
               bytes / 1048576.0, P, wpc, wpc * 64 * P, loads / (ms * 1e-3) / 1e9, ms * 1e6 / steps);
    }
}

__global__ void k_fill(uint4 *t, uint64_t n16)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        t[i] = make_uint4((uint32_t)mix(i), (uint32_t)(mix(i) >> 32), (uint32_t)i, 0u);
}

int main(int argc, char **argv)
{
    (void)argc; (void)argv;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t *sink;
    CHK(hipMalloc(&sink, 4));
    // GATHER_SWEEP=1: table sizes from 1 MB (L2) to 3 GB, independent gathers and 12 / 16-wave chains only
    const bool sweep = getenv("GATHER_SWEEP") != nullptr;
    const uint64_t sizes_all[2] = {100ull << 20, 3ull << 30};
    const uint64_t sizes_sw[7] = {1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20, 100ull << 20, 256ull << 20, 1ull << 30};
    const int nsz = sweep ? 7 : 2;
    for (int zi = 0; zi < nsz; ++zi) {
        const uint64_t bytes = sweep ? sizes_sw[zi] : sizes_all[zi];
        uint4 *t;
        CHK(hipMalloc(&t, bytes));
        const uint64_t n16 = bytes / 16, nblk = bytes / 32;
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, t, n16);
        CHK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CHK(hipEventCreate(&a));
        CHK(hipEventCreate(&b));
        float ms = 0;
        // independent gathers: 16 waves per CU of 256-thread blocks, 256 trips x 8 blocks per lane; best of 5
        for (int wpc : {4, 8, 16}) {
            const int grid = cus * wpc / 4, trips = sweep ? 64 : 256;
            ms = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                float m = 0;
                CHK(hipEventRecord(a));
                hipLaunchKernelGGL(k_indep, dim3(grid), dim3(256), 0, 0, t, nblk, trips, sink);
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                CHK(hipEventElapsedTime(&m, a, b));
                ms = m < ms ? m : ms;
            }
            const double blocks = (double)grid * 256 * trips * 8;
            printf("table %6.0f MB  indep (%2d waves/CU): %.2f G blocks/s  %.0f GB/s of 32-B blocks\n", bytes / 1048576.0, wpc,
                   blocks / (ms * 1e-3) / 1e9, blocks * 32 / (ms * 1e-3) / 1e9);
        }
        // dependent chains: 4..16 one-wave blocks per CU; best of 5
        for (int wpc : {4, 8, 12, 16}) {
            const int grid = cus * wpc, steps = 2048;
            ms = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                float m = 0;
                CHK(hipEventRecord(a));
                hipLaunchKernelGGL(k_chain, dim3(grid), dim3(64), 0, 0, t, nblk, steps, sink);
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                CHK(hipEventElapsedTime(&m, a, b));
                ms = m < ms ? m : ms;
            }
            const double loads = (double)grid * 64 * steps;
            printf("table %6.0f MB  chain (%2d waves/CU): %.2f G blocks/s  %.0f GB/s  %.0f ns per dependent load\n",
                   bytes / 1048576.0, wpc, loads / (ms * 1e-3) / 1e9, loads * 32 / (ms * 1e-3) / 1e9,
                   ms * 1e6 / steps);
        }
        if (sweep) { CHK(hipFree(t)); continue; }
        sweep_chains<1>(t, nblk, bytes, cus, sink, a, b);
        sweep_chains<2>(t, nblk, bytes, cus, sink, a, b);
        sweep_chains<4>(t, nblk, bytes, cus, sink, a, b);
        sweep_m<1, 1>(t, nblk, bytes, cus, sink, a, b);
        sweep_m<2, 1>(t, nblk, bytes, cus, sink, a, b);
        sweep_m<1, 2>(t, nblk, bytes, cus, sink, a, b);
        sweep_m<2, 2>(t, nblk, bytes, cus, sink, a, b);
        CHK(hipFree(t));
    }
    return 0;
}
