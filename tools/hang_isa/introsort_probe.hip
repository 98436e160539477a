// ISA probe of klib's partition scan over a lane-interleaved index array (DESIGN.md section 3, round-2 hang).
// Compiled (never run) by tools/hang_isa/hang_isa.sh with and without BSQ_INTROSORT_UNBOUNDED: one kernel sorts
// each lane's region ids by `re` exactly as sort_dedup_patch does, over SP<int, 64> scratch (S = 64) and over
// contiguous per-thread scratch (S = 1), so the scan loops can be read without the 8,000 lines of k_extend.
#include "../../bioseqdb_amd/csrc/align_kernels.hip"

namespace bsq {
template <int S>
__global__ void __launch_bounds__(64) k_introsort_probe(const Reg *regs, const int *n_regs, int cap, uint8_t *scratch,
                                                         int *out)
{
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = S == 1 ? 0 : (tid & 63);
    uint8_t *wb = scratch + (S == 1 ? (size_t)tid : (size_t)(tid >> 6) * 64) * (size_t)(cap * 4 + 192 * 4);
    SP<int, S> idx{reinterpret_cast<int *>(wb) + lane};
    SP<int, S> stk{reinterpret_cast<int *>(wb + (size_t)cap * 4 * S) + lane};
    const int n = n_regs[tid];
    const Reg *a = regs + (size_t)tid * cap;
    for (int i = 0; i < n; ++i) idx[i] = i;
    ks_introsort(idx, n, [a](int x, int y) { return a[x].re < a[y].re; }, stk);
    for (int i = 0; i < n; ++i) out[(size_t)tid * cap + i] = idx[i];
}
template __global__ void k_introsort_probe<64>(const Reg *, const int *, int, uint8_t *, int *);
template __global__ void k_introsort_probe<1>(const Reg *, const int *, int, uint8_t *, int *);
}  // namespace bsq
