// scc_group.hip — device side of the group-pair runs (more consensus clusters
// than one engine run holds, scc_runtime.cpp de_run_grouped).
//
// One engine run ranks <= 128 clusters (7-bit cluster codes in the rank
// kernels).  Every per-pair quantity of both DE paths is a function of the
// pair's two clusters alone (Fast:229-351 per ComputePairWiseDE call;
// slow:90-187 per (i, j)), so K > 128 clusters are cut into groups of <= 64
// and one run per group pair assembles the pairs; these kernels move a run's
// per-pair rows / vectors into the global (i, j) order (segment copies) and
// fold its first-occurrence keys (the union order, Fast:386-392 / slow:209-227)
// into the global key array.
#include "scc_common.hpp"

#include <algorithm>

// segments: [n][3] = {source offset, destination offset, length} in elements;
// one workgroup per segment (grid-stride), lanes over its elements
template <class T>
__global__ void __launch_bounds__(256) k_seg_copy(const T* __restrict__ src, T* __restrict__ dst,
                                                  const long long* __restrict__ seg, long long nseg)
{
    for (long long s = blockIdx.x; s < nseg; s += gridDim.x) {
        const long long so = seg[3 * s], d0 = seg[3 * s + 1], n = seg[3 * s + 2];
        for (long long i = threadIdx.x; i < n; i += 256) dst[d0 + i] = src[so + i];
    }
}

// a run's per-gene first-occurrence keys (local pair << 32 | rank in the
// pair, ~0 = not selected) -> global pair numbering, MIN into the global keys.
// The local -> global pair map is increasing (a run's clusters keep the global
// order), so the run's minimum maps to the minimum over its global pairs.
__global__ void __launch_bounds__(256) k_first_remap(const u64* __restrict__ local, int G,
                                                     const long long* __restrict__ lp2gp, u64* __restrict__ global)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= G) return;
    const u64 k = local[g];
    if (k == ~0ull) return;
    const u64 gk = ((u64)lp2gp[k >> 32] << 32) | (k & 0xFFFFFFFFull);
    if (gk < global[g]) atomicMin((unsigned long long*)&global[g], (unsigned long long)gk);
}

// stored values per gene row of a CSC (the device list's gene-block weights)
__global__ void __launch_bounds__(256) k_row_hist(const int* __restrict__ rows, long long nnz, int G,
                                                  unsigned int* __restrict__ cnt)
{
    for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < nnz; k += (long long)gridDim.x * 256) {
        const int r = rows[k];
        if (r >= 0 && r < G) atomicAdd(&cnt[r], 1u);
    }
}

extern "C" hipError_t scc_launch_row_hist(const int* rows, long long nnz, int G, unsigned int* cnt, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(cnt, 0, sizeof(unsigned int) * (size_t)G, st);
    if (e != hipSuccess || nnz <= 0) return e;
    const unsigned grid = (unsigned)std::min<long long>((nnz + 255) / 256, 4096);
    hipLaunchKernelGGL(k_row_hist, dim3(grid), dim3(256), 0, st, rows, nnz, G, cnt);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_seg_copy(const void* src, void* dst, int elem_bytes, const long long* seg,
                                          long long nseg, hipStream_t st)
{
    if (nseg <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<long long>(nseg, 8192);
    switch (elem_bytes) {
        case 8:
            hipLaunchKernelGGL(k_seg_copy<u64>, dim3(grid), dim3(256), 0, st, (const u64*)src, (u64*)dst, seg, nseg);
            break;
        case 4:
            hipLaunchKernelGGL(k_seg_copy<u32>, dim3(grid), dim3(256), 0, st, (const u32*)src, (u32*)dst, seg, nseg);
            break;
        case 1:
            hipLaunchKernelGGL(k_seg_copy<uint8_t>, dim3(grid), dim3(256), 0, st, (const uint8_t*)src, (uint8_t*)dst,
                               seg, nseg);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_first_remap(const unsigned long long* local, int G, const long long* lp2gp,
                                             unsigned long long* global, hipStream_t st)
{
    hipLaunchKernelGGL(k_first_remap, dim3((G + 255) / 256), dim3(256), 0, st, (const u64*)local, G, lp2gp,
                       (u64*)global);
    return hipGetLastError();
}
