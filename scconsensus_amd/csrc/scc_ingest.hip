// scc_ingest.hip — boundary ingest: the R dgCMatrix (CSC over cells) or dense
// column-major matrix plus per-cell cluster codes become a gene-major array of
// (orderable 64-bit value key, cluster code) for the kept nonzeros, resident
// in HBM.  Replaces the reference's per-pair `as.matrix(dataMatrix)` and
// name-indexed column subsets (R/reclusterDEConsensusFast.R:361-368).
//
// A block-local counting sort (no global atomics):
//   k_ing_hist     one workgroup per chunk of cells: LDS histogram over genes
//                  (kept nonzeros), nodg per cell (Fast:440-443, x > 0 over ALL
//                  cells), optional sum of expm1 over all entries (slow:36),
//                  non-finite / bad-row flag; histogram row -> cnt[w][g]
//   k_ing_colscan  per gene: exclusive prefix over chunks (in place), total[g]
//   scan           gene starts gstart[G+1] (three-kernel device scan)
//   k_ing_scatter  per chunk: LDS cursors = gstart[g] + cnt[w][g]; write keys
//                  and codes.
// Zeros are implicit (the tie group every Wilcoxon statistic handles in
// closed form).  Within a gene the order is chunk-major (cell order across
// chunks); the rank kernel sorts each gene anyway.
#include "scc_common.hpp"
#include "scc_kernels.hpp"

#define ING_T 256

template <bool DENSE>
__device__ inline void cell_range(const i64* indptr, int c, int G, i64& b, i64& e)
{
    if (DENSE) {
        b = (i64)c * G;
        e = b + G;
    } else {
        b = indptr[c];
        e = indptr[c + 1];
    }
}

template <bool DENSE>
__global__ void __launch_bounds__(ING_T) k_ing_hist(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                    const double* __restrict__ vals, int N, int G, int cells_per_wg,
                                                    const int* __restrict__ code, u32* __restrict__ cnt,
                                                    int* __restrict__ nodg, dd* __restrict__ wave_expm1,
                                                    int want_expm1, int* __restrict__ err)
{
    extern __shared__ __attribute__((aligned(16))) u32 hist[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int g = threadIdx.x; g < G; g += ING_T) hist[g] = 0;
    __syncthreads();
    const int c0 = blockIdx.x * cells_per_wg, c1 = min(N, c0 + cells_per_wg);
    dd se{0.0, 0.0};
    int bad = 0;
    for (int c = c0 + wv; c < c1; c += ING_T / 64) {
        i64 b, e;
        cell_range<DENSE>(indptr, c, G, b, e);
        const int a = code[c];
        u32 pos = 0;
        for (i64 k = b + lane; k < e; k += 64) {
            const double x = vals[k];
            const int g = DENSE ? (int)(k - b) : rows[k];
            const bool gok = (g >= 0) & (g < G);
            bad |= !(x - x == 0.0) | !gok;
            pos += (x > 0.0);
            if (want_expm1) se = dd_add_d(se, expm1(x));
            if (a >= 0 && x != 0.0 && gok) atomicAdd(&hist[g], 1u);
        }
        pos = u32_wave_sum(pos);
        if (lane == 0) nodg[c] = (int)pos;
    }
    if (want_expm1) {
        se = dd_wave_sum(se);
        if (lane == 0) wave_expm1[blockIdx.x * (ING_T / 64) + wv] = se;
    }
    if (bad) atomicOr(err, 1);
    __syncthreads();
    u32* row = cnt + (size_t)blockIdx.x * G;
    for (int g = threadIdx.x; g < G; g += ING_T) row[g] = hist[g];
}

__global__ void __launch_bounds__(256) k_ing_colscan(u32* __restrict__ cnt, int nwg, int G, u32* __restrict__ total)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= G) return;
    u32 run = 0;
    for (int w = 0; w < nwg; ++w) {
        const u32 v = cnt[(size_t)w * G + g];
        cnt[(size_t)w * G + g] = run;
        run += v;
    }
    total[g] = run;
}

template <bool DENSE>
__global__ void __launch_bounds__(ING_T) k_ing_scatter(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                       const double* __restrict__ vals, int N, int G,
                                                       int cells_per_wg, const int* __restrict__ code,
                                                       const u32* __restrict__ cnt, const i64* __restrict__ gstart,
                                                       u64* __restrict__ keys, u8* __restrict__ codes)
{
    extern __shared__ __attribute__((aligned(16))) u32 cur[];  // offset inside the gene
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const u32* row = cnt + (size_t)blockIdx.x * G;
    for (int g = threadIdx.x; g < G; g += ING_T) cur[g] = row[g];
    __syncthreads();
    const int c0 = blockIdx.x * cells_per_wg, c1 = min(N, c0 + cells_per_wg);
    for (int c = c0 + wv; c < c1; c += ING_T / 64) {
        const int a = code[c];
        if (a < 0) continue;
        i64 b, e;
        cell_range<DENSE>(indptr, c, G, b, e);
        for (i64 k = b + lane; k < e; k += 64) {
            const double x = vals[k];
            const int g = DENSE ? (int)(k - b) : rows[k];
            if (x != 0.0 && g >= 0 && g < G) {
                const u64 pos = (u64)gstart[g] + atomicAdd(&cur[g], 1u);
                keys[pos] = scc_key_of(x);
                codes[pos] = (u8)a;
            }
        }
    }
}

// ------------------------------------------------------------ exclusive scan
// Three-kernel device-wide exclusive scan of u32 counts into i64 offsets.
#define SCAN_T 256
#define SCAN_PER 8
__global__ void __launch_bounds__(SCAN_T) k_scan_block_sums(const u32* __restrict__ in, i64 n, i64* __restrict__ bsum)
{
    __shared__ i64 s[SCAN_T];
    const i64 base = (i64)blockIdx.x * SCAN_T * SCAN_PER;
    i64 acc = 0;
    for (int k = 0; k < SCAN_PER; ++k) {
        i64 i = base + (i64)k * SCAN_T + threadIdx.x;
        if (i < n) acc += in[i];
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int st = SCAN_T / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) s[threadIdx.x] += s[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = s[0];
}

// single block: exclusive scan of nb block sums (nb <= a few thousand)
__global__ void __launch_bounds__(1024) k_scan_top(i64* __restrict__ bsum, int nb, i64* __restrict__ total)
{
    __shared__ i64 s[1024];
    i64 carry = 0;
    for (int base = 0; base < nb; base += 1024) {
        int i = base + threadIdx.x;
        i64 v = (i < nb) ? bsum[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            i64 t = ((int)threadIdx.x >= off) ? s[threadIdx.x - off] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < nb) bsum[i] = carry + s[threadIdx.x] - v;
        i64 blk = s[1023];
        __syncthreads();
        carry += blk;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ void __launch_bounds__(SCAN_T) k_scan_apply(const u32* __restrict__ in, i64 n, const i64* __restrict__ bsum,
                                                       i64* __restrict__ out)
{
    __shared__ i64 s[SCAN_T * SCAN_PER];
    __shared__ i64 t[SCAN_T];
    const i64 base = (i64)blockIdx.x * SCAN_T * SCAN_PER;
    for (int k = 0; k < SCAN_PER; ++k) {
        int li = k * SCAN_T + threadIdx.x;
        i64 i = base + li;
        s[li] = (i < n) ? (i64)in[i] : 0;
    }
    __syncthreads();
    i64 acc = 0;
    for (int k = 0; k < SCAN_PER; ++k) acc += s[threadIdx.x * SCAN_PER + k];
    t[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 1; off < SCAN_T; off <<= 1) {
        i64 v = ((int)threadIdx.x >= off) ? t[threadIdx.x - off] : 0;
        __syncthreads();
        t[threadIdx.x] += v;
        __syncthreads();
    }
    i64 run = bsum[blockIdx.x] + t[threadIdx.x] - acc;
    for (int k = 0; k < SCAN_PER; ++k) {
        i64 i = base + threadIdx.x * SCAN_PER + k;
        i64 v = s[threadIdx.x * SCAN_PER + k];
        if (i < n) out[i] = run;
        run += v;
    }
}

__global__ void k_reduce_dd(const dd* __restrict__ parts, int n, dd* __restrict__ out)
{
    // one wave, fixed order -> deterministic
    dd s{0.0, 0.0};
    for (int i = threadIdx.x; i < n; i += 64) s = dd_add(s, parts[i]);
    s = dd_wave_sum(s);
    if (threadIdx.x == 0) *out = s;
}

// ------------------------------------------------------------ host launchers
extern "C" int scc_ingest_chunks(int N, int* cells_per_wg)
{
    int nwg = N / 16;
    if (nwg > 1024) nwg = 1024;
    if (nwg < 1) nwg = 1;
    *cells_per_wg = (N + nwg - 1) / nwg;
    return (N + *cells_per_wg - 1) / *cells_per_wg;
}

extern "C" hipError_t scc_launch_ingest_hist(const i64* indptr, const int* rows, const double* vals,
                                             const double* dense, int N, int G, int nwg, int cells_per_wg,
                                             const int* code, u32* cnt, int* nodg, dd* wave_expm1, int want_expm1,
                                             int* err, hipStream_t st)
{
    const size_t lds = sizeof(u32) * (size_t)G;
    if (dense) {
        hipFuncSetAttribute((const void*)k_ing_hist<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_ing_hist<true>, dim3(nwg), dim3(ING_T), lds, st, nullptr, nullptr, dense, N, G,
                           cells_per_wg, code, cnt, nodg, wave_expm1, want_expm1, err);
    } else {
        hipFuncSetAttribute((const void*)k_ing_hist<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_ing_hist<false>, dim3(nwg), dim3(ING_T), lds, st, indptr, rows, vals, N, G, cells_per_wg,
                           code, cnt, nodg, wave_expm1, want_expm1, err);
    }
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_ingest_colscan(u32* cnt, int nwg, int G, u32* total, hipStream_t st)
{
    hipLaunchKernelGGL(k_ing_colscan, dim3((G + 255) / 256), dim3(256), 0, st, cnt, nwg, G, total);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_ingest_scatter(const i64* indptr, const int* rows, const double* vals,
                                                const double* dense, int N, int G, int nwg, int cells_per_wg,
                                                const int* code, const u32* cnt, const i64* gstart, u64* keys,
                                                u8* codes, hipStream_t st)
{
    const size_t lds = sizeof(u32) * (size_t)G;
    if (dense) {
        hipFuncSetAttribute((const void*)k_ing_scatter<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_ing_scatter<true>, dim3(nwg), dim3(ING_T), lds, st, nullptr, nullptr, dense, N, G,
                           cells_per_wg, code, cnt, gstart, keys, codes);
    } else {
        hipFuncSetAttribute((const void*)k_ing_scatter<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_ing_scatter<false>, dim3(nwg), dim3(ING_T), lds, st, indptr, rows, vals, N, G,
                           cells_per_wg, code, cnt, gstart, keys, codes);
    }
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_scan(const u32* in, i64 n, i64* out, i64* bsum_scratch, i64* total, hipStream_t st)
{
    const i64 per = (i64)SCAN_T * SCAN_PER;
    int nb = (int)((n + per - 1) / per);
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(k_scan_block_sums, dim3(nb), dim3(SCAN_T), 0, st, in, n, bsum_scratch);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, st, bsum_scratch, nb, total);
    hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(SCAN_T), 0, st, in, n, bsum_scratch, out);
    return hipGetLastError();
}

extern "C" int scc_scan_scratch_blocks(i64 n)
{
    const i64 per = (i64)SCAN_T * SCAN_PER;
    i64 nb = (n + per - 1) / per;
    return (int)(nb < 1 ? 1 : nb);
}

extern "C" hipError_t scc_launch_reduce_dd(const dd* parts, int n, dd* out, hipStream_t st)
{
    hipLaunchKernelGGL(k_reduce_dd, dim3(1), dim3(64), 0, st, parts, n, out);
    return hipGetLastError();
}
