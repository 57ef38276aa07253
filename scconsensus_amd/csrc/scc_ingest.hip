// scc_ingest.hip — boundary ingest: the R dgCMatrix (CSC over cells) or dense
// column-major matrix, plus per-cell cluster codes, becomes a per-(gene,
// cluster) bucketed array of orderable 64-bit keys resident in HBM.
//
// Replaces the reference's per-pair `as.matrix(dataMatrix)` + name-indexed
// column subsets (R/reclusterDEConsensusFast.R:361-368) with one streaming pass.
// Layout out:  seg_off[g*K + a] .. seg_off[g*K + a + 1]  = keys of gene g,
// cluster a (value != 0, cell kept).  Zeros are implicit (the tie group every
// Wilcoxon statistic treats in closed form).
#include "scc_common.hpp"
#include "scc_kernels.hpp"

// One wave per cell: lanes stride the cell's stored entries (coalesced).
// Counts kept nonzeros per (gene, cluster), negatives per (gene, cluster),
// nodg per cell (Fast:440-443, x > 0 over ALL cells), non-finite flag, and
// optionally the global sum of expm1 over all entries (slow:36).
__global__ void __launch_bounds__(256) k_ingest_count(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                      const double* __restrict__ vals, int N, int G, int K,
                                                      const int* __restrict__ code, u32* __restrict__ cnt,
                                                      u32* __restrict__ neg, int* __restrict__ nodg,
                                                      dd* __restrict__ wave_expm1, int want_expm1,
                                                      int* __restrict__ err)
{
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    const int wid = blockIdx.x * wpb + (threadIdx.x >> 6);
    const int nw = gridDim.x * wpb;
    dd se{0.0, 0.0};
    int bad = 0;
    for (int c = wid; c < N; c += nw) {
        const i64 b = indptr[c], e = indptr[c + 1];
        const int a = code[c];
        u32 pos = 0;
        for (i64 k = b + lane; k < e; k += 64) {
            const double x = vals[k];
            const int g = rows[k];
            bad |= !(x - x == 0.0) | (g < 0) | (g >= G);
            pos += (x > 0.0);
            if (want_expm1) se = dd_add_d(se, expm1(x));
            if (a >= 0 && x != 0.0 && g >= 0 && g < G) {
                atomicAdd(&cnt[(size_t)g * K + a], 1u);
                if (x < 0.0) atomicAdd(&neg[(size_t)g * K + a], 1u);
            }
        }
        pos = u32_wave_sum(pos);
        if (lane == 0) nodg[c] = (int)pos;
    }
    if (want_expm1) {
        se = dd_wave_sum(se);
        if (lane == 0) wave_expm1[wid] = se;
    }
    if (bad) atomicOr(err, 1);
}

// Dense R matrix (G x N column-major): same outputs.  One wave per cell column.
__global__ void __launch_bounds__(256) k_ingest_count_dense(const double* __restrict__ X, int N, int G, int K,
                                                            const int* __restrict__ code, u32* __restrict__ cnt,
                                                            u32* __restrict__ neg, int* __restrict__ nodg,
                                                            dd* __restrict__ wave_expm1, int want_expm1,
                                                            int* __restrict__ err)
{
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    const int wid = blockIdx.x * wpb + (threadIdx.x >> 6);
    const int nw = gridDim.x * wpb;
    dd se{0.0, 0.0};
    int bad = 0;
    for (int c = wid; c < N; c += nw) {
        const double* col = X + (size_t)c * G;
        const int a = code[c];
        u32 pos = 0;
        for (int g = lane; g < G; g += 64) {
            const double x = col[g];
            bad |= !(x - x == 0.0);
            pos += (x > 0.0);
            if (want_expm1) se = dd_add_d(se, expm1(x));
            if (a >= 0 && x != 0.0) {
                atomicAdd(&cnt[(size_t)g * K + a], 1u);
                if (x < 0.0) atomicAdd(&neg[(size_t)g * K + a], 1u);
            }
        }
        pos = u32_wave_sum(pos);
        if (lane == 0) nodg[c] = (int)pos;
    }
    if (want_expm1) {
        se = dd_wave_sum(se);
        if (lane == 0) wave_expm1[wid] = se;
    }
    if (bad) atomicOr(err, 1);
}

// Scatter kept nonzeros into their (gene, cluster) bucket as orderable keys.
__global__ void __launch_bounds__(256) k_ingest_scatter(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                        const double* __restrict__ vals, int N, int G, int K,
                                                        const int* __restrict__ code, const i64* __restrict__ seg_off,
                                                        u32* __restrict__ cursor, u64* __restrict__ keys)
{
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    const int wid = blockIdx.x * wpb + (threadIdx.x >> 6);
    const int nw = gridDim.x * wpb;
    for (int c = wid; c < N; c += nw) {
        const int a = code[c];
        if (a < 0) continue;
        const i64 b = indptr[c], e = indptr[c + 1];
        for (i64 k = b + lane; k < e; k += 64) {
            const double x = vals[k];
            const int g = rows[k];
            if (x != 0.0 && g >= 0 && g < G) {
                const size_t s = (size_t)g * K + a;
                const u32 slot = atomicAdd(&cursor[s], 1u);
                keys[seg_off[s] + slot] = scc_key_of(x);
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_ingest_scatter_dense(const double* __restrict__ X, int N, int G, int K,
                                                              const int* __restrict__ code,
                                                              const i64* __restrict__ seg_off,
                                                              u32* __restrict__ cursor, u64* __restrict__ keys)
{
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    const int wid = blockIdx.x * wpb + (threadIdx.x >> 6);
    const int nw = gridDim.x * wpb;
    for (int c = wid; c < N; c += nw) {
        const int a = code[c];
        if (a < 0) continue;
        const double* col = X + (size_t)c * G;
        for (int g = lane; g < G; g += 64) {
            const double x = col[g];
            if (x != 0.0) {
                const size_t s = (size_t)g * K + a;
                const u32 slot = atomicAdd(&cursor[s], 1u);
                keys[seg_off[s] + slot] = scc_key_of(x);
            }
        }
    }
}

// ------------------------------------------------------------ exclusive scan
// Three-kernel device-wide exclusive scan of u32 counts into i64 offsets
// (n up to G*K = 2M buckets at the 1M-cell config).
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
    const i64 base = (i64)blockIdx.x * SCAN_T * SCAN_PER;
    for (int k = 0; k < SCAN_PER; ++k) {
        int li = k * SCAN_T + threadIdx.x;
        i64 i = base + li;
        s[li] = (i < n) ? (i64)in[i] : 0;
    }
    __syncthreads();
    // each thread scans SCAN_PER contiguous, then block scan of thread totals
    __shared__ i64 t[SCAN_T];
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
extern "C" hipError_t scc_launch_ingest_count(const i64* indptr, const int* rows, const double* vals,
                                              const double* dense, int N, int G, int K, const int* code,
                                              u32* cnt, u32* neg, int* nodg, dd* wave_expm1, int nwaves,
                                              int want_expm1, int* err, hipStream_t st)
{
    int blocks = nwaves / 4;
    if (dense)
        hipLaunchKernelGGL(k_ingest_count_dense, dim3(blocks), dim3(256), 0, st, dense, N, G, K, code, cnt, neg, nodg,
                           wave_expm1, want_expm1, err);
    else
        hipLaunchKernelGGL(k_ingest_count, dim3(blocks), dim3(256), 0, st, indptr, rows, vals, N, G, K, code, cnt, neg,
                           nodg, wave_expm1, want_expm1, err);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_ingest_scatter(const i64* indptr, const int* rows, const double* vals,
                                                const double* dense, int N, int G, int K, const int* code,
                                                const i64* seg_off, u32* cursor, u64* keys, int nwaves, hipStream_t st)
{
    int blocks = nwaves / 4;
    if (dense)
        hipLaunchKernelGGL(k_ingest_scatter_dense, dim3(blocks), dim3(256), 0, st, dense, N, G, K, code, seg_off,
                           cursor, keys);
    else
        hipLaunchKernelGGL(k_ingest_scatter, dim3(blocks), dim3(256), 0, st, indptr, rows, vals, N, G, K, code, seg_off,
                           cursor, keys);
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
