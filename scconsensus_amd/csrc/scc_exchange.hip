// scc_exchange.hip — compact per-(pair, tested gene) records for the sharded
// DE exchange ("gather of compact per-(pair, gene) records").
//
// The reference's pair loop runs in PSOCK workers and rbind()s their data
// frames in i order (R/reclusterDEConsensusFast.R:61-65,359-384).  Here each
// rank ranks its gene row-block; the cells a pair tests (FAST: the features
// passing Fast:242-291; SLOW: every gene, slow:90) are packed as 64-byte
// records in (pair, gene) order, all-gathered over RCCL, and scattered back
// into the dense [pair][gene] layout the selection kernels read.
#include "scc_common.hpp"
#include "scc.h"

#define RC_T 256
#define RC_PER 4  // cells per thread
#define RC_BLOCK (RC_T * RC_PER)

__device__ inline bool rec_take(const u8* flags, int G, int glo, int W, int all, long long e, long long total, int& p,
                                int& g)
{
    if (e >= total) return false;
    p = (int)(e / W);
    g = glo + (int)(e - (long long)p * W);
    return all || (flags[(size_t)p * G + g] & 1);
}

// records per block of RC_BLOCK consecutive cells
__global__ void __launch_bounds__(RC_T) k_rec_count(const u8* __restrict__ flags, int G, int glo, int W, int all,
                                                    long long total, u32* __restrict__ cnt)
{
    __shared__ u32 ws[RC_T / 64];
    const long long e0 = (long long)blockIdx.x * RC_BLOCK + (long long)threadIdx.x * RC_PER;
    u32 c = 0;
#pragma unroll
    for (int q = 0; q < RC_PER; ++q) {
        int p, g;
        c += rec_take(flags, G, glo, W, all, e0 + q, total, p, g) ? 1u : 0u;
    }
    c = u32_wave_sum(c);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 s = 0;
        for (int w = 0; w < RC_T / 64; ++w) s += ws[w];
        cnt[blockIdx.x] = s;
    }
}

// the records of each block at its scanned offset, in cell order
__global__ void __launch_bounds__(RC_T) k_rec_pack(const u8* __restrict__ flags, int G, int glo, int W, int all,
                                                   long long total, const long long* __restrict__ off,
                                                   const double* __restrict__ p_, const double* __restrict__ lfc,
                                                   const double* __restrict__ pct1, const double* __restrict__ pct2,
                                                   const long long* __restrict__ u2, const long long* __restrict__ t,
                                                   scc_de_record* __restrict__ out)
{
    __shared__ u32 ws[RC_T / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const long long e0 = (long long)blockIdx.x * RC_BLOCK + (long long)tid * RC_PER;
    bool take[RC_PER];
    int pp[RC_PER], gg[RC_PER];
    u32 c = 0;
#pragma unroll
    for (int q = 0; q < RC_PER; ++q) {
        take[q] = rec_take(flags, G, glo, W, all, e0 + q, total, pp[q], gg[q]);
        c += take[q] ? 1u : 0u;
    }
    u32 incl = c;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    long long pos = off[blockIdx.x] + (incl - c);
    for (int v = 0; v < w; ++v) pos += ws[v];
#pragma unroll
    for (int q = 0; q < RC_PER; ++q) {
        if (!take[q]) continue;
        const size_t e = (size_t)pp[q] * G + gg[q];
        scc_de_record r;
        r.pair = pp[q];
        r.gene = gg[q];
        r.p = p_[e];
        r.avg_logfc = lfc[e];
        r.pct1 = pct1 ? pct1[e] : 0.0;
        r.pct2 = pct2 ? pct2[e] : 0.0;
        r.u2 = u2[e];
        r.ties = t[e];
        r.flags = flags[e];
        r.reserved = 0;
        out[pos++] = r;
    }
}

__global__ void __launch_bounds__(256) k_rec_scatter(const scc_de_record* __restrict__ rec, long long n, int G, int P,
                                                     double* __restrict__ p_, double* __restrict__ lfc,
                                                     double* __restrict__ pct1, double* __restrict__ pct2,
                                                     long long* __restrict__ u2, long long* __restrict__ t,
                                                     u8* __restrict__ flags, int* __restrict__ err, int plo, int phi)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const scc_de_record r = rec[i];
        if (r.pair < 0 || r.pair >= P || r.gene < 0 || r.gene >= G) {
            atomicOr(err, 16);  // a malformed record
            continue;
        }
        if (r.pair < plo || r.pair >= phi) continue;  // another rank's pair block (pair-split selection)
        const size_t e = (size_t)r.pair * G + r.gene;
        p_[e] = r.p;
        lfc[e] = r.avg_logfc;
        if (pct1) pct1[e] = r.pct1;
        if (pct2) pct2[e] = r.pct2;
        u2[e] = r.u2;
        t[e] = r.ties;
        flags[e] = (u8)r.flags;
    }
}

extern "C" int scc_rec_blocks(long long cells) { return (int)((cells + RC_BLOCK - 1) / RC_BLOCK); }

extern "C" hipError_t scc_launch_rec_count(const uint8_t* flags, int G, int P, int glo, int ghi, int all, u32* cnt,
                                           hipStream_t st)
{
    const int W = ghi - glo;
    const long long total = (long long)P * W;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rec_count, dim3(scc_rec_blocks(total)), dim3(RC_T), 0, st, flags, G, glo, W, all, total, cnt);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_rec_pack(const uint8_t* flags, int G, int P, int glo, int ghi, int all,
                                          const long long* off, const double* p, const double* lfc, const double* pct1,
                                          const double* pct2, const long long* u2, const long long* t,
                                          scc_de_record* out, hipStream_t st)
{
    const int W = ghi - glo;
    const long long total = (long long)P * W;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rec_pack, dim3(scc_rec_blocks(total)), dim3(RC_T), 0, st, flags, G, glo, W, all, total, off, p,
                       lfc, pct1, pct2, u2, t, out);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_rec_scatter(const scc_de_record* rec, long long n, int G, int P, double* p,
                                             double* lfc, double* pct1, double* pct2, long long* u2, long long* t,
                                             uint8_t* flags, int* err, int plo, int phi, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    const long long nb = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
    hipLaunchKernelGGL(k_rec_scatter, dim3((unsigned)nb), dim3(256), 0, st, rec, n, G, P, p, lfc, pct1, pct2, u2, t,
                       flags, err, plo, phi);
    return hipGetLastError();
}
