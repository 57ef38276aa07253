// scc_rank_seg.hip — the segment rank engine: all-pairs Wilcoxon rank sums of
// every ranked gene from value segments of <= SG_CAP nonzeros, each sorted by
// one workgroup and counted on the int8 matrix cores.
//
// Replaces the reference's per-(pair, gene) `wilcox.test` rank sums
// (R/reclusterDEConsensusFast.R:78-91; R/reclusterDEConsensus.R:99-103) with
// the exact integer accumulators the pair test reads (scc_select.hip
// k_pair_test adds the implicit zero group):
//   S_ab = #{(i in a, j in b): x_j < x_i} over the nonzeros (pair a < b)
//   E_ab = sum over groups of equal values t_a t_b
//   X_ab = sum over groups t_a t_b (t_a + t_b)
//   F_a  = sum over runs of equal values inside cluster a of t^3 - t
//
// Kernels:
//   k_seg_classify  per gene: a ranked gene of <= SG_CAP nonzeros is one
//                   segment, read where the ingest left it (its codes from the
//                   cluster offsets); larger genes go to the splitter.
//   k_seg_split     one 1024-thread workgroup per large gene: distinct
//                   splitters from a regular sample sorted in LDS; the
//                   segments are the open value intervals between splitters
//                   and each splitter's equality class (one repeated value:
//                   closed form, any size); the gene is scattered into
//                   segment order (keys2 / codes2) through an LDS stage, so
//                   every run leaves as consecutive stores.
//   k_seg_rank      one workgroup per segment: the composite key
//                   (key - min) << 7 | cluster sorted bitonically (registers,
//                   DPP / permlane lane swaps, LDS only for strides >= 512);
//                   then per 64-element block (one wave each) M = L O and
//                   S += O^T M on v_mfma_i32_16x16x64_i8 (L: strict lower
//                   triangle of positions, O: the block's one-hot codes), the
//                   cross-block part H^T Cex as two more int8 products (H: the
//                   blocks' cluster counts, Cex their exclusive prefix split
//                   into 6-bit halves); tie groups in closed form.
//   k_seg_cross     one workgroup per split gene: the cross-segment part
//                   sum over segments hseg[a] * (b-elements of earlier segments).
//
// Why the positional count is the strict one: the composite order puts equal
// values by ascending cluster, so for a < b no b-element precedes an equal
// a-element; ties go to E / X / F only.  All sums are integer atomics (order
// free), so the accumulators are bitwise deterministic.
#include "scc_common.hpp"
#include "scc_kernels.hpp"

#define SG_T (SG_CAP / 8)       // the workgroup kernel (wide key ranges): 8 elements per thread
#define SG_KPT 8
#define SG_QMAX (SG_CAP / 64)   // blocks per segment (32)
#define SP2_T 1024              // splitter workgroup
#define SP2_SMAX 4096           // sample keys sorted in LDS
#define SP2_MMAX 2047           // distinct splitters (<= 4095 segments per gene)
#define SP2_CH 4096             // elements per scatter chunk (LDS stage)

typedef int sg_v4i __attribute__((ext_vector_type(4)));

__device__ inline sg_v4i sg_mfma(sg_v4i a, sg_v4i b, sg_v4i c)
{
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// bytes [base + q < x], q = 0..3
__device__ inline u32 sg_lt_bytes(int x, int base)
{
    int v = x - base;
    v = v < 0 ? 0 : (v > 4 ? 4 : v);
    return (u32)((0x01010101ull << (8 * v)) >> 32);
}

// bytes of w equal to c (0 / 1 each)
__device__ inline u32 sg_eq_bytes(u32 w, u32 c)
{
    const u32 x = w ^ (c * 0x01010101u);
    const u32 nz = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;  // bit 7 of a byte: the byte is not zero
    return (~nz >> 7) & 0x01010101u;
}

__device__ inline u32 sg_pack(sg_v4i m)  // four counts < 128 into four bytes
{
    return (u32)(m[0] & 0xff) | ((u32)(m[1] & 0xff) << 8) | ((u32)(m[2] & 0xff) << 16) | ((u32)(m[3] & 0xff) << 24);
}

__device__ inline void sg_wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// pair index of clusters a < b (R's (i, j) loop order, Fast:359)
__device__ inline int sg_pair(int a, int b, int K) { return a * (2 * K - a - 1) / 2 + (b - a - 1); }

__device__ inline bool sg_tested(const ScSegLaunch& A, int p, int g)
{
    return A.all_pairs || (A.flags[(size_t)p * A.G + g] & 1);
}

// position slot of element x (0..63) of a block: the byte its code takes in the
// MFMA operands.  Lane group g, byte t holds element e(g, t) = 16 (t >> 2) +
// 4 g + (t & 3) -- the row the accumulator layout puts in register t & 3 of
// lane group g of row tile t >> 2 -- so the four packed row tiles of M = L O
// are the next product's operand as they stand.
__device__ inline int sg_slot(int x) { return 16 * ((x >> 2) & 3) + 4 * (x >> 4) + (x & 3); }

// SCC_SEG_STAMPS diagnostics: per-phase cycles of workgroup-thread 0, summed
// over segments ([0] load, [1] sort, [2] codes / LDS, [3] blocks, [4] prefix +
// cross-block, [5] flush, [6] ties, [7] segments)
__device__ unsigned long long g_seg_stamps[8];

// ===================================================================== classify
__global__ void k_seg_classify(ScSegLaunch A)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= A.G) return;
    const i64 base = A.gstart[g];
    const i64 n = A.gstart[g + 1] - base;
    if (n <= 0) return;
    if (!A.all_pairs) {
        bool any = false;
        for (int p0 = 0; p0 < A.P && !any; p0 += 16) {
            u8 f[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) f[u] = A.flags[(size_t)min(p0 + u, A.P - 1) * A.G + g];
#pragma unroll
            for (int u = 0; u < 16; ++u) any |= (f[u] & 1) != 0;
        }
        if (!any) return;
    }
    if (n <= SG_CAP) {
        const int s = atomicAdd(&A.counts[0], 1);
        if (s < A.seg_cap)
            A.segs[s] = ScSeg{base, (int)n, g, 0, -1};
        else
            atomicOr(A.err, SCC_SEG_OVERFLOW);
    } else {
        A.big[atomicAdd(&A.counts[1], 1)] = g;
    }
}

// ===================================================================== tested flags, gene-major
// tbg[g][p] = does pair p test gene g (flags[p][g] bit 0, or every pair): a
// segment then reads its gene's P flags as consecutive bytes (the [P][G]
// layout cost P scattered loads per segment).  32 x 32 tiles through LDS.
__global__ void __launch_bounds__(256) k_seg_flags_t(ScSegLaunch A)
{
    __shared__ u8 t[32][33];
    const int p0 = blockIdx.y * 32, g0 = blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
    for (int r = ty; r < 32; r += 8) {
        const int p = p0 + r, g = g0 + tx;
        t[r][tx] = (p < A.P && g < A.G) ? (A.all_pairs ? 1 : (A.flags[(size_t)p * A.G + g] & 1)) : 0;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int g = g0 + r, p = p0 + tx;
        if (g < A.G && p < A.P) A.tbg[(size_t)g * A.P + p] = t[tx][r];
    }
}

// ===================================================================== split
struct Sp2Lds {
    int off[SCC_MAX_K + 1];
    u64 spl[SP2_MMAX + 1];
    u32 hist[2 * SP2_MMAX + 2];  // per segment: gene counts, then the running write cursor
    u32 boff[2 * SP2_MMAX + 2];
    u32 chist[2 * SP2_MMAX + 2];
    u32 lscan[2 * SP2_MMAX + 2];
    u32 dst[2 * SP2_MMAX + 2];
    u32 wsum[SP2_T / 64 + 1];
    int m, nne, s0, h0, next;
    // the sample sort and, after it, the scatter stage
    u64 stk[SP2_CH];
    u8 stc[SP2_CH];
    uint16_t stb[SP2_CH];
};
static_assert(sizeof(Sp2Lds) <= 160 * 1024, "splitter LDS");

// exclusive block scan of one value per thread (1024 threads); returns the
// prefix, *total the sum (uniform)
__device__ inline u32 sp2_scan(u32 v, Sp2Lds& L, u32* total)
{
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32 incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) L.wsum[w] = incl;
    __syncthreads();
    u32 pre = 0, tot = 0;
    for (int q = 0; q < SP2_T / 64; ++q) {
        const u32 s = L.wsum[q];
        pre += q < w ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return pre + incl - v;
}

__device__ inline int sp2_code(const Sp2Lds& L, int K, int i)  // cluster of gene element i (cluster-grouped order)
{
    int lo = 0, hi = K - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (L.off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// segment of key x: 2 lb + [x == spl[lb]], lb = #{splitters < x}
__device__ inline int sp2_bucket(const Sp2Lds& L, int m, u64 x)
{
    int lo = 0, hi = m;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (L.spl[mid] < x) lo = mid + 1; else hi = mid;
    }
    return 2 * lo + ((lo < m && L.spl[lo] == x) ? 1 : 0);
}

__device__ void seg_split_gene(const ScSegLaunch& A, int bi, int g, Sp2Lds& L)
{
    const int K = A.K, G = A.G;
    const int tid = threadIdx.x;
    const i64 base = A.gstart[g];
    const int n = (int)(A.gstart[g + 1] - base);
    const u64* key = A.keys + base;
    if (tid <= K) L.off[tid] = (int)A.coff[(size_t)A.cl_cc[tid] * G + g];
    // ---- 1. a regular sample, sorted in LDS (bitonic)
    const int nseg = min(SP2_MMAX + 1, max(2, (n + SG_TGT - 1) / SG_TGT));
    const int s = min(n, min(SP2_SMAX, A.sample_os * nseg));  // sample_os: oversampling (32; tests: 1)
    int S2 = 64;
    while (S2 < s) S2 <<= 1;
    for (int k = tid; k < S2; k += SP2_T) L.stk[k] = k < s ? key[(i64)k * n / s] : ~0ull;
    __syncthreads();
    for (int k = 2; k <= S2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int e = tid; e < S2 / 2; e += SP2_T) {
                const int i = 2 * j * (e / j) + (e % j), p = i + j;  // i has bit j clear
                const u64 a = L.stk[i], b = L.stk[p];
                const bool asc = (i & k) == 0;
                if (asc ? (b < a) : (a < b)) {
                    L.stk[i] = b;
                    L.stk[p] = a;
                }
            }
            __syncthreads();
        }
    // ---- 2. distinct splitters: candidates at nseg - 1 regular sample ranks
    {
        const int j = tid + 1;  // candidate j of 1 .. nseg - 1
        u64 v = 0;
        bool keep = false;
        if (j < nseg) {
            v = L.stk[(i64)j * s / nseg];
            keep = j == 1 || v != L.stk[(i64)(j - 1) * s / nseg];
        }
        u32 tot;
        const u32 pos = sp2_scan(keep ? 1u : 0u, L, &tot);
        if (keep) L.spl[pos] = v;
        if (tid == 0) L.m = (int)tot;
    }
    __syncthreads();
    const int m = L.m, nb = 2 * m + 1;
    for (int b = tid; b < nb; b += SP2_T) L.hist[b] = 0;
    __syncthreads();
    // ---- 3. segment sizes
    for (int i = tid; i < n; i += SP2_T) atomicAdd(&L.hist[sp2_bucket(L, m, key[i])], 1u);
    __syncthreads();
    {
        const u32 h0 = 2 * tid < nb ? L.hist[2 * tid] : 0u, h1 = 2 * tid + 1 < nb ? L.hist[2 * tid + 1] : 0u;
        u32 tot;
        const u32 pre = sp2_scan(h0 + h1, L, &tot);
        if (2 * tid < nb) L.boff[2 * tid] = pre;
        if (2 * tid + 1 < nb) L.boff[2 * tid + 1] = pre + h0;
        const u32 ne = (h0 > 0) + (h1 > 0);
        u32 totne;
        const u32 r = sp2_scan(ne, L, &totne);
        if (tid == 0) {
            L.nne = (int)totne;
            L.s0 = atomicAdd(&A.counts[0], (int)totne);
            L.h0 = atomicAdd(&A.counts[2], (int)totne);
        }
        __syncthreads();
        const int s0 = L.s0, hr0 = L.h0;
        const bool fits = s0 + (int)totne <= A.seg_cap && hr0 + (int)totne <= A.hrow_cap;
        if (!fits) {
            if (tid == 0) atomicOr(A.err, SCC_SEG_OVERFLOW);
        } else {
            if (h0) A.segs[s0 + r] = ScSeg{base + pre, (int)h0, g, 1, hr0 + (int)r};
            // an interval segment larger than a workgroup's sort (the sample
            // missed a dense stretch): cut again after the scatter (k_seg_refine)
            if (h0 > SG_CAP) {
                const int o = atomicAdd(&A.counts[4], 1);
                if (o < A.ovf_cap) A.ovf[o] = s0 + (int)r; else atomicOr(A.err, SCC_SEG_OVERFLOW);
            }
            if (h1) A.segs[s0 + r + (h0 > 0)] = ScSeg{base + pre + h0, (int)h1, g, 2, hr0 + (int)r + (h0 > 0)};
        }
        if (tid == 0) A.gseg[bi] = int4{hr0, fits ? (int)totne : 0, g, 0};
    }
    __syncthreads();
    // ---- 4. scatter into segment order through the LDS stage (write cursors in hist)
    for (int b = tid; b < nb; b += SP2_T) L.hist[b] = L.boff[b];
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += SP2_CH) {
        const int cn = min(SP2_CH, n - c0);
        for (int b = tid; b < nb; b += SP2_T) L.chist[b] = 0;
        __syncthreads();
        constexpr int PT = SP2_CH / SP2_T;
        u64 kv[PT];
        int bk[PT];
        u32 lr[PT];
#pragma unroll
        for (int q = 0; q < PT; ++q) {
            const int i = c0 + q * SP2_T + tid;
            bk[q] = -1;
            if (i < c0 + cn) {
                kv[q] = key[i];
                bk[q] = sp2_bucket(L, m, kv[q]);
                lr[q] = atomicAdd(&L.chist[bk[q]], 1u);
            }
        }
        __syncthreads();
        {
            const u32 h0 = 2 * tid < nb ? L.chist[2 * tid] : 0u, h1 = 2 * tid + 1 < nb ? L.chist[2 * tid + 1] : 0u;
            u32 tot;
            const u32 pre = sp2_scan(h0 + h1, L, &tot);
            if (2 * tid < nb) {
                L.lscan[2 * tid] = pre;
                L.dst[2 * tid] = L.hist[2 * tid];
                L.hist[2 * tid] += h0;
            }
            if (2 * tid + 1 < nb) {
                L.lscan[2 * tid + 1] = pre + h0;
                L.dst[2 * tid + 1] = L.hist[2 * tid + 1];
                L.hist[2 * tid + 1] += h1;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PT; ++q) {
            if (bk[q] >= 0) {
                const int i = c0 + q * SP2_T + tid;
                const u32 sp = L.lscan[bk[q]] + lr[q];
                L.stk[sp] = kv[q];
                L.stc[sp] = (u8)sp2_code(L, K, i);
                L.stb[sp] = (uint16_t)bk[q];
            }
        }
        __syncthreads();
        for (int sp = tid; sp < cn; sp += SP2_T) {
            const int b = L.stb[sp];
            const i64 d = base + L.dst[b] + (sp - L.lscan[b]);
            A.keys2[d] = L.stk[sp];
            A.codes2[d] = L.stc[sp];
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(SP2_T) k_seg_split(ScSegLaunch A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Sp2Lds& L = *(Sp2Lds*)smem;
    const int cnt = A.counts[1];
    for (;;) {  // genes from a queue (their sizes vary by orders of magnitude)
        if (threadIdx.x == 0) L.next = atomicAdd(&A.counts[3], 1);
        __syncthreads();
        const int i = L.next;
        __syncthreads();
        if (i >= cnt) break;
        seg_split_gene(A, i, A.big[i], L);
    }
}

// ===================================================================== rank
// one element of the sort: the composite key (C) or key and code (wide range)
template <bool C>
struct SgEl;
// (selects are member-wise on values: a conditional between two struct
// lvalues selects an address, which put the whole register array in scratch)
template <>
struct SgEl<true> {
    u64 k;
    __device__ bool lt(const SgEl& o) const { return k < o.k; }
    __device__ static SgEl sel(bool c, SgEl x, SgEl y) { return SgEl{c ? x.k : y.k}; }
};
template <>
struct SgEl<false> {
    u64 k;
    u32 c;
    __device__ bool lt(const SgEl& o) const { return k < o.k || (k == o.k && c < o.c); }
    __device__ static SgEl sel(bool b, SgEl x, SgEl y) { return SgEl{b ? x.k : y.k, b ? x.c : y.c}; }
};

template <int D>
__device__ inline u64 sg_xor64(u64 v)
{
    return ((u64)scc_xor_lane<D>((u32)(v >> 32)) << 32) | scc_xor_lane<D>((u32)v);
}
template <int D>
__device__ inline SgEl<true> sg_xor(const SgEl<true>& e)
{
    return SgEl<true>{sg_xor64<D>(e.k)};
}
template <int D>
__device__ inline SgEl<false> sg_xor(const SgEl<false>& e)
{
    return SgEl<false>{sg_xor64<D>(e.k), scc_xor_lane<D>(e.c)};
}

template <bool C>
__device__ inline void sg_ce(SgEl<C>& a, SgEl<C>& b, bool asc)  // a: the lower index
{
    const bool sw = asc ? b.lt(a) : a.lt(b);
    const SgEl<C> x = SgEl<C>::sel(sw, b, a), y = SgEl<C>::sel(sw, a, b);
    a = x;
    b = y;
}

// one stride-d lane-swap stage: keep the min where (t & d) == 0 matches asc
template <int D, bool C>
__device__ inline void sg_lane_stage(SgEl<C> (&v)[SG_KPT], bool keep_min)
{
#pragma unroll
    for (int i = 0; i < SG_KPT; ++i) {
        const SgEl<C> p = sg_xor<D>(v[i]);
        const bool take = keep_min ? p.lt(v[i]) : v[i].lt(p);
        v[i] = SgEl<C>::sel(take, p, v[i]);
    }
}

struct SegRankLds {
    int off[SCC_MAX_K + 1];
    int any_tie;
    ScSeg seg;
    u64 kmn_w[SG_T / 64], kmx_w[SG_T / 64];
    u64 sk[SG_CAP];    // the sort's LDS stages, then the sorted key (composite: key << 7 | code)
    u8 cn[SG_CAP];     // sorted codes, natural order
    alignas(16) u8 cs[SG_CAP];  // sorted codes, operand-slot order per 64-element block
    u32 hc[SCC_MAX_K]; // the equality segment's cluster counts
};
// after SegRankLds (dynamic LDS): HT, CL, CH [Kp][32] u8, then Sred [NT][256] u32

template <int KT>
__device__ constexpr int sg_tile(int u0, int u1)  // upper tiles (u0 <= u1) in row order
{
    return u0 * KT - u0 * (u0 - 1) / 2 + (u1 - u0);
}

template <bool C>
__device__ inline void sg_sort(SgEl<C> (&v)[SG_KPT], int M, SegRankLds& L, const bool active)
{
    const int t = threadIdx.x;
    // k = 2, 4, 8 inside the thread's 8 consecutive elements (directions from e = 8 t + i)
    if (active) {
#pragma unroll
        for (int k = 2; k <= 8; k <<= 1)
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
                for (int i = 0; i < SG_KPT; ++i)
                    if ((i & j) == 0) sg_ce<C>(v[i], v[i | j], ((8 * t + i) & k) == 0);
    }
    for (int k = 16; k <= M; k <<= 1) {
        const bool asc = ((8 * t) & k) == 0;
        for (int j = k >> 1; j >= 8; j >>= 1) {
            if (j >= 512) {  // across waves: through LDS
                __syncthreads();
                if constexpr (C) {
#pragma unroll
                    for (int i = 0; i < SG_KPT; ++i) L.sk[8 * t + i] = v[i].k;
                } else {
#pragma unroll
                    for (int i = 0; i < SG_KPT; ++i) {
                        L.sk[8 * t + i] = v[i].k;
                        L.cn[8 * t + i] = (u8)v[i].c;
                    }
                }
                __syncthreads();
#pragma unroll
                for (int i = 0; i < SG_KPT; ++i) {
                    const int e = 8 * t + i, pe = e ^ j;
                    SgEl<C> p;
                    p.k = L.sk[pe];
                    if constexpr (!C) p.c = L.cn[pe];
                    const bool keep_min = ((e & j) == 0) == asc;
                    const bool take = keep_min ? p.lt(v[i]) : v[i].lt(p);
                    v[i] = SgEl<C>::sel(take, p, v[i]);
                }
            } else if (active) {
                const int d = j >> 3;
                const bool keep_min = ((t & d) == 0) == asc;
                switch (d) {
                case 1: sg_lane_stage<1, C>(v, keep_min); break;
                case 2: sg_lane_stage<2, C>(v, keep_min); break;
                case 4: sg_lane_stage<4, C>(v, keep_min); break;
                case 8: sg_lane_stage<8, C>(v, keep_min); break;
                case 16: sg_lane_stage<16, C>(v, keep_min); break;
                default: sg_lane_stage<32, C>(v, keep_min); break;
                }
            }
        }
        if (active) {
#pragma unroll
            for (int j = 4; j > 0; j >>= 1)
#pragma unroll
                for (int i = 0; i < SG_KPT; ++i)
                    if ((i & j) == 0) sg_ce<C>(v[i], v[i | j], asc);
        }
    }
}

// The composite-key sort (u64 per element) with lane masks: a compare-exchange
// is two lane moves, one 64-bit compare into a lane mask, one scalar XNOR with
// the stage's keep-min (or ascending) mask and two selects -- the bool
// selects of the generic form compiled to ~15 instructions per element.
__device__ inline u32 sgc_sel(u64 m, u32 a, u32 b)  // per lane: bit set -> b
{
    u32 r;
    asm("" : "+s"(m));  // the mask in an SGPR pair (a folded constant is no operand of this form)
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
__device__ inline u64 sgc_sel64(u64 m, u64 a, u64 b)
{
    return ((u64)sgc_sel(m, (u32)(a >> 32), (u32)(b >> 32)) << 32) | sgc_sel(m, (u32)a, (u32)b);
}
// a (lower index) and b: the min to a where the lane's bit of am is set (ascending)
__device__ inline void sgc_ce(u64& a, u64& b, u64 am)
{
    const u64 sw = ~(__ballot(b < a) ^ am);  // ascending: swap if b < a; descending: if not
    const u64 x = sgc_sel64(sw, a, b), y = sgc_sel64(sw, b, a);
    a = x;
    b = y;
}
template <int D>
__device__ inline void sgc_lane_stage(u64 (&v)[SG_KPT], u64 km)
{
#pragma unroll
    for (int i = 0; i < SG_KPT; ++i) {
        const u64 p = sg_xor64<D>(v[i]);
        const u64 take = ~(__ballot(p < v[i]) ^ km);  // keep-min lanes take a smaller partner, keep-max a larger
        v[i] = sgc_sel64(take, v[i], p);
    }
}

template <int D, int EPL>
__device__ inline void sgc_lane_stage_n(u64 (&v)[EPL], u64 km)
{
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
        const u64 p = sg_xor64<D>(v[i]);
        const u64 take = ~(__ballot(p < v[i]) ^ km);
        v[i] = sgc_sel64(take, v[i], p);
    }
}
__device__ inline u64 sw_shfl_down64(u64 v, int d)
{
    return ((u64)(u32)__shfl_down((int)(u32)(v >> 32), d, 64) << 32) | (u32)__shfl_down((int)(u32)v, d, 64);
}
__device__ inline u64 sw_shfl_up64(u64 v, int d)
{
    return ((u64)(u32)__shfl_up((int)(u32)(v >> 32), d, 64) << 32) | (u32)__shfl_up((int)(u32)v, d, 64);
}

__device__ inline void sgc_sort(u64 (&v)[SG_KPT], int M, SegRankLds& L, const bool active)
{
    const int t = threadIdx.x;
    if (active) {
        // k = 2, 4: directions from the register index; k = 8: from bit 0 of t
#pragma unroll
        for (int i = 0; i < SG_KPT; i += 2) sgc_ce(v[i], v[i + 1], (i & 2) == 0 ? ~0ull : 0ull);
#pragma unroll
        for (int j = 2; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < SG_KPT; ++i)
                if ((i & j) == 0) sgc_ce(v[i], v[i | j], (i & 4) == 0 ? ~0ull : 0ull);
        const u64 a8 = __ballot((t & 1) == 0);
#pragma unroll
        for (int j = 4; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < SG_KPT; ++i)
                if ((i & j) == 0) sgc_ce(v[i], v[i | j], a8);
    }
    for (int k = 16; k <= M; k <<= 1) {
        const bool asc = ((8 * t) & k) == 0;
        for (int j = k >> 1; j >= 8; j >>= 1) {
            if (j >= 512) {  // across waves: through LDS
                __syncthreads();
#pragma unroll
                for (int i = 0; i < SG_KPT; ++i) L.sk[8 * t + i] = v[i];
                __syncthreads();
#pragma unroll
                for (int i = 0; i < SG_KPT; ++i) {
                    const int e = 8 * t + i;
                    const u64 p = L.sk[e ^ j];
                    const bool keep_min = ((e & j) == 0) == asc;
                    v[i] = keep_min ? (p < v[i] ? p : v[i]) : (p > v[i] ? p : v[i]);
                }
            } else if (active) {
                const int d = j >> 3;
                const u64 km = __ballot(((t & d) == 0) == asc);
                switch (d) {
                case 1: sgc_lane_stage<1>(v, km); break;
                case 2: sgc_lane_stage<2>(v, km); break;
                case 4: sgc_lane_stage<4>(v, km); break;
                case 8: sgc_lane_stage<8>(v, km); break;
                case 16: sgc_lane_stage<16>(v, km); break;
                default: sgc_lane_stage<32>(v, km); break;
                }
            }
        }
        if (active) {
            const u64 am = __ballot(asc);
#pragma unroll
            for (int j = 4; j > 0; j >>= 1)
#pragma unroll
                for (int i = 0; i < SG_KPT; ++i)
                    if ((i & j) == 0) sgc_ce(v[i], v[i | j], am);
        }
    }
}

// one segment of n <= SG_CAP elements (kind 0 / 1): sort, blocks, cross-block
// part, flush, ties, the segment's cluster counts
template <int KT, bool C>
__device__ void seg_rank_sorted(const ScSegLaunch& A, SegRankLds& L, u8* HT, u8* CL, u8* CH, u32* Sred,
                                u32* Ep, u32* Xp, u64* Fc, const u64 kmn)
{
    constexpr int Kp = 16 * KT, NT = KT * (KT + 1) / 2;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g4 = lane >> 4, r16 = lane & 15;
    const ScSeg sg = L.seg;
    const int n = sg.n, g = sg.gene, K = A.K, G = A.G;
    int M = 64;
    while (M < n) M <<= 1;
    const bool active = 512 * w < M;
    const bool stm = A.stamps && tid == 0;
    u64 tprev = stm ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int ph) {
        if (stm) {
            const u64 t = __builtin_amdgcn_s_memtime();
            atomicAdd(&g_seg_stamps[ph], (unsigned long long)(t - tprev));
            tprev = t;
        }
    };
    // the gene's tested pairs (one flag byte per pair, loaded once per segment)
    u8* tb = (u8*)(Fc + K);
    for (int p = tid; p < A.P; p += SG_T) tb[p] = sg_tested(A, p, g) ? 1 : 0;
    // ---- load (elements 8 t .. 8 t + 7) and the sort key
    SgEl<C> v[SG_KPT];
    {
        const u64* src = sg.kind == 0 ? A.keys : A.keys2;
        int a = 0;
        if (sg.kind == 0 && 8 * tid < n) {  // cluster of the first element: the gene's cluster offsets
            int lo = 0, hi = K - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (L.off[mid] <= 8 * tid) lo = mid; else hi = mid - 1;
            }
            a = lo;
        }
#pragma unroll
        for (int i = 0; i < SG_KPT; ++i) {
            const int e = 8 * tid + i;
            u64 k = ~0ull;
            u32 c = SCC_CODE_MASK;
            if (e < n) {
                k = src[sg.base + e];
                if (sg.kind == 0) {
                    while (a + 1 < K && L.off[a + 1] <= e) ++a;
                    c = (u32)a;
                } else {
                    c = A.codes2[sg.base + e];
                }
            }
            if constexpr (C) {
                v[i].k = e < n ? (((k - kmn) << SCC_CODE_BITS) | c) : ~0ull;
            } else {
                v[i].k = k;
                v[i].c = e < n ? c : 0xffu;
            }
        }
    }
    stamp(0);
    if (!(A.dbg & 1)) {
        if constexpr (C) {
            u64 ck[SG_KPT];
#pragma unroll
            for (int i = 0; i < SG_KPT; ++i) ck[i] = v[i].k;
            sgc_sort(ck, M, L, active);
#pragma unroll
            for (int i = 0; i < SG_KPT; ++i) v[i].k = ck[i];
        } else {
            sg_sort<C>(v, M, L, active);
        }
    }
    __syncthreads();  // every LDS stage read is done before sk is rewritten
    stamp(1);
    // ---- sorted key and codes to LDS; the slot-ordered codes of the blocks
    const int nq = (n + 63) >> 6;
#pragma unroll
    for (int i = 0; i < SG_KPT; ++i) {
        const int e = 8 * tid + i;
        if (e < nq * 64) {
            u32 c;
            if constexpr (C) c = (u32)(v[i].k & SCC_CODE_MASK); else c = v[i].c;
            if (e >= n) c = 0xffu;
            L.cs[(e & ~63) + sg_slot(e & 63)] = (u8)c;
            if (e < n) {
                L.cn[e] = (u8)c;
                L.sk[e] = v[i].k;
            }
        }
    }
    for (int i = tid; i < Kp * 32; i += SG_T) {
        ((u8*)HT)[i] = 0;
    }
    for (int i = tid; i < NT * 256; i += SG_T) Sred[i] = 0;
    if (tid == 0) L.any_tie = 0;
    __syncthreads();
    // ---- ties (equal values next to each other)?
    {
        bool tie = false;
#pragma unroll
        for (int i = 0; i < SG_KPT; ++i) {
            const int e = 8 * tid + i;
            if (e + 1 < n) {
                if constexpr (C) tie |= (L.sk[e] >> SCC_CODE_BITS) == (L.sk[e + 1] >> SCC_CODE_BITS);
                else tie |= L.sk[e] == L.sk[e + 1];
            }
        }
        if (__any(tie) && lane == 0) atomicOr(&L.any_tie, 1);
    }
    stamp(2);
    // ---- blocks: one wave each; M = L O and S += O^T M per block
    sg_v4i Lm[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int d = 0; d < 4; ++d) Lm[mt][d] = (int)sg_lt_bytes(16 * mt + r16, 16 * d + 4 * g4);
    const sg_v4i zero = {0, 0, 0, 0};
    sg_v4i S[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) S[q] = zero;
    for (int q = w; q < ((A.dbg & 2) ? 0 : nq); q += SG_T / 64) {
        const uint4 cw = *(const uint4*)&L.cs[64 * q + 16 * g4];
        sg_v4i Ob[KT];
#pragma unroll
        for (int u = 0; u < KT; ++u) {
            const u32 c = (u32)(16 * u + r16);
            Ob[u] = sg_v4i{(int)sg_eq_bytes(cw.x, c), (int)sg_eq_bytes(cw.y, c), (int)sg_eq_bytes(cw.z, c),
                           (int)sg_eq_bytes(cw.w, c)};
        }
#pragma unroll
        for (int u = 0; u < KT; ++u) {
            const sg_v4i m0 = sg_mfma(Lm[0], Ob[u], zero);
            const sg_v4i m1 = sg_mfma(Lm[1], Ob[u], zero);
            const sg_v4i m2 = sg_mfma(Lm[2], Ob[u], zero);
            const sg_v4i m3 = sg_mfma(Lm[3], Ob[u], zero);
            // H[q][b] = M[63][b] + [code of element 63 == b]: lane group 3, register 3 of row tile 3
            if (g4 == 3) {
                const int b = 16 * u + r16;
                HT[b * 32 + q] = (u8)(m3[3] + (((cw.w >> 24) & 0xffu) == (u32)b ? 1 : 0));
            }
            const sg_v4i Mb = {(int)sg_pack(m0), (int)sg_pack(m1), (int)sg_pack(m2), (int)sg_pack(m3)};
#pragma unroll
            for (int u0 = 0; u0 <= u; ++u0) S[sg_tile<KT>(u0, u)] = sg_mfma(Ob[u0], Mb, S[sg_tile<KT>(u0, u)]);
        }
    }
    __syncthreads();
    stamp(3);
    // ---- the blocks' exclusive prefix per cluster (6-bit halves) and the segment's counts
    if (tid < Kp) {
        const int c = tid;
        u32 run = 0;
        for (int q = 0; q < 32; ++q) {
            const u32 h = HT[c * 32 + q];
            CL[c * 32 + q] = (u8)(run & 63u);
            CH[c * 32 + q] = (u8)(run >> 6);
            run += h;
        }
        if (sg.hrow >= 0 && c < K) A.hseg[(size_t)sg.hrow * K + c] = run;
    }
    __syncthreads();
    // ---- cross-block part H^T Cex (k = block index), tiles dealt to the waves
#pragma unroll
    for (int u0 = 0; u0 < KT; ++u0)
#pragma unroll
        for (int u1 = u0; u1 < KT; ++u1) {
            const int ti = sg_tile<KT>(u0, u1);
            if (ti % (SG_T / 64) != w) continue;
            sg_v4i a = zero, bl = zero, bh = zero;
            if (g4 < 2) {
                const uint4 x = *(const uint4*)&HT[(16 * u0 + r16) * 32 + 16 * g4];
                const uint4 y = *(const uint4*)&CL[(16 * u1 + r16) * 32 + 16 * g4];
                const uint4 z = *(const uint4*)&CH[(16 * u1 + r16) * 32 + 16 * g4];
                a = sg_v4i{(int)x.x, (int)x.y, (int)x.z, (int)x.w};
                bl = sg_v4i{(int)y.x, (int)y.y, (int)y.z, (int)y.w};
                bh = sg_v4i{(int)z.x, (int)z.y, (int)z.z, (int)z.w};
            }
            const sg_v4i hi = sg_mfma(a, bh, zero);
            sg_v4i s = sg_mfma(a, bl, S[ti]);
#pragma unroll
            for (int r = 0; r < 4; ++r) s[r] += hi[r] << 6;
            S[ti] = s;
        }
    // ---- the four waves' tiles summed in LDS
#pragma unroll
    for (int ti = 0; ti < NT; ++ti)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (S[ti][r]) atomicAdd(&Sred[ti * 256 + (4 * g4 + r) * 16 + r16], (u32)S[ti][r]);
    __syncthreads();
    stamp(4);
    // ---- flush: one integer atomic per tested pair with a nonzero count
    for (int idx = tid; idx < Kp * Kp; idx += SG_T) {
        const int a = idx / Kp, b = idx % Kp;
        if (a >= b || b >= K) continue;
        const u32 x = Sred[sg_tile<KT>(a >> 4, b >> 4) * 256 + (a & 15) * 16 + (b & 15)];
        if (!x) continue;
        const int p = sg_pair(a, b, K);
        if (tb[p]) atomicAdd(&A.accS[(size_t)p * G + g], (unsigned long long)x);
    }
    stamp(5);
    // ---- tie groups: F from runs, E and X from pairs of runs (clusters
    // ascending inside a group), summed in LDS and flushed once per segment
    // (per-group global atomics hit the same (pair, gene) words from every
    // group of a gene: at PBMC shape three quarters of a big gene's values tie)
    if (L.any_tie && !(A.dbg & 4)) {
        auto kp = [&](int e) -> u64 {
            if constexpr (C) return L.sk[e] >> SCC_CODE_BITS; else return L.sk[e];
        };
        const int P = A.P;
        for (int i = tid; i < P; i += SG_T) Ep[i] = Xp[i] = 0;
        for (int c = tid; c < K; c += SG_T) Fc[c] = 0;
        __syncthreads();
        // one thread per run of one cluster inside a tie group (runs are the
        // unit of work: a thread per group re-walked the group once per run)
        for (int e = tid; e < n; e += SG_T) {
            const u64 k0 = kp(e);
            const int c = L.cn[e];
            const bool grp = (e + 1 < n && kp(e + 1) == k0) || (e > 0 && kp(e - 1) == k0);
            if (!grp || (e > 0 && kp(e - 1) == k0 && L.cn[e - 1] == c)) continue;  // not a run start in a group
            int r1 = e + 1;
            while (r1 < n && kp(r1) == k0 && L.cn[r1] == c) ++r1;
            const u32 la = (u32)(r1 - e);
            if (la >= 2) atomicAdd(&Fc[c], (u64)la * la * la - la);
            int h = r1;
            while (h < n && kp(h) == k0) {  // the later runs of the group (clusters ascending)
                const int c2 = L.cn[h];
                int r2 = h + 1;
                while (r2 < n && kp(r2) == k0 && L.cn[r2] == c2) ++r2;
                const u32 lb = (u32)(r2 - h);
                const int p = sg_pair(c, c2, K);
                // (a segment holds <= SG_CAP = 2^10 values: E <= 2^20 and X <= 2^31 fit 32 bits)
                atomicAdd(&Ep[p], la * lb);
                atomicAdd(&Xp[p], la * lb * (la + lb));
                h = r2;
            }
        }
        __syncthreads();
        for (int p = tid; p < P; p += SG_T) {
            const u32 e2 = Ep[p];
            if (!e2 || !tb[p]) continue;
            atomicAdd(&A.accE[(size_t)p * G + g], (unsigned long long)e2);
            atomicAdd(&A.accX[(size_t)p * G + g], (unsigned long long)Xp[p]);
        }
        for (int c = tid; c < K; c += SG_T)
            if (Fc[c]) atomicAdd(&A.accF[(size_t)c * G + g], (unsigned long long)Fc[c]);
    }
    stamp(6);
    if (stm) atomicAdd(&g_seg_stamps[7], 1ull);
}

// an equality segment (one repeated value, any size): its cluster counts give
// everything in closed form (no positional pairs: S_ab gets nothing inside it)
__device__ void seg_rank_equal(const ScSegLaunch& A, SegRankLds& L)
{
    const int tid = threadIdx.x;
    const ScSeg sg = L.seg;
    const int K = A.K, G = A.G, g = sg.gene;
    for (int c = tid; c < K; c += SG_T) L.hc[c] = 0;
    __syncthreads();
    for (int e = tid; e < sg.n; e += SG_T) atomicAdd(&L.hc[A.codes2[sg.base + e]], 1u);
    __syncthreads();
    for (int idx = tid; idx < K * K; idx += SG_T) {
        const int a = idx / K, b = idx % K;
        if (a >= b) continue;
        const u64 ha = L.hc[a], hb = L.hc[b];
        if (!ha || !hb) continue;
        const int p = sg_pair(a, b, K);
        if (!sg_tested(A, p, g)) continue;
        atomicAdd(&A.accE[(size_t)p * G + g], ha * hb);
        atomicAdd(&A.accX[(size_t)p * G + g], ha * hb * (ha + hb));
    }
    for (int c = tid; c < K; c += SG_T) {
        const u64 h = L.hc[c];
        if (h >= 2) atomicAdd(&A.accF[(size_t)c * G + g], h * h * h - h);
        if (sg.hrow >= 0) A.hseg[(size_t)sg.hrow * K + c] = (u32)h;
    }
}

template <int KT>
__global__ void __launch_bounds__(SG_T) k_seg_rank(ScSegLaunch A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    SegRankLds& L = *(SegRankLds*)smem;
    constexpr int Kp = 16 * KT;
    u8* HT = (u8*)smem + ((sizeof(SegRankLds) + 15) & ~(size_t)15);
    u8* CL = HT + Kp * 32;
    u8* CH = CL + Kp * 32;
    u32* Sred = (u32*)(CH + Kp * 32);
    constexpr int NT = KT * (KT + 1) / 2;
    const int Ppad = (A.P + 1) & ~1;
    u32* Ep = Sred + NT * 256;  // per-pair tie sums of the segment
    u32* Xp = Ep + Ppad;
    u64* Fc = (u64*)(Xp + Ppad);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // wide_mode: only the segments the wave kernel passed on (key range too wide
    // for the composite key: the (key, cluster) sort below)
    const int nseg = A.wide_mode ? min(A.counts[5], A.wide_cap) : min(A.counts[0], A.seg_cap);
    for (int s = blockIdx.x; s < nseg; s += gridDim.x) {
        __syncthreads();  // the previous segment is done with the LDS
        if (tid == 0) L.seg = A.segs[A.wide_mode ? A.wide[s] : s];
        __syncthreads();
        const ScSeg sg = L.seg;
        if (sg.kind == 3) continue;  // cut into sub-segments by k_seg_refine
        if (sg.kind == 2) {
            seg_rank_equal(A, L);
            continue;
        }
        if (sg.n > SG_CAP) {  // (cannot happen for kind 0; the splitter flagged a kind-1 overflow)
            if (tid == 0) atomicOr(A.err, SCC_SEG_OVERFLOW);
            continue;
        }
        if (sg.kind == 0 && tid <= A.K) L.off[tid] = (int)A.coff[(size_t)A.cl_cc[tid] * A.G + sg.gene];
        // key range of the segment: the composite key needs (max - min) < 2^57 - 1
        u64 mn = ~0ull, mx = 0;
        const u64* src = sg.kind == 0 ? A.keys : A.keys2;
        for (int e = tid; e < sg.n; e += SG_T) {
            const u64 k = src[sg.base + e];
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const u64 a = ((u64)__shfl_xor((u32)(mn >> 32), o, 64) << 32) | __shfl_xor((u32)mn, o, 64);
            const u64 b = ((u64)__shfl_xor((u32)(mx >> 32), o, 64) << 32) | __shfl_xor((u32)mx, o, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
        }
        if (lane == 0) {
            L.kmn_w[w] = mn;
            L.kmx_w[w] = mx;
        }
        __syncthreads();
        mn = L.kmn_w[0];
        mx = L.kmx_w[0];
#pragma unroll
        for (int q = 1; q < SG_T / 64; ++q) {
            mn = L.kmn_w[q] < mn ? L.kmn_w[q] : mn;
            mx = L.kmx_w[q] > mx ? L.kmx_w[q] : mx;
        }
        if (mx - mn < (1ull << (64 - SCC_CODE_BITS)) - 1)
            seg_rank_sorted<KT, true>(A, L, HT, CL, CH, Sred, Ep, Xp, Fc, mn);
        else
            seg_rank_sorted<KT, false>(A, L, HT, CL, CH, Sred, Ep, Xp, Fc, mn);
    }
}

// ===================================================================== rank, one wave per segment
// The same counts with one wave per segment (no barriers; the 4 waves of a
// workgroup work on 4 segments): lane l holds sorted elements EPL l .. EPL l +
// EPL - 1 in registers; the bitonic stages with stride < EPL stay in the lane,
// the others are DPP / permlane lane swaps.  The tie groups are walked run to
// run (next-run positions precomputed), summed in the wave's LDS and flushed
// once.  A segment whose key range does not fit the composite key goes to the
// workgroup kernel above (its (key, cluster) sort).
struct SwLayout {
    size_t fc, ep, xp, off, hc, cs, cn, nrs, ht, cl, ch, tb, bytes;
};
__host__ __device__ inline SwLayout sw_layout(int K)
{
    const int KT = (K + 15) / 16, Kp = 16 * KT, P = K * (K - 1) / 2, Ppad = (P + 1) & ~1;
    SwLayout L;
    size_t o = 0;
    auto take = [&](size_t b, size_t al) {
        o = (o + al - 1) & ~(al - 1);
        const size_t r = o;
        o += b;
        return r;
    };
    L.fc = take(8 * (size_t)K, 8);
    L.ep = take(4 * (size_t)Ppad, 16);
    L.xp = take(4 * (size_t)Ppad, 16);
    L.off = take(4 * (size_t)(K + 1), 4);
    L.hc = take(4 * (size_t)K, 4);
    L.cs = take(SG_CAP, 16);
    L.cn = take(SG_CAP, 16);
    L.nrs = take(2 * SG_CAP, 16);
    L.ht = take(32 * (size_t)Kp, 16);
    L.cl = take(32 * (size_t)Kp, 16);
    L.ch = take(32 * (size_t)Kp, 16);
    L.tb = take((size_t)P, 16);
    L.bytes = (o + 15) & ~(size_t)15;
    return L;
}

__device__ inline u64 sw_umin(u64 a, u64 b) { return a < b ? a : b; }
__device__ inline u64 sw_shfl_xor64(u64 v, int m)
{
    return ((u64)__shfl_xor((u32)(v >> 32), m, 64) << 32) | __shfl_xor((u32)v, m, 64);
}

// bitonic sort of the wave's 64 EPL composite keys (element e = EPL lane + i).
// Levels k <= EPL stay inside the lane (directions: per register below EPL,
// bit 0 of the lane at EPL); above, the strides >= EPL are lane swaps and the
// strides < EPL register exchanges, both with lane masks from ballots (the
// masks must stay scalar: a runtime select between constant masks went to
// vector registers).
template <int EPL>
__device__ inline void sw_sort(u64 (&ck)[EPL])
{
    constexpr int M = 64 * EPL;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 2; k < EPL; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < EPL; ++i)
                if ((i & j) == 0) sgc_ce(ck[i], ck[i | j], (i & k) == 0 ? ~0ull : 0ull);
    {
        const u64 am = __ballot((lane & 1) == 0);  // k = EPL
#pragma unroll
        for (int j = EPL >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < EPL; ++i)
                if ((i & j) == 0) sgc_ce(ck[i], ck[i | j], am);
    }
    for (int k = 2 * EPL; k <= M; k <<= 1) {
        const bool asc = ((EPL * lane) & k) == 0;
        for (int d = k / (2 * EPL); d >= 1; d >>= 1) {  // strides j = d EPL >= EPL: lane distance d
            const u64 km = __ballot(((lane & d) == 0) == asc);
            switch (d) {
            case 1: sgc_lane_stage_n<1, EPL>(ck, km); break;
            case 2: sgc_lane_stage_n<2, EPL>(ck, km); break;
            case 4: sgc_lane_stage_n<4, EPL>(ck, km); break;
            case 8: sgc_lane_stage_n<8, EPL>(ck, km); break;
            case 16: sgc_lane_stage_n<16, EPL>(ck, km); break;
            default: sgc_lane_stage_n<32, EPL>(ck, km); break;
            }
        }
        const u64 am = __ballot(asc);
#pragma unroll
        for (int j = EPL >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < EPL; ++i)
                if ((i & j) == 0) sgc_ce(ck[i], ck[i | j], am);
    }
}

// an equality segment with one wave
__device__ void sw_equal(const ScSegLaunch& A, const ScSeg& sg, u32* hc)
{
    const int lane = threadIdx.x & 63, K = A.K, G = A.G, g = sg.gene;
    for (int c = lane; c < K; c += 64) hc[c] = 0;
    sg_wsync();
    for (int e = lane; e < sg.n; e += 64) atomicAdd(&hc[A.codes2[sg.base + e]], 1u);
    sg_wsync();
    for (int idx = lane; idx < K * K; idx += 64) {
        const int a = idx / K, b = idx % K;
        if (a >= b) continue;
        const u64 ha = hc[a], hb = hc[b];
        if (!ha || !hb) continue;
        const int p = sg_pair(a, b, K);
        if (!sg_tested(A, p, g)) continue;
        atomicAdd(&A.accE[(size_t)p * G + g], ha * hb);
        atomicAdd(&A.accX[(size_t)p * G + g], ha * hb * (ha + hb));
    }
    for (int c = lane; c < K; c += 64) {
        const u64 h = hc[c];
        if (h >= 2) atomicAdd(&A.accF[(size_t)c * G + g], h * h * h - h);
        if (sg.hrow >= 0) A.hseg[(size_t)sg.hrow * K + c] = (u32)h;
    }
    sg_wsync();
}

template <int KT, int EPL>
__device__ void sw_segment(const ScSegLaunch& A, const ScSeg& sg, int sidx, char* wl, const SwLayout& Y)
{
    constexpr int Kp = 16 * KT, NT = KT * (KT + 1) / 2;
    const int lane = threadIdx.x & 63, g4 = lane >> 4, r16 = lane & 15;
    const int n = sg.n, g = sg.gene, K = A.K, G = A.G, P = A.P;
    u8* cs = (u8*)(wl + Y.cs);
    u8* cn = (u8*)(wl + Y.cn);
    uint16_t* nrs = (uint16_t*)(wl + Y.nrs);
    u8* HT = (u8*)(wl + Y.ht);
    u8* CL = (u8*)(wl + Y.cl);
    u8* CH = (u8*)(wl + Y.ch);
    u8* tb = (u8*)(wl + Y.tb);
    int* off = (int*)(wl + Y.off);
    u32* Ep = (u32*)(wl + Y.ep);
    u32* Xp = (u32*)(wl + Y.xp);
    u64* Fc = (u64*)(wl + Y.fc);
    const bool stm = A.stamps && lane == 0 && (threadIdx.x >> 6) == 0;
    u64 tprev = stm ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int ph) {
        if (stm) {
            const u64 t = __builtin_amdgcn_s_memtime();
            atomicAdd(&g_seg_stamps[ph], (unsigned long long)(t - tprev));
            tprev = t;
        }
    };
    {  // the gene's tested-pair flags: P consecutive bytes of tbg
        const u8* src = A.tbg + (size_t)g * P;
        for (int p = lane; p < P; p += 64) tb[p] = src[p];
    }
    if (sg.kind == 0)
        for (int c = lane; c <= K; c += 64) off[c] = (int)A.coff[(size_t)A.cl_cc[c] * G + g];
    for (int i = lane; i < Kp * 8; i += 64) ((u32*)HT)[i] = 0;
    sg_wsync();
    // ---- load: keys and codes of elements EPL lane + i
    const int e0 = EPL * lane;
    u64 ck[EPL];
    u32 cp[EPL / 4];
    {
        const u64* src = sg.kind == 0 ? A.keys : A.keys2;
        int a = 0;
        if (sg.kind == 0 && e0 < n) {
            int lo = 0, hi = K - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (off[mid] <= e0) lo = mid; else hi = mid - 1;
            }
            a = lo;
        }
#pragma unroll
        for (int q = 0; q < EPL / 4; ++q) cp[q] = 0;
#pragma unroll
        for (int i = 0; i < EPL; ++i) {
            const int e = e0 + i;
            const int ec = e < n ? e : n - 1;  // clamped unconditional load
            const u64 k = src[sg.base + ec];
            u32 c;
            if (sg.kind == 0) {
                while (a + 1 < K && off[a + 1] <= e) ++a;
                c = (u32)a;
            } else {
                c = A.codes2[sg.base + ec];
            }
            ck[i] = e < n ? k : ~0ull;
            cp[i >> 2] |= (e < n ? c : 0u) << (8 * (i & 3));
        }
    }
    u64 mn = ~0ull, mx = 0;
#pragma unroll
    for (int i = 0; i < EPL; ++i)
        if (e0 + i < n) {
            mn = ck[i] < mn ? ck[i] : mn;
            mx = ck[i] > mx ? ck[i] : mx;
        }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const u64 a = sw_shfl_xor64(mn, o), b = sw_shfl_xor64(mx, o);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if (mx - mn >= (1ull << (64 - SCC_CODE_BITS)) - 1) {  // too wide for the composite key: the workgroup kernel
        if (lane == 0) {
            const int o = atomicAdd(&A.counts[5], 1);
            if (o < A.wide_cap) A.wide[o] = sidx; else atomicOr(A.err, SCC_SEG_OVERFLOW);
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < EPL; ++i)
        ck[i] = e0 + i < n ? (((ck[i] - mn) << SCC_CODE_BITS) | ((cp[i >> 2] >> (8 * (i & 3))) & 0xffu)) : ~0ull;
    stamp(0);
    if (!(A.dbg & 1)) sw_sort<EPL>(ck);
    stamp(1);
    // ---- codes to LDS (block slot order, and natural order for the ties); tie test
    const int nq = (n + 63) >> 6;
    bool tie = false;
    const u64 nxt0 = sw_shfl_down64(ck[0], 1);  // the next lane's first element
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
        const int e = e0 + i;
        const u32 c = e < n ? (u32)(ck[i] & SCC_CODE_MASK) : 0xffu;
        if (e < nq * 64) cs[(e & ~63) + sg_slot(e & 63)] = (u8)c;
        if (e < n) cn[e] = (u8)c;
        const u64 nx = i + 1 < EPL ? ck[i + 1 < EPL ? i + 1 : 0] : nxt0;
        tie |= (e + 1 < n) && ((nx >> SCC_CODE_BITS) == (ck[i] >> SCC_CODE_BITS));
    }
    const bool any_tie = __ballot(tie) != 0;
    stamp(2);
    // ---- tie groups: runs (equal key and cluster) inside groups (equal key),
    // walked run to run from the next-run positions
    if (any_tie && !(A.dbg & 4)) {
        const u64 prv = sw_shfl_up64(ck[EPL - 1], 1);  // the previous lane's last element
        u32 rsm = 0, gsm = 0;  // run / group starts of this lane's elements (bit i)
#pragma unroll
        for (int i = 0; i < EPL; ++i) {
            const int e = e0 + i;
            const u64 pv = i > 0 ? ck[i > 0 ? i - 1 : 0] : prv;
            const bool gs = e == 0 || (pv >> SCC_CODE_BITS) != (ck[i] >> SCC_CODE_BITS);
            const bool rs = gs || (pv & SCC_CODE_MASK) != (ck[i] & SCC_CODE_MASK);
            if (e < n) {
                gsm |= (gs ? 1u : 0u) << i;
                rsm |= (rs ? 1u : 0u) << i;
            }
        }
        // first run / group start of each lane, then the nearest one in a later lane
        u32 frs = rsm ? (u32)(e0 + __builtin_ctz(rsm)) : 0xffffu, fgs = gsm ? (u32)(e0 + __builtin_ctz(gsm)) : 0xffffu;
        u32 nr = (u32)__shfl_down((int)frs, 1, 64), ng = (u32)__shfl_down((int)fgs, 1, 64);
        if (lane == 63) nr = ng = 0xffffu;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {  // suffix minimum over the later lanes
            const u32 a = (u32)__shfl_down((int)nr, o, 64), b = (u32)__shfl_down((int)ng, o, 64);
            if (lane + o < 64) {
                nr = a < nr ? a : nr;
                ng = b < ng ? b : ng;
            }
        }
        if (nr > (u32)n) nr = (u32)n;
        if (ng > (u32)n) ng = (u32)n;
        // backwards over the lane: next run start (nrs) and group end of each run start
        u32 gend[EPL];
#pragma unroll
        for (int i = EPL - 1; i >= 0; --i) {
            gend[i] = ng;
            if ((rsm >> i) & 1u) {
                nrs[e0 + i] = (uint16_t)nr;
                nr = (u32)(e0 + i);
            }
            if ((gsm >> i) & 1u) ng = (u32)(e0 + i);
        }
        sg_wsync();
#pragma unroll
        for (int i = 0; i < EPL; ++i) {
            if (!((rsm >> i) & 1u)) continue;
            const int e = e0 + i;
            const u32 c = (u32)(ck[i] & SCC_CODE_MASK);
            const u32 t = (u32)nrs[e] - (u32)e;
            if (t >= 2) atomicAdd(&Fc[c], (u64)t * t * t - t);
            for (u32 r = (u32)e + t; r < gend[i];) {  // the later runs of the group
                const u32 c2 = cn[r], t2 = (u32)nrs[r] - r;
                const int p = sg_pair((int)c, (int)c2, K);
                // (a segment holds <= SG_CAP = 2^10 values: E <= 2^20 and X <= 2^31 fit 32 bits)
                atomicAdd(&Ep[p], t * t2);
                atomicAdd(&Xp[p], t * t2 * (t + t2));
                r += t2;
            }
        }
        sg_wsync();
        for (int p = lane; p < P; p += 64) {
            const u32 e2 = Ep[p], x2 = Xp[p];
            if (e2) {
                if (tb[p]) {
                    atomicAdd(&A.accE[(size_t)p * G + g], (unsigned long long)e2);
                    atomicAdd(&A.accX[(size_t)p * G + g], (unsigned long long)x2);
                }
                Ep[p] = 0;
                Xp[p] = 0;
            }
        }
        for (int c = lane; c < K; c += 64)
            if (Fc[c]) {
                atomicAdd(&A.accF[(size_t)c * G + g], (unsigned long long)Fc[c]);
                Fc[c] = 0;
            }
    }
    stamp(6);
    // ---- blocks: M = L O and S += O^T M per 64-element block
    sg_v4i Lm[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int d = 0; d < 4; ++d) Lm[mt][d] = (int)sg_lt_bytes(16 * mt + r16, 16 * d + 4 * g4);
    const sg_v4i zero = {0, 0, 0, 0};
    sg_v4i S[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) S[q] = zero;
    for (int q = 0; q < ((A.dbg & 2) ? 0 : nq); ++q) {
        const uint4 cw = *(const uint4*)&cs[64 * q + 16 * g4];
        sg_v4i Ob[KT];
#pragma unroll
        for (int u = 0; u < KT; ++u) {
            const u32 c = (u32)(16 * u + r16);
            Ob[u] = sg_v4i{(int)sg_eq_bytes(cw.x, c), (int)sg_eq_bytes(cw.y, c), (int)sg_eq_bytes(cw.z, c),
                           (int)sg_eq_bytes(cw.w, c)};
        }
#pragma unroll
        for (int u = 0; u < KT; ++u) {
            const sg_v4i m0 = sg_mfma(Lm[0], Ob[u], zero);
            const sg_v4i m1 = sg_mfma(Lm[1], Ob[u], zero);
            const sg_v4i m2 = sg_mfma(Lm[2], Ob[u], zero);
            const sg_v4i m3 = sg_mfma(Lm[3], Ob[u], zero);
            if (g4 == 3) {  // H[q][b] = M[63][b] + [code of element 63 == b]
                const int b = 16 * u + r16;
                HT[b * 32 + q] = (u8)(m3[3] + (((cw.w >> 24) & 0xffu) == (u32)b ? 1 : 0));
            }
            const sg_v4i Mb = {(int)sg_pack(m0), (int)sg_pack(m1), (int)sg_pack(m2), (int)sg_pack(m3)};
#pragma unroll
            for (int u0 = 0; u0 <= u; ++u0) S[sg_tile<KT>(u0, u)] = sg_mfma(Ob[u0], Mb, S[sg_tile<KT>(u0, u)]);
        }
    }
    sg_wsync();
    stamp(3);
    // ---- the blocks' exclusive prefix per cluster (6-bit halves), the segment's counts
    for (int c = lane; c < Kp; c += 64) {
        u32 run = 0;
#pragma unroll 8
        for (int q = 0; q < 32; ++q) {
            const u32 h = HT[c * 32 + q];
            CL[c * 32 + q] = (u8)(run & 63u);
            CH[c * 32 + q] = (u8)(run >> 6);
            run += h;
        }
        if (sg.hrow >= 0 && c < K) A.hseg[(size_t)sg.hrow * K + c] = run;
    }
    sg_wsync();
    // ---- cross-block part H^T Cex
#pragma unroll
    for (int u0 = 0; u0 < KT; ++u0)
#pragma unroll
        for (int u1 = u0; u1 < KT; ++u1) {
            const int ti = sg_tile<KT>(u0, u1);
            sg_v4i a = zero, bl = zero, bh = zero;
            if (g4 < 2) {
                const uint4 x = *(const uint4*)&HT[(16 * u0 + r16) * 32 + 16 * g4];
                const uint4 y = *(const uint4*)&CL[(16 * u1 + r16) * 32 + 16 * g4];
                const uint4 z = *(const uint4*)&CH[(16 * u1 + r16) * 32 + 16 * g4];
                a = sg_v4i{(int)x.x, (int)x.y, (int)x.z, (int)x.w};
                bl = sg_v4i{(int)y.x, (int)y.y, (int)y.z, (int)y.w};
                bh = sg_v4i{(int)z.x, (int)z.y, (int)z.z, (int)z.w};
            }
            const sg_v4i hi = sg_mfma(a, bh, zero);
            sg_v4i s2 = sg_mfma(a, bl, S[ti]);
#pragma unroll
            for (int r = 0; r < 4; ++r) s2[r] += hi[r] << 6;
            S[ti] = s2;
        }
    stamp(4);
    // ---- flush from the accumulators: one integer atomic per tested pair with a nonzero count
#pragma unroll
    for (int u0 = 0; u0 < KT; ++u0)
#pragma unroll
        for (int u1 = u0; u1 < KT; ++u1) {
            const int ti = sg_tile<KT>(u0, u1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int a = 16 * u0 + 4 * g4 + r, b = 16 * u1 + r16;
                const u32 x = (u32)S[ti][r];
                if (a < b && b < K && x) {
                    const int p = sg_pair(a, b, K);
                    if (tb[p]) atomicAdd(&A.accS[(size_t)p * G + g], (unsigned long long)x);
                }
            }
        }
    sg_wsync();
    stamp(5);
    if (stm) atomicAdd(&g_seg_stamps[7], 1ull);
}

template <int KT>
__global__ void __launch_bounds__(256) k_seg_wave(ScSegLaunch A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = scc_wave_id(), wpg = blockDim.x >> 6;
    const SwLayout Y = sw_layout(A.K);
    char* wl = smem + (size_t)w * Y.bytes;
    {  // the tie sums start at zero (each flush zeroes what it read)
        u32* Ep = (u32*)(wl + Y.ep);
        u32* Xp = (u32*)(wl + Y.xp);
        u64* Fc = (u64*)(wl + Y.fc);
        for (int p = lane; p < A.P; p += 64) Ep[p] = Xp[p] = 0;
        for (int c = lane; c < A.K; c += 64) Fc[c] = 0;
        sg_wsync();
    }
    const int nseg = min(A.counts[0], A.seg_cap);
    for (int s = blockIdx.x * wpg + w; s < nseg; s += gridDim.x * wpg) {
        // the descriptor, wave-uniform (scalar registers: uniform branches below)
        const ScSeg sv = A.segs[s];
        ScSeg sg;
        sg.base = (long long)(((u64)(u32)__builtin_amdgcn_readfirstlane((int)((u64)sv.base >> 32)) << 32) |
                              (u32)__builtin_amdgcn_readfirstlane((int)(u32)(u64)sv.base));
        sg.n = __builtin_amdgcn_readfirstlane(sv.n);
        sg.gene = __builtin_amdgcn_readfirstlane(sv.gene);
        sg.kind = __builtin_amdgcn_readfirstlane(sv.kind);
        sg.hrow = __builtin_amdgcn_readfirstlane(sv.hrow);
        if (sg.kind == 3) continue;  // cut into sub-segments by k_seg_refine
        if (sg.kind == 2) {
            sw_equal(A, sg, (u32*)(wl + Y.hc));
            continue;
        }
        if (sg.n > SG_CAP) {
            if (lane == 0) atomicOr(A.err, SCC_SEG_OVERFLOW);
            continue;
        }
        if (sg.n <= 512)
            sw_segment<KT, 8>(A, sg, s, wl, Y);
        else
            sw_segment<KT, 16>(A, sg, s, wl, Y);
    }
}

// ===================================================================== refine
// An interval segment the splitter left with more than SG_CAP elements: one
// 1024-thread workgroup sorts it by key in LDS (<= REF_CAP elements), writes it
// back in order, cuts it into sub-segments of <= SG_CAP at value changes (a run
// of one value longer than SG_CAP becomes an equality sub-segment), adds the
// cross-sub-segment part of S itself, and writes the parent's cluster counts
// (its hseg row).  The parent becomes kind 3 (k_seg_rank skips it).
#define REF_T 1024
#define REF_CAP 8192
#define REF_SUBS 64

struct RefLds {
    u64 k[REF_CAP];
    u8 c[REF_CAP];
    u32 h[REF_SUBS][SCC_MAX_K];
    int cut[REF_SUBS + 1];
    int nsub, idx;
    ScSeg seg;
};
static_assert(sizeof(RefLds) <= 160 * 1024, "refine LDS");

__global__ void __launch_bounds__(REF_T) k_seg_refine(ScSegLaunch A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    RefLds& L = *(RefLds*)smem;
    const int tid = threadIdx.x, K = A.K, G = A.G, P = A.P;
    const int novf = A.counts[4];
    for (int oi = blockIdx.x; oi < min(novf, A.ovf_cap); oi += gridDim.x) {
        __syncthreads();
        if (tid == 0) {
            L.idx = A.ovf[oi];
            L.seg = A.segs[L.idx];
        }
        __syncthreads();
        const ScSeg sg = L.seg;
        const int n = sg.n, g = sg.gene;
        if (n > REF_CAP) {
            if (tid == 0) atomicOr(A.err, SCC_SEG_OVERFLOW);
            continue;
        }
        int M = 64;
        while (M < n) M <<= 1;
        for (int e = tid; e < M; e += REF_T) {
            L.k[e] = e < n ? A.keys2[sg.base + e] : ~0ull;
            L.c[e] = e < n ? A.codes2[sg.base + e] : (u8)0;
        }
        __syncthreads();
        for (int k = 2; k <= M; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int e = tid; e < M / 2; e += REF_T) {
                    const int i = 2 * j * (e / j) + (e % j), q = i + j;
                    const u64 a = L.k[i], b = L.k[q];
                    const bool asc = (i & k) == 0;
                    if (asc ? (b < a) : (a < b)) {
                        const u8 ca = L.c[i];
                        L.k[i] = b;
                        L.k[q] = a;
                        L.c[i] = L.c[q];
                        L.c[q] = ca;
                    }
                }
                __syncthreads();
            }
        for (int e = tid; e < n; e += REF_T) {
            A.keys2[sg.base + e] = L.k[e];
            A.codes2[sg.base + e] = L.c[e];
        }
        // cuts (one thread: overflows are rare): sub-segments of <= SG_CAP ending
        // at a change of value; a longer run of one value stands alone
        if (tid == 0) {
            int ns = 0, st = 0;
            L.cut[0] = 0;
            while (st < n && ns < REF_SUBS) {
                int en = min(n, st + SG_CAP);
                if (en < n)
                    while (en > st && L.k[en - 1] == L.k[en]) --en;
                if (en == st) {  // one value over more than SG_CAP elements
                    en = st;
                    while (en < n && L.k[en] == L.k[st]) ++en;
                }
                L.cut[++ns] = en;
                st = en;
            }
            L.nsub = st < n ? -1 : ns;
        }
        __syncthreads();
        const int ns = L.nsub;
        if (ns < 0) {
            if (tid == 0) atomicOr(A.err, SCC_SEG_OVERFLOW);
            continue;
        }
        for (int i = tid; i < ns * SCC_MAX_K; i += REF_T) L.h[i / SCC_MAX_K][i % SCC_MAX_K] = 0;
        __syncthreads();
        for (int q = 0; q < ns; ++q)
            for (int e = L.cut[q] + tid; e < L.cut[q + 1]; e += REF_T) atomicAdd(&L.h[q][L.c[e]], 1u);
        __syncthreads();
        if (tid < ns) {  // the sub-segments (no hseg row: the parent keeps its own)
            const int a0 = L.cut[tid], a1 = L.cut[tid + 1];
            const bool one = L.k[a0] == L.k[a1 - 1];
            const int s = atomicAdd(&A.counts[0], 1);
            if (s < A.seg_cap)
                A.segs[s] = ScSeg{sg.base + a0, a1 - a0, g, (one && a1 - a0 > SG_CAP) ? 2 : 1, -1};
            else
                atomicOr(A.err, SCC_SEG_OVERFLOW);
        }
        if (tid == 0) A.segs[L.idx].kind = 3;
        for (int c = tid; c < K; c += REF_T) {  // the parent's cluster counts
            u32 t = 0;
            for (int q = 0; q < ns; ++q) t += L.h[q][c];
            if (sg.hrow >= 0) A.hseg[(size_t)sg.hrow * K + c] = t;
        }
        // S across the sub-segments: sum_q h_q[a] * (b-elements of earlier subs)
        for (int p = tid; p < P; p += REF_T) {
            if (!sg_tested(A, p, g)) continue;
            int a = 0, rem = p;
            while (rem >= K - 1 - a) {
                rem -= K - 1 - a;
                ++a;
            }
            const int b = a + 1 + rem;
            u64 acc = 0, run = 0;
            for (int q = 0; q < ns; ++q) {
                acc += (u64)L.h[q][a] * run;
                run += L.h[q][b];
            }
            if (acc) atomicAdd(&A.accS[(size_t)p * G + g], (unsigned long long)acc);
        }
    }
}

// ===================================================================== cross
// S_ab += sum over the gene's segments (value order) of hseg[s][a] * (b-elements
// of the segments before s)
__global__ void __launch_bounds__(256) k_seg_cross(ScSegLaunch A)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    u32* hs = (u32*)smem;
    const int K = A.K, G = A.G, P = A.P;
    const int nbig = A.counts[1];
    for (int bi = blockIdx.x; bi < nbig; bi += gridDim.x) {
        const int4 gs = A.gseg[bi];
        const int h0 = gs.x, ns = gs.y, g = gs.z;
        const bool in_lds = (size_t)ns * K * 4 <= A.cross_lds;
        __syncthreads();
        if (in_lds)
            for (int i = threadIdx.x; i < ns * K; i += blockDim.x) hs[i] = A.hseg[(size_t)h0 * K + i];
        __syncthreads();
        const u32* H = in_lds ? hs : A.hseg + (size_t)h0 * K;
        for (int p = threadIdx.x; p < P; p += blockDim.x) {
            if (!sg_tested(A, p, g)) continue;
            int a = 0, rem = p;
            while (rem >= K - 1 - a) {
                rem -= K - 1 - a;
                ++a;
            }
            const int b = a + 1 + rem;
            u64 acc = 0, run = 0;
            for (int s = 0; s < ns; ++s) {
                acc += (u64)H[(size_t)s * K + a] * run;
                run += H[(size_t)s * K + b];
            }
            if (acc) atomicAdd(&A.accS[(size_t)p * G + g], (unsigned long long)acc);
        }
    }
}

// ===================================================================== host
extern "C" size_t scc_seg_rank_lds(int K)
{
    const int KT = (K + 15) / 16, P = K * (K - 1) / 2, Ppad = (P + 1) & ~1;
    return ((sizeof(SegRankLds) + 15) & ~(size_t)15) + 3 * (size_t)(16 * KT) * 32 +
           (size_t)KT * (KT + 1) / 2 * 256 * 4 + 2 * (size_t)Ppad * 4 + (size_t)K * 8 + (size_t)P + 16;
}

template <int KT>
static hipError_t launch_rank(const ScSegLaunch* L, int ncu, hipStream_t st)
{
    const size_t lds = scc_seg_rank_lds(L->K);
    static bool attr = false;  // (one attribute call per instantiation and process: the largest K of the tile count)
    if (!attr) {
        scc_set_lds((const void*)k_seg_rank<KT>, (int)scc_seg_rank_lds(16 * KT));
        attr = true;
    }
    const int per_cu = std::max(1, std::min(4, (int)((160 * 1024) / std::max<size_t>(lds, 1))));
    hipLaunchKernelGGL(k_seg_rank<KT>, dim3(per_cu * ncu), dim3(SG_T), lds, st, *L);
    return hipGetLastError();
}

template <int KT>
static hipError_t launch_wave(const ScSegLaunch* L, int ncu, hipStream_t st)
{
    static bool attr = false;
    if (!attr) {
        scc_set_lds((const void*)k_seg_wave<KT>, 160 * 1024);
        attr = true;
    }
    const size_t wb = sw_layout(L->K).bytes;
    // waves per workgroup: the most resident waves per CU under the LDS budget
    int best_w = 1, best_n = 0;
    for (int wpg : {4, 2, 1}) {
        const int per_cu = std::min(8, (int)((160 * 1024) / (wpg * wb)));
        if (per_cu * wpg > best_n) {
            best_n = per_cu * wpg;
            best_w = wpg;
        }
    }
    const int per_cu = std::max(1, best_n / best_w);
    hipLaunchKernelGGL(k_seg_wave<KT>, dim3(per_cu * ncu), dim3(64 * best_w), best_w * wb, st, *L);
    return hipGetLastError();
}

hipError_t scc_launch_seg_rank(const ScSegLaunch* L, int ncu, hipStream_t st)
{
    if (L->G <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_seg_classify, dim3((L->G + 255) / 256), dim3(256), 0, st, *L);
    hipLaunchKernelGGL(k_seg_flags_t, dim3((L->G + 31) / 32, (L->P + 31) / 32), dim3(256), 0, st, *L);
    static bool attr = false;
    if (!attr) {
        scc_set_lds((const void*)k_seg_split, (int)sizeof(Sp2Lds));
        scc_set_lds((const void*)k_seg_cross, 64 * 1024);
        scc_set_lds((const void*)k_seg_refine, (int)sizeof(RefLds));
        attr = true;
    }
    hipLaunchKernelGGL(k_seg_split, dim3(ncu), dim3(SP2_T), sizeof(Sp2Lds), st, *L);
    hipLaunchKernelGGL(k_seg_refine, dim3(64), dim3(REF_T), sizeof(RefLds), st, *L);
    hipError_t e;
    switch ((L->K + 15) / 16) {
    case 1: e = launch_wave<1>(L, ncu, st); break;
    case 2: e = launch_wave<2>(L, ncu, st); break;
    case 3: e = launch_wave<3>(L, ncu, st); break;
    case 4: e = launch_wave<4>(L, ncu, st); break;
    case 5: e = launch_wave<5>(L, ncu, st); break;
    case 6: e = launch_wave<6>(L, ncu, st); break;
    case 7: e = launch_wave<7>(L, ncu, st); break;
    default: e = launch_wave<8>(L, ncu, st); break;
    }
    if (e != hipSuccess) return e;
    ScSegLaunch W = *L;  // the wide-range segments the wave kernel passed on
    W.wide_mode = 1;
    switch ((L->K + 15) / 16) {
    case 1: e = launch_rank<1>(&W, ncu, st); break;
    case 2: e = launch_rank<2>(&W, ncu, st); break;
    case 3: e = launch_rank<3>(&W, ncu, st); break;
    case 4: e = launch_rank<4>(&W, ncu, st); break;
    case 5: e = launch_rank<5>(&W, ncu, st); break;
    case 6: e = launch_rank<6>(&W, ncu, st); break;
    case 7: e = launch_rank<7>(&W, ncu, st); break;
    default: e = launch_rank<8>(&W, ncu, st); break;
    }
    if (e != hipSuccess) return e;
    ScSegLaunch C = *L;
    C.cross_lds = 64 * 1024;
    hipLaunchKernelGGL(k_seg_cross, dim3(2 * ncu), dim3(256), 64 * 1024, st, C);
    return hipGetLastError();
}

extern "C" void scc_seg_stamps(hipStream_t st, int print)
{
    unsigned long long h[8];
    if (print) {
        (void)hipStreamSynchronize(st);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_seg_stamps), sizeof(h), 0, hipMemcpyDeviceToHost);
        const double ns = (double)(h[7] ? h[7] : 1);
        fprintf(stderr, "[scc seg stamps] %llu sorted segments, mean cycles: load %.0f sort %.0f codes %.0f blocks %.0f "
                "prefix %.0f flush %.0f ties %.0f\n", h[7], h[0] / ns, h[1] / ns, h[2] / ns, h[3] / ns, h[4] / ns,
                h[5] / ns, h[6] / ns);
    }
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_seg_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice, st);
    (void)hipStreamSynchronize(st);
}
