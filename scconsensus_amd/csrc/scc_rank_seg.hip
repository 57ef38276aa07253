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

#define SG_T 256
#define SG_KPT (SG_CAP / SG_T)  // elements per thread in the sort (8)
#define SG_QMAX (SG_CAP / 64)   // blocks per segment (32)
#define SP2_T 1024              // splitter workgroup
#define SP2_SMAX 4096           // sample keys sorted in LDS
#define SP2_MMAX 1023           // distinct splitters (<= 2047 segments per gene)
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
    const int s = min(n, min(SP2_SMAX, 32 * nseg));
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
        // an interval segment larger than a workgroup's sort: the run falls back
        // to the bucket engine (equality segments take any size)
        if (h0 > SG_CAP) atomicOr(A.err, SCC_SEG_OVERFLOW);
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
template <>
struct SgEl<true> {
    u64 k;
    __device__ bool lt(const SgEl& o) const { return k < o.k; }
};
template <>
struct SgEl<false> {
    u64 k;
    u32 c;
    __device__ bool lt(const SgEl& o) const { return k < o.k || (k == o.k && c < o.c); }
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
    const SgEl<C> x = sw ? b : a, y = sw ? a : b;
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
        v[i] = take ? p : v[i];
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
                    v[i] = take ? p : v[i];
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

// one segment of n <= SG_CAP elements (kind 0 / 1): sort, blocks, cross-block
// part, flush, ties, the segment's cluster counts
template <int KT, bool C>
__device__ void seg_rank_sorted(const ScSegLaunch& A, SegRankLds& L, u8* HT, u8* CL, u8* CH, u32* Sred,
                                const u64 kmn)
{
    constexpr int Kp = 16 * KT, NT = KT * (KT + 1) / 2;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g4 = lane >> 4, r16 = lane & 15;
    const ScSeg sg = L.seg;
    const int n = sg.n, g = sg.gene, K = A.K, G = A.G;
    int M = 64;
    while (M < n) M <<= 1;
    const bool active = 512 * w < M;
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
    sg_sort<C>(v, M, L, active);
    __syncthreads();  // every LDS stage read is done before sk is rewritten
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
    for (int q = w; q < nq; q += SG_T / 64) {
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
            if ((ti & 3) != w) continue;
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
    // ---- flush: one integer atomic per tested pair with a nonzero count
    for (int idx = tid; idx < Kp * Kp; idx += SG_T) {
        const int a = idx / Kp, b = idx % Kp;
        if (a >= b || b >= K) continue;
        const u32 x = Sred[sg_tile<KT>(a >> 4, b >> 4) * 256 + (a & 15) * 16 + (b & 15)];
        if (!x) continue;
        const int p = sg_pair(a, b, K);
        if (sg_tested(A, p, g)) atomicAdd(&A.accS[(size_t)p * G + g], (unsigned long long)x);
    }
    // ---- tie groups (rare): F from runs, E and X from pairs of runs
    if (L.any_tie) {
        auto kp = [&](int e) -> u64 {
            if constexpr (C) return L.sk[e] >> SCC_CODE_BITS; else return L.sk[e];
        };
        for (int e = tid; e < n; e += SG_T) {
            const u64 k0 = kp(e);
            if (e + 1 >= n || kp(e + 1) != k0 || (e > 0 && kp(e - 1) == k0)) continue;
            int f = e;
            while (f < n && kp(f) == k0) {  // runs of one cluster, clusters ascending
                const int c = L.cn[f];
                int r1 = f;
                while (r1 < n && kp(r1) == k0 && L.cn[r1] == c) ++r1;
                const u64 la = (u64)(r1 - f);
                if (la >= 2) atomicAdd(&A.accF[(size_t)c * G + g], la * la * la - la);
                int h = r1;
                while (h < n && kp(h) == k0) {
                    const int c2 = L.cn[h];
                    int r2 = h;
                    while (r2 < n && kp(r2) == k0 && L.cn[r2] == c2) ++r2;
                    const u64 lb = (u64)(r2 - h);
                    const int p = sg_pair(c, c2, K);
                    if (sg_tested(A, p, g)) {
                        atomicAdd(&A.accE[(size_t)p * G + g], la * lb);
                        atomicAdd(&A.accX[(size_t)p * G + g], la * lb * (la + lb));
                    }
                    h = r2;
                }
                f = r1;
            }
        }
    }
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
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nseg = min(A.counts[0], A.seg_cap);
    for (int s = blockIdx.x; s < nseg; s += gridDim.x) {
        __syncthreads();  // the previous segment is done with the LDS
        if (tid == 0) L.seg = A.segs[s];
        __syncthreads();
        const ScSeg sg = L.seg;
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
            seg_rank_sorted<KT, true>(A, L, HT, CL, CH, Sred, mn);
        else
            seg_rank_sorted<KT, false>(A, L, HT, CL, CH, Sred, mn);
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
    const int KT = (K + 15) / 16;
    return ((sizeof(SegRankLds) + 15) & ~(size_t)15) + 3 * (size_t)(16 * KT) * 32 + (size_t)KT * (KT + 1) / 2 * 256 * 4;
}

template <int KT>
static hipError_t launch_rank(const ScSegLaunch* L, int ncu, hipStream_t st)
{
    const size_t lds = scc_seg_rank_lds(16 * KT);
    static bool attr = false;  // (one attribute call per instantiation and process)
    if (!attr) {
        hipFuncSetAttribute((const void*)k_seg_rank<KT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    const int per_cu = std::max(1, std::min(4, (int)((160 * 1024) / std::max<size_t>(lds, 1))));
    hipLaunchKernelGGL(k_seg_rank<KT>, dim3(per_cu * ncu), dim3(SG_T), lds, st, *L);
    return hipGetLastError();
}

hipError_t scc_launch_seg_rank(const ScSegLaunch* L, int ncu, hipStream_t st)
{
    if (L->G <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_seg_classify, dim3((L->G + 255) / 256), dim3(256), 0, st, *L);
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_seg_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(Sp2Lds));
        hipFuncSetAttribute((const void*)k_seg_cross, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_seg_split, dim3(ncu), dim3(SP2_T), sizeof(Sp2Lds), st, *L);
    hipError_t e;
    switch ((L->K + 15) / 16) {
    case 1: e = launch_rank<1>(L, ncu, st); break;
    case 2: e = launch_rank<2>(L, ncu, st); break;
    case 3: e = launch_rank<3>(L, ncu, st); break;
    case 4: e = launch_rank<4>(L, ncu, st); break;
    case 5: e = launch_rank<5>(L, ncu, st); break;
    case 6: e = launch_rank<6>(L, ncu, st); break;
    case 7: e = launch_rank<7>(L, ncu, st); break;
    default: e = launch_rank<8>(L, ncu, st); break;
    }
    if (e != hipSuccess) return e;
    ScSegLaunch C = *L;
    C.cross_lds = 64 * 1024;
    hipLaunchKernelGGL(k_seg_cross, dim3(2 * ncu), dim3(256), 64 * 1024, st, C);
    return hipGetLastError();
}
