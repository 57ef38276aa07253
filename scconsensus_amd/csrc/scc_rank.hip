// scc_rank.hip — per-gene Wilcoxon rank-sum engine (all cluster pairs at once).
//
// Replaces, for every gene and every cluster pair (i<j) simultaneously, the
// reference's per-(pair, gene) `wilcox.test(data.use[x, ] ~ group)` call
// (R/reclusterDEConsensusFast.R:78-91; R/reclusterDEConsensus.R:99-103) and the
// per-pair log-mean/pct statistics (Fast:229-271, slow:104-113).
//
// One workgroup per gene.  The ingest leaves each gene's kept nonzeros
// grouped by cluster (cluster a at [off_a, off_a+1) of the segment), so:
//   1. per-cluster statistics (dd sums of x and expm1(x), counts of x > 0 /
//      x < 0) are contiguous reductions over <= K + W balanced pieces
//   2. the segment is sorted by value with a stable LSD radix sort of an index
//      permutation (8-bit digits, wave match-ranking, no compare network) on a
//      32-bit window of the orderable key: bits [sh, sh+32) of key - kmin.
//      Equal windows with different doubles ("mixed runs", values closer than
//      2^-28 relative) are re-sorted exactly by one wave each; if any is
//      longer than 64 the gene is re-sorted on all bits.  Stability keeps
//      equal values in cluster order, which the sweep relies on.
//   3. one sweep per wave chunk (register accumulators): S[a][b] = #{b before
//      an a-element}; with ties ordered by code, for a < b this is exactly
//      #{(x in a, y in b): x > y}.  The same sweep counts, per tie group,
//      E_ab = c_a c_b, X_ab = c_a c_b (c_a + c_b) and F_a = sum c_a^3 - c_a
//   5. per pair:  2U = 2*(S + z_a*neg_b + pos_a*z_b) + z_a*z_b + E_ab
//                 T  = F_a + F_b + 3*z_a*z_b*(z_a+z_b) + 3*X_ab
//      where z = implicit zeros of the cluster; T = sum(NTIES^3 - NTIES).
// 2U and T are exact int64 — R's W = 2U/2 and its tie term bit for bit.
// Genes too large for LDS keep their index arrays in HBM (same code).
#include "scc_common.hpp"
#include "scc_kernels.hpp"
#include <type_traits>

__device__ inline u64 f_tie(u64 c) { return c * c * c - c; }

__device__ inline void pair_decode(int p, int K, int& a, int& b)
{
    a = 0;
    int rem = p;
    while (rem >= K - 1 - a) {
        rem -= K - 1 - a;
        ++a;
    }
    b = a + 1 + rem;
}

__device__ inline u32 lanes_below(u64 m)  // popcount of m over lanes < this lane
{
    return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
}

__device__ inline u64 shfl_xor_u64(u64 v, int m)
{
    const u32 lo = __shfl_xor((u32)v, m, 64), hi = __shfl_xor((u32)(v >> 32), m, 64);
    return ((u64)hi << 32) | lo;
}

struct RankArgs {
    const int* gene_list;
    const int* list_count;
    const i64* gstart;   // [G+1] gene segment starts
    const u64* keys;     // kept nonzeros' value keys, cluster-grouped per gene
    int G, K, P;
    const int* n_clu;    // kept cells per cluster
    const u32* coff;     // [nc+1][G] per-gene offsets of the count chunks
    const int* cl_cc;    // [K+1] first count chunk of each cluster
    double* mean_x;      // [K][G]
    double* mean_e;      // [K][G]
    u32* cnt_pos;        // [K][G]
    i64* u2_base;        // [P][G]
    i64* t_base;         // [P][G]
    u32* gix;            // [2][nnz] index ping-pong of HBM-resident genes
    u8* guc;             // [nnz] code by segment position (HBM-resident genes)
    u8* gsc;             // [nnz] sorted codes (HBM-resident genes)
    i64 nnz;
    u64* stamps;         // diagnostic phase clocks [block][8] (nullptr in normal runs)
};

#define STAMP(A, ph)                                                                      \
    do {                                                                                  \
        if ((A).stamps && threadIdx.x == 0)                                               \
            (A).stamps[(size_t)blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memtime();    \
    } while (0)

#define RK_RUNS 256  // mixed-run list capacity

struct StatItem {
    double sx_hi, sx_lo, se_hi, se_lo;
    u64 kmin, kmax;
    u32 pos, neg;
};

// small per-block LDS state (both variants)
template <int T>
struct RankSmall {
    static constexpr int W = T / 64;
    u32 hist[W * 256];
    u32 dtot[256 + W];
    u32 whist[W * 64];
    u32 posc[64], negc[64];
    u64 F[64];
    int off[65];
    StatItem item[64 + W];
    int run_s[RK_RUNS], run_l[RK_RUNS];
    int nruns, flag, redo, pad;
    u64 kmin, kmax;
};

// One stable LSD pass on digit (key[id] - kmin) >> shift & 255: in -> out.
// Each wave owns a contiguous range; per-(wave, digit) offsets; inside a
// 64-element tile, equal digits are ranked by lane order (match by ballots).
template <int T, class KP, class IX>
__device__ void radix_pass(KP key, u64 kmin, int shift, const IX* in, IX* out, int n, RankSmall<T>& L)
{
    constexpr int W = T / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    const int R = (((n + W - 1) / W) + 63) & ~63;
    const int lo = min(n, w * R), hi = min(n, lo + R);
    u32* hw = L.hist + w * 256;
    for (int d = lane; d < 256; d += 64) hw[d] = 0;
    for (int i = lo + lane; i < hi; i += 64) {
        const u32 d = (u32)((key[in[i]] - kmin) >> shift) & 255u;
        atomicAdd(&hw[d], 1u);
    }
    __syncthreads();
    u32 tot = 0, incl = 0;
    if (tid < 256) {
        u32 s = 0;
        for (int v = 0; v < W; ++v) {
            const u32 c = L.hist[v * 256 + tid];
            L.hist[v * 256 + tid] = s;
            s += c;
        }
        tot = s;
        incl = s;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) L.dtot[256 + w] = incl;
    }
    __syncthreads();
    if (tid < 256) {
        u32 base = incl - tot;
        for (int v = 0; v < w; ++v) base += L.dtot[256 + v];
        for (int v = 0; v < W; ++v) L.hist[v * 256 + tid] += base;
    }
    __syncthreads();
    for (int i0 = lo; i0 < hi; i0 += 64) {
        const int i = i0 + lane;
        const bool ok = i < hi;
        const IX id = ok ? in[i] : (IX)0;
        const u32 d = ok ? ((u32)((key[id] - kmin) >> shift) & 255u) : 0u;
        u64 peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const u64 bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        if (ok) {
            const u32 rank = lanes_below(peers);
            const u32 base = hw[d];
            out[base + rank] = id;
            if (rank == 0) hw[d] = base + (u32)__popcll(peers);
        }
    }
    __syncthreads();
}

// exact order of one mixed run (length <= 64) by (key, index): one wave
template <class KP, class IX>
__device__ void wave_sort_run(KP key, IX* ix, int s, int len)
{
    const int lane = threadIdx.x & 63;
    u64 k = ~0ull;
    u32 id = 0x80000000u + lane;
    if (lane < len) {
        id = (u32)ix[s + lane];
        k = key[id];
    }
    for (int size = 2; size <= 64; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const u64 ok = shfl_xor_u64(k, stride);
            const u32 oid = __shfl_xor(id, stride, 64);
            const bool up = (lane & size) == 0 || size == 64;
            const bool lower = (lane & stride) == 0;
            const bool other_less = (ok < k) || (ok == k && oid < id);
            const bool take = (lower == up) ? other_less : !other_less;
            if (take) {
                k = ok;
                id = oid;
            }
        }
    }
    if (lane < len) ix[s + lane] = (IX)id;
}

template <int T, bool BIG>
__global__ void __launch_bounds__(T) k_gene_rank(RankArgs A, int cap)
{
    using IX = typename std::conditional<BIG, u32, unsigned short>::type;
    using ST = typename std::conditional<BIG, u64, u32>::type;
    constexpr int W = T / 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((int)blockIdx.x >= *A.list_count) return;
    const int g = A.gene_list[blockIdx.x];
    const int K = A.K, tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    STAMP(A, 0);
    RankSmall<T>& L = *(RankSmall<T>*)smem;
    u64* const EX = (u64*)(smem + sizeof(RankSmall<T>));  // tie terms E[K][K], X[K][K]
    ST* S = (ST*)(smem + sizeof(RankSmall<T>) + 16 * (size_t)K * K);
    char* big = (char*)S + ((sizeof(ST) * K * K + 15) & ~(size_t)15);
    const i64 base = A.gstart[g];
    const int n = (int)(A.gstart[g + 1] - base);
    const u64* gkey = A.keys + base;
    u64* lkey = (u64*)big;
    IX* ix0;
    IX* ix1;
    u8* uc;
    u8* sc;
    if (BIG) {
        ix0 = (IX*)(A.gix + base);
        ix1 = (IX*)(A.gix + A.nnz + base);
        uc = A.guc + base;
        sc = A.gsc + base;
    } else {
        ix0 = (IX*)(lkey + cap);
        ix1 = ix0 + cap;
        uc = (u8*)(ix1 + cap);
        sc = uc + cap;
    }
    const u64* key = BIG ? gkey : (const u64*)lkey;
    for (int i = tid; i < K * K; i += T) S[i] = 0;
    for (int i = tid; i < 2 * K * K; i += T) EX[i] = 0;
    for (int i = tid; i < W * K; i += T) L.whist[i] = 0;
    for (int i = tid; i < K; i += T) L.F[i] = 0;
    if (tid <= K) L.off[tid] = (int)A.coff[(size_t)A.cl_cc[tid] * A.G + g];
    if (tid == 0) {
        L.nruns = 0;
        L.flag = 0;
        L.redo = 0;
    }
    if (!BIG)
        for (int i = tid; i < n; i += T) lkey[i] = gkey[i];
    __syncthreads();
    STAMP(A, 1);
    // ---- 1. statistics over balanced cluster pieces
    const int Lp = max(64, (((n + W - 1) / W) + 63) & ~63);
    for (int it = w;; it += W) {
        int a = 0, acc = 0, ni = 0;
        for (; a < K; ++a) {
            const int len = L.off[a + 1] - L.off[a];
            ni = (len + Lp - 1) / Lp;
            if (it < acc + ni) break;
            acc += ni;
        }
        if (a == K) break;
        const int s0 = L.off[a] + (it - acc) * Lp, s1 = min(L.off[a + 1], s0 + Lp);
        dd sx{0.0, 0.0}, se{0.0, 0.0};
        u32 pos = 0, neg = 0;
        u64 kmn = ~0ull, kmx = 0;
        for (int i = s0 + lane; i < s1; i += 64) {
            const u64 kk = key[i];
            uc[i] = (u8)a;
            const double x = scc_val_of(kk);
            sx = dd_add_d(sx, x);
            se = dd_add_d(se, expm1(x));
            pos += (x > 0.0);
            neg += (x < 0.0);
            kmn = kk < kmn ? kk : kmn;
            kmx = kk > kmx ? kk : kmx;
        }
        sx = dd_wave_sum(sx);
        se = dd_wave_sum(se);
        pos = u32_wave_sum(pos);
        neg = u32_wave_sum(neg);
        for (int m = 32; m >= 1; m >>= 1) {
            const u64 o1 = shfl_xor_u64(kmn, m), o2 = shfl_xor_u64(kmx, m);
            kmn = o1 < kmn ? o1 : kmn;
            kmx = o2 > kmx ? o2 : kmx;
        }
        if (lane == 0) {
            StatItem& I = L.item[it];
            I.sx_hi = sx.hi;
            I.sx_lo = sx.lo;
            I.se_hi = se.hi;
            I.se_lo = se.lo;
            I.pos = pos;
            I.neg = neg;
            I.kmin = kmn;
            I.kmax = kmx;
        }
    }
    __syncthreads();
    if (tid < K) {  // combine the pieces of cluster a in order
        const int a = tid;
        int first = 0;
        for (int b = 0; b < a; ++b) first += (L.off[b + 1] - L.off[b] + Lp - 1) / Lp;
        const int ni = (L.off[a + 1] - L.off[a] + Lp - 1) / Lp;
        dd sx{0.0, 0.0}, se{0.0, 0.0};
        u32 pos = 0, neg = 0;
        for (int q = first; q < first + ni; ++q) {
            sx = dd_add(sx, dd{L.item[q].sx_hi, L.item[q].sx_lo});
            se = dd_add(se, dd{L.item[q].se_hi, L.item[q].se_lo});
            pos += L.item[q].pos;
            neg += L.item[q].neg;
        }
        const double na = (double)A.n_clu[a];
        A.mean_x[(size_t)a * A.G + g] = dd_div_n(sx, na);
        A.mean_e[(size_t)a * A.G + g] = dd_div_n(se, na);
        A.cnt_pos[(size_t)a * A.G + g] = pos;
        L.posc[a] = pos;
        L.negc[a] = neg;
    }
    if (tid == 0) {
        int nit = 0;
        for (int b = 0; b < K; ++b) nit += (L.off[b + 1] - L.off[b] + Lp - 1) / Lp;
        u64 kmn = ~0ull, kmx = 0;
        for (int q = 0; q < nit; ++q) {
            kmn = L.item[q].kmin < kmn ? L.item[q].kmin : kmn;
            kmx = L.item[q].kmax > kmx ? L.item[q].kmax : kmx;
        }
        L.kmin = kmn;
        L.kmax = kmx;
    }
    for (int i = tid; i < n; i += T) ix0[i] = (IX)i;
    __syncthreads();
    STAMP(A, 2);
    // ---- 2. stable radix sort of the index permutation
    const u64 kmin = L.kmin;
    const u64 range = (n > 0) ? L.kmax - kmin : 0;
    const int bits = range ? 64 - __clzll((long long)range) : 0;
    const int sh = bits > 32 ? bits - 32 : 0;
    IX* in = ix0;
    IX* out = ix1;
    for (int p = 0; sh + 8 * p < bits; ++p) {
        radix_pass<T>(key, kmin, sh + 8 * p, in, out, n, L);
        IX* t = in;
        in = out;
        out = t;
    }
    if (sh > 0) {  // exact fix-up of windows that merged distinct doubles
        for (int i = tid; i + 1 < n; i += T) {
            const u64 k0 = key[in[i]], k1 = key[in[i + 1]];
            if (k0 != k1 && ((k0 - kmin) >> sh) == ((k1 - kmin) >> sh)) L.flag = 1;
        }
        __syncthreads();
        if (L.flag) {
            for (int i = tid; i < n; i += T) {
                const u64 k0 = key[in[i]];
                const u64 w0 = (k0 - kmin) >> sh;
                const bool start = (i == 0 || ((key[in[i - 1]] - kmin) >> sh) != w0) && i + 1 < n &&
                                   ((key[in[i + 1]] - kmin) >> sh) == w0;
                if (!start) continue;
                int e = i + 1;
                bool mixed = false;
                while (e < n) {
                    const u64 ke = key[in[e]];
                    if (((ke - kmin) >> sh) != w0) break;
                    mixed |= ke != k0;
                    ++e;
                }
                if (!mixed) continue;
                if (e - i <= 64) {
                    const int slot = atomicAdd(&L.nruns, 1);
                    if (slot < RK_RUNS) {
                        L.run_s[slot] = i;
                        L.run_l[slot] = e - i;
                    } else {
                        L.redo = 1;
                    }
                } else {
                    L.redo = 1;
                }
            }
            __syncthreads();
            if (L.redo) {  // pathological: exact sort on every bit
                for (int i = tid; i < n; i += T) ix0[i] = (IX)i;
                __syncthreads();
                in = ix0;
                out = ix1;
                for (int p = 0; 8 * p < bits; ++p) {
                    radix_pass<T>(key, kmin, 8 * p, in, out, n, L);
                    IX* t = in;
                    in = out;
                    out = t;
                }
            } else {
                for (int r = w; r < L.nruns; r += W) wave_sort_run(key, in, L.run_s[r], L.run_l[r]);
                __syncthreads();
            }
        }
    }
    // sorted codes; bit 7: equal to the next element (tie group continues)
    for (int i = tid; i < n; i += T) {
        const IX id = in[i];
        const u64 k0 = key[id];
        const bool eqn = (i + 1 < n) && key[in[i + 1]] == k0;
        sc[i] = (u8)(uc[id] | (eqn ? 128 : 0));
    }
    __syncthreads();
    STAMP(A, 6);
    // ---- 3+4. sweep.  Wave w walks its chunk in order; lane b holds C_b = #b
    // before the element and G_b = #b before it inside its tie group.  At an
    // element of code a:  S[a][b] += C_b;  for b < a in the same group
    // E[b][a] += G_b, X[b][a] += G_b (2 G_a + 1 + G_b);  F_a += 3 G_a (G_a + 1).
    // Summed over a group these are c_a c_b, c_a c_b (c_a + c_b), c^3 - c.
    const int ch = (n + W - 1) / W;
    const int c0 = min(n, w * ch), c1 = min(n, c0 + ch);
    for (int i = c0 + lane; i < c1; i += 64) atomicAdd(&L.whist[w * K + (sc[i] & 63)], 1u);
    __syncthreads();
    STAMP(A, 3);
    {
        u32 C = 0, Gc = 0;
        u64 Facc = 0;
        if (lane < K)
            for (int v = 0; v < w; ++v) C += L.whist[v * K + lane];
        bool peq = false;
        if (c0 < c1 && c0 > 0 && (sc[c0 - 1] & 128)) {  // a tie group runs into this chunk
            peq = true;
            for (int j = c0 - 1; j >= 0; --j) {
                const int v = sc[j];
                if (j < c0 - 1 && !(v & 128)) break;
                Gc += ((v & 63) == lane);
            }
        }
        u64* E = EX;
        u64* X = EX + K * K;
        if (K <= 32) {
            u32 acc[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) acc[q] = 0;
            for (int i0 = c0; i0 < c1; i0 += 64) {
                const int cv = (i0 + lane < c1) ? (int)sc[i0 + lane] : 0;
                const int cnt = __builtin_amdgcn_readfirstlane(min(64, c1 - i0));
                for (int j = 0; j < cnt; ++j) {
                    const int v = __builtin_amdgcn_readlane(cv, j);
                    const int a = v & 63;
                    if (!peq) {
                        Gc = 0;
                    } else {
                        const u32 Ga = __builtin_amdgcn_readlane(Gc, a);
                        if (lane < a && Gc) {
                            atomicAdd((unsigned long long*)&E[lane * K + a], (unsigned long long)Gc);
                            atomicAdd((unsigned long long*)&X[lane * K + a],
                                      (unsigned long long)Gc * (2ull * Ga + 1ull + Gc));
                        }
                    }
                    const bool me = lane == a;
                    Facc += me ? 3ull * Gc * (Gc + 1ull) : 0ull;
                    acc[a & 31] += C;
                    C += me;
                    Gc += me;
                    peq = (v & 128) != 0;
                }
            }
            if (lane < K)
                for (int q = 0; q < lane; ++q) atomicAdd(&S[q * K + lane], (ST)acc[q]);
        } else {
            for (int i0 = c0; i0 < c1; i0 += 64) {
                const int cv = (i0 + lane < c1) ? (int)sc[i0 + lane] : 0;
                const int cnt = __builtin_amdgcn_readfirstlane(min(64, c1 - i0));
                for (int j = 0; j < cnt; ++j) {
                    const int v = __builtin_amdgcn_readlane(cv, j);
                    const int a = v & 63;
                    if (!peq) {
                        Gc = 0;
                    } else {
                        const u32 Ga = __builtin_amdgcn_readlane(Gc, a);
                        if (lane < a && Gc) {
                            atomicAdd((unsigned long long*)&E[lane * K + a], (unsigned long long)Gc);
                            atomicAdd((unsigned long long*)&X[lane * K + a],
                                      (unsigned long long)Gc * (2ull * Ga + 1ull + Gc));
                        }
                    }
                    const bool me = lane == a;
                    Facc += me ? 3ull * Gc * (Gc + 1ull) : 0ull;
                    if (lane > a && lane < K) atomicAdd(&S[a * K + lane], (ST)C);
                    C += me;
                    Gc += me;
                    peq = (v & 128) != 0;
                }
            }
        }
        if (lane < K && Facc) atomicAdd((unsigned long long*)&L.F[lane], (unsigned long long)Facc);
    }
    __syncthreads();
    STAMP(A, 4);
    // ---- 5. per pair outputs: exact 2U and tie term
    for (int p = tid; p < A.P; p += T) {
        int a, b;
        pair_decode(p, K, a, b);
        const u64 za = (u64)A.n_clu[a] - L.posc[a] - L.negc[a];
        const u64 zb = (u64)A.n_clu[b] - L.posc[b] - L.negc[b];
        const u64 s = (u64)S[a * K + b] + za * L.negc[b] + (u64)L.posc[a] * zb;  // S^pos + zero-group pairs
        const u64 u2 = 2 * s + za * zb + EX[a * K + b];
        const u64 t = L.F[a] + f_tie(za) + L.F[b] + f_tie(zb) + 3 * za * zb * (za + zb) + 3 * EX[K * K + a * K + b];
        A.u2_base[(size_t)p * A.G + g] = (i64)u2;
        A.t_base[(size_t)p * A.G + g] = (i64)t;
    }
    STAMP(A, 5);
}

// bytes of LDS for class cls at capacity cap (0: 256 threads, 1: 1024, 2: 1024 HBM-resident)
__host__ inline size_t rank_lds_bytes(int cls, int cap, int K)
{
    const size_t small = (cls == 0) ? sizeof(RankSmall<256>) : sizeof(RankSmall<1024>);
    const size_t s = 16 * (size_t)K * K + (((size_t)K * K * (cls == 2 ? 8 : 4) + 15) & ~(size_t)15);
    const size_t per = (cls == 2) ? 0 : (8 + 2 * 2 + 1 + 1);
    return small + s + per * (size_t)cap;
}

// Size classes: 0 small (n <= cap_s), 1 medium (n <= cap_m), 2 big.
__global__ void k_classify(const i64* __restrict__ gstart, int G, int cap_s, int cap_m, int* lists, int* counts)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const i64 n = gstart[g + 1] - gstart[g];
    const int cls = (n <= cap_s) ? 0 : ((n <= cap_m) ? 1 : 2);
    const int slot = atomicAdd(&counts[cls], 1);
    lists[(size_t)cls * G + slot] = g;
}

extern "C" hipError_t scc_launch_classify(const i64* gstart, int G, int cap_s, int cap_m, int* lists, int* counts,
                                          hipStream_t st)
{
    hipLaunchKernelGGL(k_classify, dim3((G + 255) / 256), dim3(256), 0, st, gstart, G, cap_s, cap_m, lists, counts);
    return hipGetLastError();
}

// largest LDS-resident capacity of class cls (0, 1) that fits the CU
extern "C" int scc_rank_cap(int cls, int want, int K)
{
    const size_t lim = 160 * 1024;
    int cap = want;
    while (cap > 64 && rank_lds_bytes(cls, cap, K) > lim) cap -= 64;
    if (cap > 65535) cap = 65535;  // u16 indices
    return cap;
}

extern "C" size_t scc_rank_lds_bytes(int cls, int cap, int K) { return rank_lds_bytes(cls, cap, K); }

extern "C" hipError_t scc_launch_gene_rank(int cls, const ScRankLaunch* L, hipStream_t st)
{
    RankArgs A;
    A.gene_list = L->gene_list;
    A.list_count = L->list_count;
    A.gstart = L->gstart;
    A.keys = L->keys;
    A.G = L->G;
    A.K = L->K;
    A.P = L->K * (L->K - 1) / 2;
    A.n_clu = L->n_clu;
    A.coff = L->coff;
    A.cl_cc = L->cl_cc;
    A.mean_x = L->mean_x;
    A.mean_e = L->mean_e;
    A.cnt_pos = L->cnt_pos;
    A.u2_base = L->u2_base;
    A.t_base = L->t_base;
    A.gix = L->gix;
    A.guc = L->guc;
    A.gsc = L->gsc;
    A.nnz = L->nnz;
    A.stamps = L->stamps;
    const int grid = L->grid;
    if (grid <= 0) return hipSuccess;
    const size_t lds = rank_lds_bytes(cls, L->cap, L->K);
    if (cls == 0) {
        hipFuncSetAttribute((const void*)k_gene_rank<256, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((k_gene_rank<256, false>), dim3(grid), dim3(256), lds, st, A, L->cap);
    } else if (cls == 1) {
        hipFuncSetAttribute((const void*)k_gene_rank<1024, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
        hipLaunchKernelGGL((k_gene_rank<1024, false>), dim3(grid), dim3(1024), lds, st, A, L->cap);
    } else {
        hipFuncSetAttribute((const void*)k_gene_rank<1024, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((k_gene_rank<1024, true>), dim3(grid), dim3(1024), lds, st, A, L->cap);
    }
    return hipGetLastError();
}
