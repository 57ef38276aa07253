// scc_rank.hip — per-gene Wilcoxon rank-sum engine (all cluster pairs at once).
//
// Replaces, for every gene and every cluster pair (i<j) simultaneously, the
// reference's per-(pair, gene) `wilcox.test(data.use[x, ] ~ group)` call
// (R/reclusterDEConsensusFast.R:78-91; R/reclusterDEConsensus.R:99-103) and the
// per-pair log-mean/pct statistics (Fast:229-271, slow:104-113).
//
// One workgroup per gene:
//   1. per-cluster statistics (dd sums of x and expm1(x), counts of x > 0 /
//      x < 0), one wave per cluster over the gene's (key, code) pairs
//   2. sort the gene's kept nonzeros by (value, cluster code)         [bitonic]
//   3. one sweep: S[a][b] = #{b-elements before an a-element}.  With ties
//      ordered by code, for a < b this is exactly #{(x in a, y in b): x > y}
//   4. tie groups of size >= 2: per-cluster f(c) = c^3 - c, and cross-cluster
//      equal pairs / cross tie terms (rare for log data)
//   5. per pair:  2U = 2*(S + z_a*neg_b + pos_a*z_b) + z_a*z_b (+ tie_e)
//                 T  = F_a + F_b + 3*z_a*z_b*(z_a+z_b)       (+ 3*tie_x)
//      where z = implicit zeros of the cluster; T = sum(NTIES^3 - NTIES).
// 2U and T are exact int64 — R's W = 2U/2 and its tie term bit for bit.
#include "scc_common.hpp"
#include "scc_kernels.hpp"
#include "scc_sort.hpp"

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

struct RankArgs {
    const int* gene_list;
    const int* list_count;
    const i64* gstart;   // [G+1] gene segment starts
    u64* keys;           // kept nonzeros' value keys (sorted in place for big genes)
    u8* codes;           // their cluster codes
    int G, K, P;
    const int* n_clu;    // kept cells per cluster
    double* mean_x;      // [K][G]
    double* mean_e;      // [K][G]
    u32* cnt_pos;        // [K][G]
    i64* u2_base;        // [P][G]
    i64* t_base;         // [P][G]
    u64* tie_e;          // [P][G] (zeroed; atomically accumulated)
    u64* tie_x;          // [P][G]
    u64* stamps;         // diagnostic phase clocks [block][8] (nullptr in normal runs)
};

#define STAMP(A, ph)                                                                      \
    do {                                                                                  \
        if ((A).stamps && threadIdx.x == 0)                                               \
            (A).stamps[(size_t)blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memtime();    \
    } while (0)

// Shared tail of both kernels: given keys/codes (LDS or HBM) sorted, and the
// per-cluster counts, do the sweep, tie groups and per-pair outputs.
template <int T, class ST>
__device__ void rank_sweep_finalize(const RankArgs& A, int g, int n, const u64* skey, const u8* scode, ST* S,
                                    u32* whist, u64* F, const u32* posc, const u32* negc)
{
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int W = T / 64;
    const int K = A.K;
    // ---- per-wave chunk histograms
    const int ch = (n + W - 1) / W;
    const int c0 = min(n, w * ch), c1 = min(n, c0 + ch);
    for (int i = c0 + lane; i < c1; i += 64) atomicAdd(&whist[w * K + scode[i]], 1u);
    __syncthreads();
    STAMP(A, 3);
    // ---- sweep: lane b keeps the running count of cluster b before position i
    if (lane < K) {
        u32 C = 0;
        for (int v = 0; v < w; ++v) C += whist[v * K + lane];
        int i = c0;
        for (; i + 4 <= c1; i += 4) {
            const int a0 = scode[i], a1 = scode[i + 1], a2 = scode[i + 2], a3 = scode[i + 3];
            atomicAdd(&S[a0 * K + lane], (ST)C);
            C += (lane == a0);
            atomicAdd(&S[a1 * K + lane], (ST)C);
            C += (lane == a1);
            atomicAdd(&S[a2 * K + lane], (ST)C);
            C += (lane == a2);
            atomicAdd(&S[a3 * K + lane], (ST)C);
            C += (lane == a3);
        }
        for (; i < c1; ++i) {
            const int a = scode[i];
            atomicAdd(&S[a * K + lane], (ST)C);
            C += (lane == a);
        }
    }
    // ---- tie groups (value runs of length >= 2); codes inside a run ascend
    for (int i = tid; i < n; i += T) {
        const u64 kv = skey[i];
        if ((i == 0 || skey[i - 1] != kv) && i + 1 < n && skey[i + 1] == kv) {
            int e = i + 1;
            while (e < n && skey[e] == kv) ++e;
            // runs of equal code within [i, e)
            for (int r = i; r < e;) {
                const int a = scode[r];
                int r2 = r + 1;
                while (r2 < e && scode[r2] == a) ++r2;
                const u64 ca = (u64)(r2 - r);
                if (ca >= 2) atomicAdd((unsigned long long*)&F[a], (unsigned long long)f_tie(ca));
                for (int s = r2; s < e;) {
                    const int b = scode[s];
                    int s2 = s + 1;
                    while (s2 < e && scode[s2] == b) ++s2;
                    const u64 cb = (u64)(s2 - s);
                    const int p = scc_pair_index(a, b, K);
                    atomicAdd((unsigned long long*)&A.tie_e[(size_t)p * A.G + g], (unsigned long long)(ca * cb));
                    atomicAdd((unsigned long long*)&A.tie_x[(size_t)p * A.G + g],
                              (unsigned long long)(ca * cb * (ca + cb)));
                    s = s2;
                }
                r = r2;
            }
        }
    }
    __syncthreads();
    STAMP(A, 4);
    // ---- per pair outputs
    for (int p = tid; p < A.P; p += T) {
        int a, b;
        pair_decode(p, K, a, b);
        const u64 za = (u64)A.n_clu[a] - posc[a] - negc[a];
        const u64 zb = (u64)A.n_clu[b] - posc[b] - negc[b];
        const u64 s = (u64)S[a * K + b] + za * negc[b] + (u64)posc[a] * zb;  // S^pos + zero-group pairs
        const u64 u2 = 2 * s + za * zb;
        const u64 t = F[a] + f_tie(za) + F[b] + f_tie(zb) + 3 * za * zb * (za + zb);
        A.u2_base[(size_t)p * A.G + g] = (i64)u2;
        A.t_base[(size_t)p * A.G + g] = (i64)t;
    }
    STAMP(A, 5);
}

// Per-cluster statistics: wave w takes clusters a = w, w+W, ... and scans the
// gene's n (key, code) pairs for its cluster (order-insensitive dd sums).
template <int T>
__device__ void cluster_stats(const RankArgs& A, int g, int n, const u64* key, const u8* code, u32* posc, u32* negc)
{
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int W = T / 64;
    for (int a = w; a < A.K; a += W) {
        dd sx{0.0, 0.0}, se{0.0, 0.0};
        u32 pos = 0, neg = 0;
        for (int i = lane; i < n; i += 64) {
            if (code[i] != a) continue;
            const double x = scc_val_of(key[i]);
            sx = dd_add_d(sx, x);
            se = dd_add_d(se, expm1(x));
            pos += (x > 0.0);
            neg += (x < 0.0);
        }
        sx = dd_wave_sum(sx);
        se = dd_wave_sum(se);
        pos = u32_wave_sum(pos);
        neg = u32_wave_sum(neg);
        if (lane == 0) {
            const double na = (double)A.n_clu[a];
            A.mean_x[(size_t)a * A.G + g] = dd_div_n(sx, na);
            A.mean_e[(size_t)a * A.G + g] = dd_div_n(se, na);
            A.cnt_pos[(size_t)a * A.G + g] = pos;
            posc[a] = pos;
            negc[a] = neg;
        }
    }
}

// LDS layout helper
struct RankLds {
    u64* skey;
    u8* scode;
    void* S;
    u32* whist;
    u64* F;
    u32* posc;
    u32* negc;
    int* off;
};

template <int T>
__device__ RankLds carve(char* smem, int cap, int K, int sbytes)
{
    RankLds L;
    size_t o = 0;
    L.skey = (u64*)(smem + o);
    o += (size_t)cap * 8;
    L.F = (u64*)(smem + o);
    o += (size_t)K * 8;
    L.S = (void*)(smem + o);
    o += (size_t)K * K * sbytes;
    L.whist = (u32*)(smem + o);
    o += (size_t)(T / 64) * K * 4;
    L.posc = (u32*)(smem + o);
    o += (size_t)K * 4;
    L.negc = (u32*)(smem + o);
    o += (size_t)K * 4;
    L.off = (int*)(smem + o);
    o += (size_t)(K + 1) * 4;
    o = (o + 15) & ~(size_t)15;
    L.scode = (u8*)(smem + o);
    return L;
}

__host__ __device__ inline size_t rank_lds_bytes(int cap, int K, int T, int sbytes)
{
    size_t o = (size_t)cap * 8 + (size_t)K * 8 + (size_t)K * K * sbytes + (size_t)(T / 64) * K * 4 + (size_t)K * 8 +
               (size_t)(K + 1) * 4;
    o = (o + 15) & ~(size_t)15;
    return o + (size_t)cap;
}

template <int T, class ST>
__device__ void zero_lds(const RankLds& L, int K)
{
    for (int i = threadIdx.x; i < K * K; i += T) ((ST*)L.S)[i] = 0;
    for (int i = threadIdx.x; i < (T / 64) * K; i += T) L.whist[i] = 0;
    for (int i = threadIdx.x; i < K; i += T) L.F[i] = 0;
}

// Genes whose kept nonzeros fit in LDS (n <= cap).
template <int T>
__global__ void __launch_bounds__(T) k_gene_rank_lds(RankArgs A, int cap)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((int)blockIdx.x >= *A.list_count) return;
    const int g = A.gene_list[blockIdx.x];
    const int K = A.K, tid = threadIdx.x;
    STAMP(A, 0);
    RankLds L = carve<T>(smem, cap, K, 4);
    const i64 base = A.gstart[g];
    const int n = (int)(A.gstart[g + 1] - base);
    zero_lds<T, u32>(L, K);
    for (int i = tid; i < n; i += T) {
        L.skey[i] = A.keys[base + i];
        L.scode[i] = A.codes[base + i];
    }
    __syncthreads();
    STAMP(A, 1);
    cluster_stats<T>(A, g, n, L.skey, L.scode, L.posc, L.negc);
    __syncthreads();  // stats read the unsorted buckets
    STAMP(A, 2);
    AccKeyCode acc{L.skey, L.scode};
    block_bitonic(acc, n, tid, T);  // ends with a barrier
    STAMP(A, 6);
    rank_sweep_finalize<T, u32>(A, g, n, L.skey, L.scode, (u32*)L.S, L.whist, L.F, L.posc, L.negc);
}

// Genes too large for LDS: keys sorted in place in HBM with LDS-staged chunks.
template <int T>
__global__ void __launch_bounds__(T) k_gene_rank_big(RankArgs A, int chunk)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((int)blockIdx.x >= *A.list_count) return;
    const int g = A.gene_list[blockIdx.x];
    const int K = A.K, tid = threadIdx.x;
    STAMP(A, 0);
    RankLds L = carve<T>(smem, chunk, K, 8);
    const i64 base = A.gstart[g];
    const int n = (int)(A.gstart[g + 1] - base);
    u64* gkey = A.keys + base;
    u8* gcode = A.codes + base;
    zero_lds<T, u64>(L, K);
    STAMP(A, 1);
    cluster_stats<T>(A, g, n, gkey, gcode, L.posc, L.negc);
    __syncthreads();
    STAMP(A, 2);
    AccKeyCode gacc{gkey, gcode}, sacc{L.skey, L.scode};
    block_bitonic_staged(gacc, n, sacc, chunk, tid, T);
    STAMP(A, 6);
    rank_sweep_finalize<T, u64>(A, g, n, gkey, gcode, (u64*)L.S, L.whist, L.F, L.posc, L.negc);
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

extern "C" size_t scc_rank_lds_bytes(int cls, int cap, int K)
{
    return rank_lds_bytes(cap, K, cls == 0 ? 256 : 1024, cls == 2 ? 8 : 4);
}

extern "C" hipError_t scc_launch_gene_rank(int cls, const ScRankLaunch* L, hipStream_t st)
{
    RankArgs A;
    A.gene_list = L->gene_list;
    A.list_count = L->list_count;
    A.gstart = L->gstart;
    A.keys = L->keys;
    A.codes = L->codes;
    A.G = L->G;
    A.K = L->K;
    A.P = L->K * (L->K - 1) / 2;
    A.n_clu = L->n_clu;
    A.mean_x = L->mean_x;
    A.mean_e = L->mean_e;
    A.cnt_pos = L->cnt_pos;
    A.u2_base = L->u2_base;
    A.t_base = L->t_base;
    A.tie_e = L->tie_e;
    A.tie_x = L->tie_x;
    A.stamps = L->stamps;
    const int grid = L->grid;
    if (grid <= 0) return hipSuccess;
    if (cls == 0) {
        size_t lds = rank_lds_bytes(L->cap, L->K, 256, 4);
        hipFuncSetAttribute((const void*)k_gene_rank_lds<256>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_gene_rank_lds<256>, dim3(grid), dim3(256), lds, st, A, L->cap);
    } else if (cls == 1) {
        size_t lds = rank_lds_bytes(L->cap, L->K, 1024, 4);
        hipFuncSetAttribute((const void*)k_gene_rank_lds<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_gene_rank_lds<1024>, dim3(grid), dim3(1024), lds, st, A, L->cap);
    } else {
        size_t lds = rank_lds_bytes(L->cap, L->K, 1024, 8);
        hipFuncSetAttribute((const void*)k_gene_rank_big<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_gene_rank_big<1024>, dim3(grid), dim3(1024), lds, st, A, L->cap);
    }
    return hipGetLastError();
}
