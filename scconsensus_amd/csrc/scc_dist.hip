// scc_dist.hip — stage 3: cell x cell distance on the DE-gene union.
//
// Reference: pca.data <- irlba::prcomp_irlba(t(X[U, ]), n = min(|U|, 15),
// center = TRUE)$x; d <- dist(pca.data, "euclidean")
// (R/reclusterDEConsensusFast.R:398-400; R/reclusterDEConsensus.R:234-236) and
// the commented alternative as.dist(1 - cor(X[U, ])) (Fast:403, slow:239).
//
// Kernels
//   k_gather_*      X[U, ] -> Xc (N x nu_pad, row-major fp64, zero padded)
//   k_colsum/center R colMeans (LDOUBLE sum restated as double-double) and centring
//   k_gram_f64      C = Xc^T Xc, fp64 MFMA (v_mfma_f64_16x16x4_f64), split over
//                   cell chunks into slabs reduced in a fixed order (deterministic)
//   k_scores        P = Xc V_k (N x 16, zero padded components)
//   k_dist_aligned  packed lower triangle in R `dist` order, line-aligned
//                   windows staged in LDS; per element the squared distance
//                   (FMA) + Newton-refined sqrt
//   k_zscore / k_pearson_mfma  Pearson: per-cell centring/scaling, then an
//                   LDS-pipelined FP32 MFMA (v_mfma_f32_32x32x2_f32) Gram with the
//                   1 - r epilogue fused into coalesced packed-column stores.
#include "scc_common.hpp"
#include <algorithm>
#include <mutex>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------ gather
// One wave per cell: its row indices stream in with 8 loads per lane in
// flight; the value is fetched only for the union genes (a few per cent of
// the nnz).  The cell's row of X[U,] (ld doubles, zero for absent genes and
// the padding columns) is assembled in LDS and leaves as whole coalesced
// lines, so the output needs no memset pass and no partial-line stores.
// Row-index and union-map loads are clamped and unconditional, the bounds
// applied by selects afterwards (a load under a lane condition is a branch
// with its own wait).  Rows outside [0, G) (invalid input, reported by the
// DE's ingest) map to no slot.
// LDSROW false (ld > GATHER_LDS_LD: a union too wide for four LDS rows): the
// values go straight to Xc, which the caller has zeroed.
#define GATHER_LDS_LD 2048
template <bool LDSROW>
__global__ void __launch_bounds__(256) k_gather_csc(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                    const double* __restrict__ vals, int N, int G,
                                                    const int* __restrict__ umap, int ld, double* __restrict__ Xc)
{
    extern __shared__ __attribute__((aligned(16))) double grow[];  // [4 waves][ld]
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    const int c = blockIdx.x * (blockDim.x >> 6) + wv;
    if (c >= N) return;  // whole waves: no workgroup barrier below
    double* row = LDSROW ? grow + (size_t)wv * ld : Xc + (size_t)c * ld;
    if (LDSROW)
        for (int u = lane; u < ld; u += 64) row[u] = 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // LDS stores drained (s_waitcnt lgkmcnt(0))
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const i64 b = indptr[c], e = indptr[c + 1];
    for (i64 k0 = b + lane; k0 < e; k0 += 512) {
        int r[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const i64 k = k0 + 64 * q;
            r[q] = rows[k < e ? k : e - 1];
        }
        int u[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int rc = min(max(r[q], 0), G - 1);
            const int x = umap[rc];
            u[q] = (k0 + 64 * q < e && r[q] == rc) ? x : -1;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (u[q] >= 0) row[u[q]] = vals[k0 + 64 * q];
    }
    if (!LDSROW) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    double* out = Xc + (size_t)c * ld;
    for (int u = lane; u < ld; u += 64) out[u] = row[u];
}

// The same gather with the union map in LDS (u16 slots, 0xffff = not in the
// union): persistent workgroups build the map from the union's gene list and
// walk cells, so a row index costs one LDS lookup instead of a dependent global
// load of umap[row] (three dependent global round trips per batch of 512
// entries become two).  Rows [N, Npad) (padding) leave as zeros, so a call
// needs no memset and no global union map before it (two launches and ~60 us
// of GPU idle at config B).  Used when the map and four LDS rows fit (G * 2 +
// 4 * ld * 8 bytes).
__global__ void __launch_bounds__(1024) k_gather_csc_lm(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                       const double* __restrict__ vals, int N, int Npad, int G,
                                                       const int* __restrict__ genes, int nu, int ld,
                                                       double* __restrict__ Xc)
{
    extern __shared__ __attribute__((aligned(16))) double grow[];  // [waves][ld], then the map
    const int nw = blockDim.x >> 6;
    unsigned short* lmap = (unsigned short*)(grow + nw * (size_t)ld);
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    for (int g = threadIdx.x; g < G; g += blockDim.x) lmap[g] = 0xffff;
    __syncthreads();
    for (int u = threadIdx.x; u < nu; u += blockDim.x) lmap[genes[u]] = (unsigned short)u;  // genes checked by the host
    __syncthreads();
    double* row = grow + (size_t)wv * ld;
    for (int c = blockIdx.x * nw + wv; c < Npad; c += gridDim.x * nw) {
        for (int u = lane; u < ld; u += 64) row[u] = 0.0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const i64 b = c < N ? indptr[c] : 0, e = c < N ? indptr[c + 1] : 0;
        for (i64 k0 = b + lane; k0 < e; k0 += 512) {
            int r[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const i64 k = k0 + 64 * q;
                r[q] = rows[k < e ? k : e - 1];
            }
            int u[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int rc = min(max(r[q], 0), G - 1);
                const int x = lmap[rc];
                u[q] = (k0 + 64 * q < e && r[q] == rc && x != 0xffff) ? x : -1;
            }
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {  // the hits' values, all in flight together
                const i64 k = k0 + 64 * q;
                v[q] = vals[u[q] >= 0 ? k : b];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (u[q] >= 0) row[u[q]] = v[q];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        double* out = Xc + (size_t)c * ld;
        for (int u = lane; u < ld; u += 64) out[u] = row[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the row is read out before the next clear
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
}

// true when the CSC gather writes every element of its rows (the caller then
// clears only the padding rows)
extern "C" int scc_gather_writes_rows(int ld) { return ld <= GATHER_LDS_LD; }

__global__ void __launch_bounds__(256) k_gather_dense(const double* __restrict__ X, int G, int N,
                                                      const int* __restrict__ genes, int nu, int ld,
                                                      double* __restrict__ Xc)
{
    const size_t total = (size_t)N * nu;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(e / nu), u = (int)(e % nu);
        Xc[(size_t)c * ld + u] = X[(size_t)c * G + genes[u]];
    }
}

// column sums in dd: grid (ceil(ld/256), nchunk); partial[chunk][u]
__global__ void __launch_bounds__(256) k_colsum(const double* __restrict__ Xc, int N, int ld, int rows_per_chunk,
                                                dd* __restrict__ part)
{
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= ld) return;
    const int c0 = blockIdx.y * rows_per_chunk, c1 = min(N, c0 + rows_per_chunk);
    dd s{0.0, 0.0};
    for (int c = c0; c < c1; ++c) s = dd_add_d(s, Xc[(size_t)c * ld + u]);
    part[(size_t)blockIdx.y * ld + u] = s;
}

// one wave per column: lane l folds partials l, l + 64, ... in order, then a
// fixed butterfly (deterministic)
__global__ void __launch_bounds__(256) k_colmean(const dd* __restrict__ part, int nchunk, int ld, int N,
                                                 double* __restrict__ mean)
{
    const int u = blockIdx.x * 4 + scc_wave_id(), lane = threadIdx.x & 63;
    if (u >= ld) return;
    dd s{0.0, 0.0};
    for (int k = lane; k < nchunk; k += 64) s = dd_add(s, part[(size_t)k * ld + u]);
    s = dd_wave_sum_dpp(s);
    if (lane == 0) mean[u] = dd_div_n(s, (double)N);
}

// two elements per thread (ld is a multiple of 64): 16-byte loads and stores
__global__ void __launch_bounds__(256) k_center(double* __restrict__ Xc, int N, int nu, int ld,
                                                const double* __restrict__ mean)
{
    const size_t total2 = (size_t)N * ld / 2;
    double2* X2 = (double2*)Xc;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total2; e += (size_t)gridDim.x * blockDim.x) {
        const int u = (int)((2 * e) % ld);
        double2 x = X2[e];
        if (u < nu) x.x -= mean[u];
        if (u + 1 < nu) x.y -= mean[u + 1];
        X2[e] = x;
    }
}

// ------------------------------------------------------------------ Gram (fp64 MFMA)
// Dispatch slot -> (output tile, cell chunk).  Slot x runs on XCD x % 8; the
// slots of one XCD take whole chunks, all tiles of a chunk together, so the
// chunk's rows of Xc come from HBM once into that XCD's L2 and every tile
// reading them hits there (with chunk-major slots across the grid, a chunk's
// tiles sat on all eight XCDs and each fetched the rows: 5.7x the operand at
// B, 8x at D).  The grid is ceil(nchunk / 8) * 8 * ntl slots; the spare ones exit.
__device__ inline bool gram_slot(int ntl, int nchunk, int& tile, int& chunk)
{
    const int x = blockIdx.x, xcd = x & 7, q = x >> 3;
    chunk = (q / ntl) * 8 + xcd;
    tile = q % ntl;
    return chunk < nchunk;
}
static inline unsigned gram_grid(int ntl, int nchunk) { return (unsigned)(((nchunk + 7) / 8) * 8 * ntl); }

#define GR_U 4  // 4-row k-steps whose loads are issued together (8: B 0.13, C 0.88, D 4.51 ms)
// WG = 4 waves -> 64x64 tile of C (upper tiles only); wave -> 32x32 = 2x2 MFMA
// 16x16x4 tiles.  Lane l holds A[i = l&15][k = l>>4] and B[k = l>>4][j = l&15];
// accumulator reg r is C[row = (l>>4) + 4r][col = l&15] (f64 layout).
// mean (nullptr: Xc is centred already): the column means subtracted on the
// fly from rows < nval (the same x - mean[u] k_center stores, so the same
// bits), rows past nval zero.  (The 128-wide kernel below keeps an explicit
// centring pass: eight more registers took it from two waves per SIMD to one.)
__global__ void __launch_bounds__(256) k_gram_f64(const double* __restrict__ Xc, int Npad, int ld, int ntile,
                                                  int nchunk, int rows_per_chunk, double* __restrict__ slabs,
                                                  const double* __restrict__ mean, int nval)
{
    // upper-triangular tile index -> (ti, tj), ti <= tj; every tile of one
    // chunk on one XCD (gram_slot)
    int t, chunk;
    if (!gram_slot(ntile * (ntile + 1) / 2, nchunk, t, chunk)) return;
    int ti = 0;
    while (t >= ntile - ti) {
        t -= ntile - ti;
        ++ti;
    }
    const int tj = ti + t;
    const int lane = threadIdx.x & 63, w = scc_wave_id();
    const int wi = (w >> 1) * 32, wj = (w & 1) * 32;
    const int i0 = ti * 64 + wi, j0 = tj * 64 + wj;
    const int c0 = chunk * rows_per_chunk, c1 = min(Npad, c0 + rows_per_chunk);
    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    const int kr = lane >> 4, cc = lane & 15;
    const double mx0 = mean ? mean[i0 + cc] : 0.0, mx1 = mean ? mean[i0 + 16 + cc] : 0.0;
    const double my0 = mean ? mean[j0 + cc] : 0.0, my1 = mean ? mean[j0 + 16 + cc] : 0.0;
    const int cv = min(c1, nval);
    // 4 GR_U rows per round: all loads of a round issued before its MFMAs
    // (clamped row, masked value past the chunk), so a round waits on memory
    // once instead of GR_U times (GR_U 4: B 0.14, C 0.89, D 4.35 ms; 1: 0.18 / 1.43 / 5.22;
    // issuing the next round's loads before this round's MFMAs: B 0.166 ms)
    for (int c = c0; c < c1; c += 4 * GR_U) {
        double a0[GR_U], a1[GR_U], b0[GR_U], b1[GR_U];
#pragma unroll
        for (int u = 0; u < GR_U; ++u) {
            const int rr = c + 4 * u + kr;
            const double* row = Xc + (size_t)min(rr, c1 - 1) * ld;
            const double x0 = row[i0 + cc], x1 = row[i0 + 16 + cc];
            const double y0 = row[j0 + cc], y1 = row[j0 + 16 + cc];
            const bool ok = rr < cv;
            a0[u] = ok ? x0 - mx0 : 0.0;
            a1[u] = ok ? x1 - mx1 : 0.0;
            b0[u] = ok ? y0 - my0 : 0.0;
            b1[u] = ok ? y1 - my1 : 0.0;
        }
#pragma unroll
        for (int u = 0; u < GR_U; ++u) {
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[u], b0[u], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[u], b1[u], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[u], b0[u], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[u], b1[u], acc[1][1], 0, 0, 0);
        }
    }
    double* S = slabs + (size_t)chunk * ld * ld;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = i0 + a * 16 + kr + 4 * r;
                const int col = j0 + b * 16 + cc;
                S[(size_t)row * ld + col] = acc[a][b][r];
            }
}

// The same Gram with 128 x 128 output tiles (each wave 64 x 64: 4 x 4 MFMA
// tiles): every row segment of Xc is fetched by half as many workgroups (the
// re-fetch factor is the number of column tiles: 14 at config D's |U| = 845
// with 64-wide tiles, 17x the operand in FETCH_SIZE).  The slab layout is
// k_gram_reduce's (64-wide blocks ti <= tj): the lower 64-block of a diagonal
// 128 tile is not computed (its mirror is), and a tile whose second 64-block
// falls past ld (ld % 128 == 64) leaves those waves idle.
__global__ void __launch_bounds__(256) k_gram_f64_128(const double* __restrict__ Xc, int Npad, int ld, int ntile,
                                                      int nchunk, int rows_per_chunk, double* __restrict__ slabs)
{
    int t, chunk;
    if (!gram_slot(ntile * (ntile + 1) / 2, nchunk, t, chunk)) return;
    int ti = 0;
    while (t >= ntile - ti) {
        t -= ntile - ti;
        ++ti;
    }
    const int tj = ti + t;
    const int lane = threadIdx.x & 63, w = scc_wave_id();
    const int wi = (w >> 1) * 64, wj = (w & 1) * 64;
    const int i0 = ti * 128 + wi, j0 = tj * 128 + wj;
    const int c0 = chunk * rows_per_chunk, c1 = min(Npad, c0 + rows_per_chunk);
    if (ti == tj && wi > wj) return;   // the mirror of (wj, wi)
    if (i0 >= ld || j0 >= ld) return;  // past the last 64-column block
    d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    const int kr = lane >> 4, cc = lane & 15;
    constexpr int U = 2;
    for (int c = c0; c < c1; c += 4 * U) {
        double av[U][4], bv[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int rr = c + 4 * u + kr;
            const double* row = Xc + (size_t)min(rr, c1 - 1) * ld;
            const bool ok = rr < c1;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const double x = row[i0 + 16 * m + cc], y = row[j0 + 16 * m + cc];
                av[u][m] = ok ? x : 0.0;
                bv[u][m] = ok ? y : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][a], bv[u][b], acc[a][b], 0, 0, 0);
    }
    double* S = slabs + (size_t)chunk * ld * ld;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = i0 + a * 16 + kr + 4 * r;
                const int col = j0 + b * 16 + cc;
                S[(size_t)row * ld + col] = acc[a][b][r];
            }
}

// C[i][j] = sum_k slabs[k][i][j] in chunk order for 64-blocks ti <= tj, and
// the same sum stored at C[j][i]: the slabs are read only where they were
// computed, in whole lines (reading the mirror column-wise for the lower
// blocks fetched a line per element: 3.5x the slabs at B); the transposed
// stores of one block come from one workgroup and merge in its XCD's L2
__global__ void __launch_bounds__(256) k_gram_reduce(const double* __restrict__ slabs, int nchunk, int ld,
                                                     double* __restrict__ C)
{
    const size_t total = (size_t)ld * ld;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / ld), j = (int)(e % ld);
        const int ti = i >> 6, tj = j >> 6;
        if (ti > tj) continue;
        double s = 0.0;
#pragma unroll 8
        for (int k = 0; k < nchunk; ++k) s += slabs[(size_t)k * total + e];
        C[e] = s;
        if (ti < tj) C[(size_t)j * ld + i] = s;
    }
}

// ------------------------------------------------------------------ scores
// P[c][q] = sum_u Xc[c][u] * Z[u][q]; Z row-major [u][16] (PC1 first, columns
// q >= k are zero).
__global__ void __launch_bounds__(256) k_scores(const double* __restrict__ Xc, int N, int nu, int ld,
                                                const double* __restrict__ Z16, int k, double* __restrict__ P,
                                                const double* __restrict__ mean)
{
    __shared__ double sv[64][16];
    const int c = blockIdx.x * 256 + threadIdx.x;
    double acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.0;
    for (int u0 = 0; u0 < nu; u0 += 64) {
        __syncthreads();
        for (int e = threadIdx.x; e < 64 * 16; e += 256) {
            const int uu = e / 16, q = e % 16;
            const int u = u0 + uu;
            sv[uu][q] = (u < nu && q < k) ? Z16[(size_t)u * 16 + q] : 0.0;
        }
        __syncthreads();
        if (c < N) {
            const int ue = min(64, nu - u0);
            const double* row = Xc + (size_t)c * ld + u0;
            for (int uu = 0; uu < ue; ++uu) {
                const double x = mean ? row[uu] - mean[u0 + uu] : row[uu];
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[q] = fma(x, sv[uu][q], acc[q]);
            }
        }
    }
    if (c < N) {
#pragma unroll
        for (int q = 0; q < 16; ++q) P[(size_t)c * 16 + q] = acc[q];
    }
}

// The same product on fp64 MFMA (16 x 16 x 4): a wave owns 16 cells, Z
// passes through LDS 64 rows at a time, and lane (i, g) loads 16 consecutive
// entries of cell i's row (two 64-byte loads; 16 cells x 4 lane groups read
// 256 contiguous bytes of every row) that feed 16 MFMA steps, step s pairing
// the row's entry 16 g + s with Z's row 16 g + s (the same k order on both
// operands).  The per-thread loop above read one double per row per
// iteration, 64 rows ld apart per load instruction.
__global__ void __launch_bounds__(256) k_scores_mfma(const double* __restrict__ Xc, int N, int nu, int ld,
                                                     const double* __restrict__ Z16, int k, double* __restrict__ P,
                                                     const double* __restrict__ mean)
{
    __shared__ double zs[64][16];
    const int lane = threadIdx.x & 63, w = scc_wave_id();
    const int c0 = (blockIdx.x * 4 + w) * 16;
    const int i = lane & 15, g = lane >> 4;
    const double* row = Xc + (size_t)min(c0 + i, N - 1) * ld;  // rows past N: computed, not stored
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int u0 = 0; u0 < nu; u0 += 64) {
        __syncthreads();
        for (int e = threadIdx.x; e < 64 * 16; e += 256) {
            const int uu = e >> 4, q = e & 15, u = u0 + uu;
            zs[uu][q] = (u < nu && q < k) ? Z16[(size_t)u * 16 + q] : 0.0;
        }
        typedef double dv2 __attribute__((ext_vector_type(2)));
        double xa[16];
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {  // (u0 + 16 g + 16 <= ld: ld is a multiple of 64)
            const dv2 v = *(const dv2*)(row + u0 + 16 * g + 2 * s2);
            xa[2 * s2] = v.x;
            xa[2 * s2 + 1] = v.y;
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int u = u0 + 16 * g + s;
            const double m = mean ? mean[min(u, nu - 1)] : 0.0;
            xa[s] = (u < nu) ? (mean ? xa[s] - m : xa[s]) : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[s], zs[16 * g + s][i], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // accumulator r: cell c0 + g + 4 r, component i
        const int cell = c0 + g + 4 * r;
        if (cell < N) P[(size_t)cell * 16 + i] = acc[r];
    }
}

// ------------------------------------------------------------------ Euclidean dist
// Per element |p_i|^2 + |p_j|^2 - 2 p_i.p_j over the k <= 15 components (the
// difference form where that cancels) and a Newton-refined sqrt (scc_sqrt_nr;
// the hardware v_sqrt_f64 alone is ~1e-8 relative: 5e-7 absolute at B); the
// contract is 1e-5 absolute (BASELINE north_star).  The kernel is bound by the
// HBM write stream (practical ceiling ~5.1 TB/s: scripts/write_bw.py).
//
// In R's packed order a column's entries are contiguous but start at any
// offset, so a fixed row partition leaves two partial 128-B lines per (column,
// tile) that the neighbouring tile completes later: read-modify-writes in HBM
// (0.5 GB fetched by a write-only kernel at config B).  Here tile rb owns, for
// column j, the rows whose packed addresses fall in the 128-B-aligned window
// [rb TR - delta_j, rb TR + TR - delta_j) (delta_j = that address mod one line;
// TR a multiple of the line, so consecutive tiles partition every column
// exactly): its 256 threads compute rows rb TR - HALO + t (HALO = one line of
// outputs), the values go through an LDS stage (NB columns at a time) and are
// stored as whole lines.  Partial lines remain only where one column's segment
// ends and the next begins.  Column scores are wave-uniform loads (scalar
// registers, no LDS broadcast per element); |p_j|^2 is formed once per tile.
#define DA_T 256
#define DA_NB 8

template <int TR, int DC>
__device__ __host__ inline int da_rbmin(int cb)
{
    const int r = (cb * DC + 1) / TR - 1;
    return r > 0 ? r : 0;
}

template <bool F32, int DC, int NB, bool NT, bool V2>
__global__ void __launch_bounds__(DA_T) k_dist_aligned(const double* __restrict__ P, int N, int nrb, int cb_lo,
                                                       int ncbl, int c_lo, int c_hi, long long obase,
                                                       void* __restrict__ out, const int2* __restrict__ tiles,
                                                       int ntiles)
{
    constexpr int HALO = F32 ? 32 : 16;  // outputs per 128-B line
    constexpr int TR = DA_T - HALO;      // rows owned per tile
    __shared__ double stage[NB][DA_T];
    __shared__ double cn[DC];
    int cb, r0;
    if (tiles) {
        // tile list in panel order (dist_tile_list), dealt to the XCDs as
        // contiguous runs: the hardware gives consecutive workgroup ids to
        // consecutive XCDs, so id -> (id % 8) * per + id / 8
        const int per = (ntiles + 7) >> 3;
        const int L = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
        if (L >= ntiles) return;
        const int2 e = tiles[L];
        cb = e.x;
        r0 = e.y * TR;
    } else {
        // folded triangle: grid row y holds column block y then its mirror
        const int y = blockIdx.y;
        int x = blockIdx.x;
        cb = cb_lo + y;
        const int cntA = nrb - da_rbmin<TR, DC>(cb);
        if (x >= cntA) {
            x -= cntA;
            const int cb2 = cb_lo + ncbl - 1 - y;
            if (cb2 <= cb) return;
            cb = cb2;
            if (x >= nrb - da_rbmin<TR, DC>(cb)) return;
        }
        r0 = (da_rbmin<TR, DC>(cb) + x) * TR;
    }
    const int jb = max(cb * DC, c_lo);
    const int je = min(min(cb * DC + DC, c_hi), min(N - 1, r0 + TR - 1));  // columns with a row in the window
    if (jb >= je) return;
    const int t = threadIdx.x;
    for (int e = t; e < DC; e += DA_T) {
        const int jj = min(cb * DC + e, N - 1);
        double nn = 0.0;
#pragma unroll
        for (int q = 0; q < 15; ++q) nn = fma(P[(size_t)jj * 16 + q], P[(size_t)jj * 16 + q], nn);
        cn[e] = nn;
    }
    const int i = r0 - HALO + t;  // this thread's row
    const int ic = min(max(i, 0), N - 1);
    double pi[15];
#pragma unroll
    for (int q = 0; q < 15; ++q) pi[q] = P[(size_t)ic * 16 + q];
    double ni = 0.0;
#pragma unroll
    for (int q = 0; q < 15; ++q) ni = fma(pi[q], pi[q], ni);
    __syncthreads();
    for (int j0 = jb; j0 < je; j0 += NB) {
#pragma unroll
        for (int c = 0; c < NB; ++c) {
            const int j = j0 + c;
            if (j >= je) break;
            const double* pj = P + (size_t)j * 16;
            double dot = 0.0;
#pragma unroll
            for (int q = 0; q < 15; ++q) dot = fma(pi[q], pj[q], dot);
            const double nsum = ni + cn[j - cb * DC];
            double s = fma(-2.0, dot, nsum);
            if (s < 0x1p-20 * nsum) {  // near-identical cells: the difference form
                s = 0.0;
#pragma unroll
                for (int q = 0; q < 15; ++q) {
                    const double dv = pi[q] - pj[q];
                    s = fma(dv, dv, s);
                }
            }
            stage[c][t] = scc_sqrt_nr(s);
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NB; ++c) {
            const int j = j0 + c;
            if (j >= je) break;
            const long long B = (long long)j * (2LL * N - j - 1) / 2 - j - 1 - obase;  // out index of (i, j) = B + i
            const int delta = (int)((B + r0) & (HALO - 1));
            if constexpr (V2) {
                // two consecutive rows per thread, one 16-B (8-B for f32) store:
                // B + r0 - delta is a multiple of HALO, so an even t2 keeps the
                // pair aligned (out itself aligned, checked by the launcher)
                const int t2 = 2 * t;
                const int i2 = r0 - delta + t2;
                if (t2 < TR && i2 + 1 > j && i2 < N) {
                    const double v0 = stage[c][HALO - delta + t2], v1 = stage[c][HALO - delta + t2 + 1];
                    if (i2 > j && i2 + 1 < N) {
                        typedef float fv2 __attribute__((ext_vector_type(2)));
                        typedef double dv2 __attribute__((ext_vector_type(2)));
                        if (F32) {
                            const fv2 w = {(float)v0, (float)v1};
                            if (NT)
                                __builtin_nontemporal_store(w, (fv2*)((float*)out + B + i2));
                            else
                                *(fv2*)((float*)out + B + i2) = w;
                        } else {
                            const dv2 w = {v0, v1};
                            if (NT)
                                __builtin_nontemporal_store(w, (dv2*)((double*)out + B + i2));
                            else
                                *(dv2*)((double*)out + B + i2) = w;
                        }
                    } else {  // the column's first row or the matrix's last: one of the two
                        const int ir = i2 > j ? i2 : i2 + 1;
                        const double v = i2 > j ? v0 : v1;
                        if (ir < N) {
                            if (F32)
                                ((float*)out)[B + ir] = (float)v;
                            else
                                ((double*)out)[B + ir] = v;
                        }
                    }
                }
                continue;
            }
            const int i2 = r0 - delta + t;
            if (t < TR && i2 > j && i2 < N) {
                const double v = stage[c][HALO - delta + t];
                if (F32) {
                    if (NT)
                        __builtin_nontemporal_store((float)v, (float*)out + B + i2);
                    else
                        ((float*)out)[B + i2] = (float)v;
                } else {
                    if (NT)
                        __builtin_nontemporal_store(v, (double*)out + B + i2);
                    else
                        ((double*)out)[B + i2] = v;
                }
            }
        }
        __syncthreads();
    }
}

// Tile order for large N (the N x 16 scores past an XCD's 4 MB L2): panels of
// R row blocks (R * TR score rows, ~2 MB), each panel's column blocks in turn
// and the panel's row blocks inside a column block, the list cut into 8
// contiguous runs, one per XCD.  A panel's row scores stay in the XCD's L2
// while its column blocks pass, a column block's scores are fetched once per
// panel.  The folded grid fetched a tile's row scores from HBM for every
// column block: 20 GB of FETCH_SIZE under 160 GB of writes at config D.
// Lists are built once per (device, N, column range, shape) and cached.
struct DistTileList {
    int dev, N, c_lo, c_hi, DC, TR;
    int2* d;
    int n;
};
static std::mutex g_dtl_mu;
static std::vector<DistTileList> g_dtl;

template <int DC>
static const int2* dist_tile_list(int N, int c_lo, int c_hi, int TR, int nrb, int* count)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_dtl_mu);
    for (const DistTileList& t : g_dtl)
        if (t.dev == dev && t.N == N && t.c_lo == c_lo && t.c_hi == c_hi && t.DC == DC && t.TR == TR) {
            *count = t.n;
            return t.d;
        }
    const int cb_lo = c_lo / DC, cb_hi = (c_hi + DC - 1) / DC;
    const int R = std::max(8, (2 << 20) / (TR * 128));
    std::vector<int2> v;
    for (int p0 = 0; p0 < nrb; p0 += R)
        for (int cb = cb_lo; cb < cb_hi; ++cb) {
            const int rmin = (cb * DC + 1) / TR - 1;
            const int lo = std::max(std::max(rmin, 0), p0), hi = std::min(nrb, p0 + R);
            for (int rb = lo; rb < hi; ++rb) v.push_back(int2{cb, rb});
        }
    int2* d = nullptr;
    if (v.empty() || hipMalloc(&d, v.size() * sizeof(int2)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, v.data(), v.size() * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    if (g_dtl.size() >= 16) {  // (streamed column ranges: keep the newest lists)
        (void)hipFree(g_dtl.front().d);
        g_dtl.erase(g_dtl.begin());
    }
    g_dtl.push_back(DistTileList{dev, N, c_lo, c_hi, DC, TR, d, (int)v.size()});
    *count = (int)v.size();
    return d;
}

template <int DC, int NB, bool NT>
static void launch_dist_aligned(const double* P, int N, int c_lo, int c_hi, void* out, int f32, hipStream_t st)
{
    const int HALO = f32 ? 32 : 16, TR = DA_T - HALO;
    const int nrb = (N + HALO - 1) / TR + 1;
    const int cb_lo = c_lo / DC, cb_hi = (c_hi + DC - 1) / DC, ncbl = cb_hi - cb_lo;
    const long long obase = (long long)c_lo * (2LL * N - c_lo - 1) / 2;
    // the panel-ordered tile list from 64k cells (SCC_DIST_ORDER=0: the folded grid; bit-identical)
    const char* oe = getenv("SCC_DIST_ORDER");
    const int order = (oe && *oe) ? atoi(oe) : (N >= 65536 ? 1 : 0);
    const int2* tiles = nullptr;
    int ntiles = 0;
    if (order) tiles = dist_tile_list<DC>(N, c_lo, c_hi, TR, nrb, &ntiles);
    dim3 grid;
    if (tiles) {
        grid = dim3((unsigned)(8 * ((ntiles + 7) / 8)));
    } else {
        const int npair = (ncbl + 1) / 2;
        int gx = 1;
        for (int y = 0; y < npair; ++y) {
            const int a = cb_lo + y, b = cb_lo + ncbl - 1 - y;
            const int ra = f32 ? da_rbmin<DA_T - 32, DC>(a) : da_rbmin<DA_T - 16, DC>(a);
            const int rbb = f32 ? da_rbmin<DA_T - 32, DC>(b) : da_rbmin<DA_T - 16, DC>(b);
            const int cnt = (nrb - ra) + (b > a ? nrb - rbb : 0);
            gx = std::max(gx, cnt);
        }
        grid = dim3((unsigned)gx, (unsigned)npair);
    }
    // paired stores need the output 16-B aligned (8-B for f32); SCC_DIST_V2=0: one entry per thread
    const char* ve = getenv("SCC_DIST_V2");
    const bool v2 = !(ve && *ve && atoi(ve) == 0) && ((uintptr_t)out % (f32 ? 8 : 16)) == 0;
    const void* fn = f32 ? (v2 ? (const void*)k_dist_aligned<true, DC, NB, NT, true>
                               : (const void*)k_dist_aligned<true, DC, NB, NT, false>)
                         : (v2 ? (const void*)k_dist_aligned<false, DC, NB, NT, true>
                               : (const void*)k_dist_aligned<false, DC, NB, NT, false>);
    void* args[] = {(void*)&P,     (void*)&N,    (void*)&nrb, (void*)&cb_lo,   (void*)&ncbl, (void*)&c_lo,
                    (void*)&c_hi,  (void*)&obase, (void*)&out, (void*)&tiles, (void*)&ntiles};
    (void)hipLaunchKernel(fn, grid, dim3(DA_T), args, 0, st);
}

// ------------------------------------------------------------------ Pearson
// Z[c][u] = (x - mean_c) / sqrt(sum (x - mean_c)^2), fp32, padded to ldz
__global__ void __launch_bounds__(256) k_zscore(const double* __restrict__ Xc, int N, int nu, int ld, int ldz,
                                                float* __restrict__ Z)
{
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + scc_wave_id();
    if (c >= N) return;
    const double* row = Xc + (size_t)c * ld;
    dd s{0.0, 0.0};
    for (int u = lane; u < nu; u += 64) s = dd_add_d(s, row[u]);
    s = dd_wave_sum(s);
    const double mean = dd_div_n(s, (double)nu);
    dd ss{0.0, 0.0};
    for (int u = lane; u < nu; u += 64) {
        const double d = row[u] - mean;
        ss = dd_add_d(ss, d * d);
    }
    ss = dd_wave_sum(ss);
    const double inv = (ss.hi > 0.0) ? 1.0 / sqrt(ss.hi + ss.lo) : 0.0;
    for (int u = lane; u < ldz; u += 64) Z[(size_t)c * ldz + u] = (u < nu) ? (float)((row[u] - mean) * inv) : 0.0f;
}

// 1 - r on FP32 MFMA (v_mfma_f32_32x32x2_f32), one 128 x 128 tile of the
// lower triangle per workgroup (4 waves, 64 x 64 each = 2 x 2 blocks of 32 x 32).
//   * Operand roles: A = the tile's column cells j, B = its row cells i, so an
//     accumulator register holds D[j][i] with i = lane & 31: the epilogue's 32
//     lanes of a half-wave store 32 consecutive entries of one packed column
//     (R `dist` order is column-major, i contiguous) — two 256-byte runs per
//     store instruction instead of 32 scattered 8-byte writes.
//   * K (the union genes, zero padded to PK) streams in chunks of PK = 32
//     floats through two LDS buffers; chunk c + 1 is loaded from global into
//     registers while chunk c feeds the MFMAs, then written to the other buffer
//     (one barrier per chunk).  Rows past N are clamped to row N - 1 (their
//     results are never stored), so the loads carry no conditions.
//   * Fragments: lane half h reads the float4 at k = 8g + 4h of its row (LDS
//     row stride 36 floats: the 16-lane groups of a ds_read_b128 hit disjoint
//     banks), i.e. MFMA step s of group g pairs k = 8g + s (half 0) with
//     8g + 4 + s (half 1) — the same pairing for A and B, so the sum over k is
//     unchanged.
//   * Tiles are dealt to XCDs in contiguous runs of the row-major lower-
//     triangle enumeration (workgroup b runs on XCD b % 8), so an XCD's tiles
//     share their row blocks in its L2.
constexpr int PT = 128, PK = 32, PLD = PK + 4;

// Tile t of the lower triangle (ti >= tj, nt tile rows) in banded order: tile
// rows come in bands of PB; a band's rectangle left of its diagonal block is
// walked column by column (the PB row panels stay in L2 while the column
// panels stream), then its diagonal triangle row by row.  At ~32 resident
// workgroups per XCD the live tiles touch ~4 column panels + PB row panels.
constexpr int PB = 8;
__device__ __forceinline__ int2 pearson_tile(long long t, int nt)
{
    // band = (row-major tile row of t) / PB: bands are contiguous row ranges
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((long long)r * (r + 1) / 2 > t) --r;
    while ((long long)(r + 1) * (r + 2) / 2 <= t) ++r;
    const int b0 = (r / PB) * PB, R = min(PB, nt - b0);
    long long l = t - (long long)b0 * (b0 + 1) / 2;
    const long long rect = (long long)R * b0;
    // the diagonal triangle: row q with q(q+1)/2 <= l - rect
    const long long l2 = l - rect;
    int q = 0;
    while ((long long)(q + 1) * (q + 2) / 2 <= l2) ++q;
    const int ti = l < rect ? b0 + (int)(l % R) : b0 + q;
    const int tj = l < rect ? (int)(l / R) : b0 + (int)(l2 - (long long)q * (q + 1) / 2);
    return make_int2(ti, tj);
}

// the first tile at or after t (stepping by stride, below tend) that has a
// column in [c_lo, c_hi); returns tend if none
__device__ __forceinline__ long long pearson_next(long long t, long long tend, long long stride, int nt, int c_lo, int c_hi,
                                         int2& tile)
{
    for (; t < tend; t += stride) {
        const int2 tt = pearson_tile(t, nt);
        if (tt.y * PT + PT > c_lo && tt.y * PT < c_hi) {
            tile = tt;
            return t;
        }
    }
    return tend;
}

// Persistent: gridDim.x = 8 x (workgroups per XCD); the workgroups of XCD x
// stride through its contiguous run [x per, (x + 1) per) of the banded tile
// order.  The last K chunk of a tile prefetches chunk 0 of the workgroup's
// next tile, so the epilogue's stores and the next tile's first loads overlap
// instead of paying a workgroup launch and a cold first chunk per tile.
template <bool F32, bool NT>
__global__ void __launch_bounds__(256, 2) k_pearson_mfma(const float* __restrict__ Z, int N, int ldz, int nt, long long ntri,
                                                         long long per_xcd, int c_lo, int c_hi, long long obase,
                                                         void* __restrict__ out, int diag_nostore)
{
    const long long tbeg = (long long)(blockIdx.x & 7) * per_xcd;
    const long long tend = min(tbeg + per_xcd, ntri);
    const long long tstride = gridDim.x >> 3;
    int2 tt;
    long long t = pearson_next(tbeg + (blockIdx.x >> 3), tend, tstride, nt, c_lo, c_hi, tt);
    int ti = tt.x, tj = tt.y;
    if (t >= tend) return;

    __shared__ __attribute__((aligned(16))) float sA[2][PT * PLD];
    __shared__ __attribute__((aligned(16))) float sB[2][PT * PLD];
    const int tid = threadIdx.x, lane = tid & 63, w = scc_wave_id();
    const int h = lane >> 5, r32 = lane & 31;
    const int wj = (w >> 1) * 64, wi = (w & 1) * 64;

    // staging: thread tid moves float4 (tid & 7) of rows (tid >> 3) + 32 q;
    // offsets (floats) of the 4 staged rows of each panel, clamped to N - 1
    const int srow = tid >> 3, sc4 = (tid & 7) * 4;
    size_t oA0, oA1, oA2, oA3, oB0, oB1, oB2, oB3;
#define PEARSON_OFFSETS(I0_, J0_)                                                                             \
    do {                                                                                                      \
        oA0 = (size_t)min((J0_) + srow, N - 1) * ldz + sc4;                                                   \
        oA1 = (size_t)min((J0_) + srow + 32, N - 1) * ldz + sc4;                                              \
        oA2 = (size_t)min((J0_) + srow + 64, N - 1) * ldz + sc4;                                              \
        oA3 = (size_t)min((J0_) + srow + 96, N - 1) * ldz + sc4;                                              \
        oB0 = (size_t)min((I0_) + srow, N - 1) * ldz + sc4;                                                   \
        oB1 = (size_t)min((I0_) + srow + 32, N - 1) * ldz + sc4;                                              \
        oB2 = (size_t)min((I0_) + srow + 64, N - 1) * ldz + sc4;                                              \
        oB3 = (size_t)min((I0_) + srow + 96, N - 1) * ldz + sc4;                                              \
    } while (0)
    float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
#define PEARSON_GLOAD(k0)                              \
    do {                                               \
        ra0 = *(const float4*)(Z + oA0 + (k0));        \
        ra1 = *(const float4*)(Z + oA1 + (k0));        \
        ra2 = *(const float4*)(Z + oA2 + (k0));        \
        ra3 = *(const float4*)(Z + oA3 + (k0));        \
        rb0 = *(const float4*)(Z + oB0 + (k0));        \
        rb1 = *(const float4*)(Z + oB1 + (k0));        \
        rb2 = *(const float4*)(Z + oB2 + (k0));        \
        rb3 = *(const float4*)(Z + oB3 + (k0));        \
    } while (0)
#define PEARSON_LSTORE(buf)                                          \
    do {                                                             \
        *(float4*)&sA[buf][(srow) * PLD + sc4] = ra0;                \
        *(float4*)&sA[buf][(srow + 32) * PLD + sc4] = ra1;           \
        *(float4*)&sA[buf][(srow + 64) * PLD + sc4] = ra2;           \
        *(float4*)&sA[buf][(srow + 96) * PLD + sc4] = ra3;           \
        *(float4*)&sB[buf][(srow) * PLD + sc4] = rb0;                \
        *(float4*)&sB[buf][(srow + 32) * PLD + sc4] = rb1;           \
        *(float4*)&sB[buf][(srow + 64) * PLD + sc4] = rb2;           \
        *(float4*)&sB[buf][(srow + 96) * PLD + sc4] = rb3;           \
    } while (0)

    const int nchunk = (ldz + PK - 1) / PK;
    PEARSON_OFFSETS(ti * PT, tj * PT);
    PEARSON_GLOAD(0);
    PEARSON_LSTORE(0);
    __syncthreads();
    int buf = 0;
    const long long twoN = 2LL * N;
    for (;;) {
        const int I0 = ti * PT, J0 = tj * PT;
        int2 nn = make_int2(0, 0);
        const long long tn = pearson_next(t + tstride, tend, tstride, nt, c_lo, c_hi, nn);
        const int tin = nn.x, tjn = nn.y;
        f16v acc[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
        for (int c = 0; c < nchunk; ++c) {
            bool more = true;
            if (c + 1 < nchunk) {
                PEARSON_GLOAD((c + 1) * PK);
            } else if (tn < tend) {
                PEARSON_OFFSETS(tin * PT, tjn * PT);  // the next tile's chunk 0
                PEARSON_GLOAD(0);
            } else {
                more = false;
            }
            const float* A = sA[buf];
            const float* B = sB[buf];
            const int ng = min(PK, ldz - c * PK) / 8;  // 8-float groups of this chunk (the last may be short)
            // fragments of group g + 1 are read from LDS while group g's MFMAs
            // run (two waves per SIMD both waiting on LDS left the MFMA pipe idle)
            float4 fa0[2], fa1[2], fb0[2], fb1[2];
#define PEARSON_FRAG(S_, G_)                                                   \
    do {                                                                       \
        const int ko_ = 8 * (G_) + 4 * h;                                      \
        fa0[S_] = *(const float4*)&A[(wj + r32) * PLD + ko_];                  \
        fa1[S_] = *(const float4*)&A[(wj + 32 + r32) * PLD + ko_];             \
        fb0[S_] = *(const float4*)&B[(wi + r32) * PLD + ko_];                  \
        fb1[S_] = *(const float4*)&B[(wi + 32 + r32) * PLD + ko_];             \
    } while (0)
            PEARSON_FRAG(0, 0);
#pragma unroll
            for (int g = 0; g < PK / 8; ++g) {
                if (g >= ng) break;
                if (g + 1 < PK / 8 && g + 1 < ng) PEARSON_FRAG((g + 1) & 1, g + 1);
                const float4 a0 = fa0[g & 1], a1 = fa1[g & 1], b0 = fb0[g & 1], b1 = fb1[g & 1];
#define PEARSON_STEP(SEL)                                                                       \
    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.SEL, b0.SEL, acc[0][0], 0, 0, 0);          \
    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.SEL, b1.SEL, acc[0][1], 0, 0, 0);          \
    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.SEL, b0.SEL, acc[1][0], 0, 0, 0);          \
    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.SEL, b1.SEL, acc[1][1], 0, 0, 0)
                PEARSON_STEP(x);
                PEARSON_STEP(y);
                PEARSON_STEP(z);
                PEARSON_STEP(w);
#undef PEARSON_STEP
            }
#undef PEARSON_FRAG
            if (more) PEARSON_LSTORE(buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }

        if (diag_nostore) {  // diagnostic (SCC_PEARSON_NOSTORE=1): keep the result live, store nothing
            float x = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) x += acc[0][0][r] + acc[0][1][r] + acc[1][0][r] + acc[1][1][r];
            if (x == 12345.678f) ((float*)out)[0] = x;
        } else {
            // epilogue: D[j][i] -> 1 - r at packed (i, j), i > j, columns of this slice
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int j = J0 + wj + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (j < c_lo || j >= c_hi) continue;
                    const long long col = (long long)j * (twoN - j - 1) / 2 - j - 1 - obase;
#pragma unroll
                    for (int b = 0; b < 2; ++b) {
                        const int i = I0 + wi + 32 * b + r32;
                        if (i < N && j < i) {
                            const float d = 1.0f - acc[a][b][r];
                            if (F32) {
                                if (NT)
                                    __builtin_nontemporal_store(d, (float*)out + (col + i));
                                else
                                    ((float*)out)[col + i] = d;
                            } else {
                                if (NT)
                                    __builtin_nontemporal_store((double)d, (double*)out + (col + i));
                                else
                                    ((double*)out)[col + i] = (double)d;
                            }
                        }
                    }
                }
        }
        if (tn >= tend) break;
        t = tn;
        ti = tin;
        tj = tjn;
    }
#undef PEARSON_OFFSETS
#undef PEARSON_GLOAD
#undef PEARSON_LSTORE
}

// ------------------------------------------------------------------ launchers
extern "C" hipError_t scc_launch_union_map(int* umap, int G, const int* genes, int nu, hipStream_t st);

__global__ void k_umap(int* umap, const int* genes, int nu)
{
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u < nu) umap[genes[u]] = u;
}

extern "C" hipError_t scc_launch_union_map(int* umap, int G, const int* genes, int nu, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(umap, 0xFF, sizeof(int) * G, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_umap, dim3((nu + 255) / 256), dim3(256), 0, st, umap, genes, nu);
    return hipGetLastError();
}

// X[U, ] of cells [0, N) into Xc rows [0, N), rows [N, Npad) zero: the union
// map and the padding clear included (the LDS-map kernel builds its own map
// and writes the padding rows; the other forms get a global map and a memset)
extern "C" hipError_t scc_launch_gather(const i64* indptr, const int* rows, const double* vals, const double* dense,
                                        int G, int N, int Npad, int* umap, const int* genes, int nu, int ld,
                                        double* Xc, hipStream_t st)
{
    const bool lm = !dense && ld <= GATHER_LDS_LD && sizeof(double) * 4 * (size_t)ld + 2 * (size_t)G <= 120 * 1024 &&
                    !(getenv("SCC_GATHER_LM") && atoi(getenv("SCC_GATHER_LM")) == 0);
    if (!lm) {
        // the CSC gathers write whole rows when they stage them in LDS: only the padding then
        const size_t r0 = (dense || ld > GATHER_LDS_LD) ? 0 : (size_t)N;
        hipError_t e = hipSuccess;
        if ((size_t)Npad > r0) e = hipMemsetAsync(Xc + r0 * ld, 0, sizeof(double) * ((size_t)Npad - r0) * ld, st);
        if (e == hipSuccess && !dense) e = scc_launch_union_map(umap, G, genes, nu, st);
        if (e != hipSuccess) return e;
    }
    if (N <= 0 && !lm) return hipSuccess;
    if (dense)
        hipLaunchKernelGGL(k_gather_dense, dim3(2048), dim3(256), 0, st, dense, G, N, genes, nu, ld, Xc);
    else if (lm) {
        // waves per workgroup (4, 8 or 16 rows in LDS beside one copy of the
        // map): the most resident waves per CU (a wave per cell is latency
        // bound: indptr, then rows, then the hits' values), the fewer waves on a tie
        const int cus = scc_device_cus(256);
        const size_t mapb = (2 * (size_t)G + 15) & ~(size_t)15, cu_lds = 160 * 1024;
        int W = 4, best = 0;
        const char* ew = getenv("SCC_GATHER_W");
        for (int w = 4; w <= 16; w *= 2) {
            const size_t l = sizeof(double) * w * (size_t)ld + mapb;
            if (l > cu_lds) break;
            const int wgs = std::min((int)(cu_lds / l), 32 / w), res = wgs * w;
            if ((ew && atoi(ew) == w) || (!ew && res > best)) { W = w; best = res; }
        }
        const size_t lds = sizeof(double) * W * (size_t)ld + mapb;
        const int wgs = std::max(1, std::min((int)(cu_lds / lds), 32 / W));
        scc_set_lds((const void*)k_gather_csc_lm, (int)lds);
        const int grid = std::max(1, std::min((Npad + W - 1) / W, wgs * cus));
        hipLaunchKernelGGL(k_gather_csc_lm, dim3(grid), dim3(64 * W), lds, st, indptr, rows, vals, N, Npad, G, genes, nu,
                           ld, Xc);
    } else if (ld <= GATHER_LDS_LD)
        hipLaunchKernelGGL(k_gather_csc<true>, dim3((N + 3) / 4), dim3(256), sizeof(double) * 4 * (size_t)ld, st,
                           indptr, rows, vals, N, G, umap, ld, Xc);
    else
        hipLaunchKernelGGL(k_gather_csc<false>, dim3((N + 3) / 4), dim3(256), 0, st, indptr, rows, vals, N, G, umap,
                           ld, Xc);
    return hipGetLastError();
}

// apply 0: the column means only (the Gram and the scores subtract them on
// the fly: the same bits, one pass over X[U, ] fewer)
extern "C" hipError_t scc_launch_center(double* Xc, int N, int nu, int ld, dd* part, int nchunk, double* mean,
                                        int apply, hipStream_t st)
{
    const int rpc = (N + nchunk - 1) / nchunk;
    hipLaunchKernelGGL(k_colsum, dim3((ld + 255) / 256, nchunk), dim3(256), 0, st, Xc, N, ld, rpc, part);
    hipLaunchKernelGGL(k_colmean, dim3((ld + 3) / 4), dim3(256), 0, st, part, nchunk, ld, N, mean);
    if (apply) hipLaunchKernelGGL(k_center, dim3(4096), dim3(256), 0, st, Xc, N, nu, ld, mean);
    return hipGetLastError();
}

// one wave per column: the double-double column sum of rows [0, n) (partials
// of k_colsum folded in the order k_colmean uses), not divided
__global__ void __launch_bounds__(256) k_colsum_fold(const dd* __restrict__ part, int nchunk, int ld, int nu,
                                                     dd* __restrict__ out)
{
    const int u = blockIdx.x * 4 + scc_wave_id(), lane = threadIdx.x & 63;
    if (u >= nu) return;
    dd s{0.0, 0.0};
    for (int k = lane; k < nchunk; k += 64) s = dd_add(s, part[(size_t)k * ld + u]);
    s = dd_wave_sum_dpp(s);
    if (lane == 0) out[u] = s;
}

// mean[u] = (sum over ranks r, in rank order, of parts[r][u]) / N
__global__ void __launch_bounds__(256) k_mean_of_parts(const dd* __restrict__ parts, int nparts, int nu, int ld,
                                                       double N, double* __restrict__ mean)
{
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= ld) return;
    if (u >= nu) {
        mean[u] = 0.0;
        return;
    }
    dd s{0.0, 0.0};
    for (int r = 0; r < nparts; ++r) s = dd_add(s, parts[(size_t)r * nu + u]);
    mean[u] = dd_div_n(s, N);
}

extern "C" hipError_t scc_launch_colsum_dd(const double* Xc, int n, int ld, int nu, dd* part, int nchunk, dd* out,
                                           hipStream_t st)
{
    const int rpc = (n + nchunk - 1) / nchunk;
    hipLaunchKernelGGL(k_colsum, dim3((ld + 255) / 256, nchunk), dim3(256), 0, st, Xc, n, ld, rpc, part);
    hipLaunchKernelGGL(k_colsum_fold, dim3((nu + 3) / 4), dim3(256), 0, st, part, nchunk, ld, nu, out);
    return hipGetLastError();
}

// centre rows [0, n) of Xc with the mean of the ranks' column sums
extern "C" hipError_t scc_launch_center_parts(double* Xc, int n, int nu, int ld, const dd* parts, int nparts,
                                              double N, double* mean, hipStream_t st)
{
    hipLaunchKernelGGL(k_mean_of_parts, dim3((ld + 255) / 256), dim3(256), 0, st, parts, nparts, nu, ld, N, mean);
    hipLaunchKernelGGL(k_center, dim3(4096), dim3(256), 0, st, Xc, n, nu, ld, mean);
    return hipGetLastError();
}

// output tile width of the Gram: 128 from |U| > 384 (half the operand re-fetch)
extern "C" int scc_gram_tile_width(int ld) { return ld > 384 ? 128 : 64; }

// mean: centre on the fly (64-wide tiles only; the caller centred Xc otherwise)
extern "C" hipError_t scc_launch_gram(const double* Xc, int Npad, int ld, int nchunk, double* slabs, double* C,
                                      const double* mean, int nval, hipStream_t st)
{
    const int rpc = ((Npad + nchunk - 1) / nchunk + 3) & ~3;
    const int tw = scc_gram_tile_width(ld);
    if (mean && tw != 64) return hipErrorInvalidValue;
    if (tw == 128) {
        const int nt = (ld + 127) / 128;
        hipLaunchKernelGGL(k_gram_f64_128, dim3(gram_grid(nt * (nt + 1) / 2, nchunk)), dim3(256), 0, st, Xc, Npad,
                           ld, nt, nchunk, rpc, slabs);
    } else {
        const int ntile = ld / 64;
        hipLaunchKernelGGL(k_gram_f64, dim3(gram_grid(ntile * (ntile + 1) / 2, nchunk)), dim3(256), 0, st, Xc, Npad,
                           ld, ntile, nchunk, rpc, slabs, mean, nval);
    }
    hipLaunchKernelGGL(k_gram_reduce, dim3(2048), dim3(256), 0, st, slabs, nchunk, ld, C);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_scores(const double* Xc, int N, int nu, int ld, const double* Z16, int k, double* P,
                                        const double* mean, hipStream_t st)
{
    // fp64 MFMA form (SCC_SCORES_MFMA=0: one thread per cell)
    const char* mfe = getenv("SCC_SCORES_MFMA");
    const bool mf = !(mfe && *mfe && atoi(mfe) == 0);
    if (mf && ld % 64 == 0)
        hipLaunchKernelGGL(k_scores_mfma, dim3((N + 63) / 64), dim3(256), 0, st, Xc, N, nu, ld, Z16, k, P, mean);
    else
        hipLaunchKernelGGL(k_scores, dim3((N + 255) / 256), dim3(256), 0, st, Xc, N, nu, ld, Z16, k, P, mean);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_dist_euclid(const double* P, int N, int c_lo, int c_hi, void* out, int f32,
                                             hipStream_t st)
{
    if (N < 2 || c_hi <= c_lo) return hipSuccess;
    // columns per tile: 64, 128 from 64k cells (config D: 32.3 -> 31.5 ms; 16 / 32
    // columns 43.8 / 34.3 ms; config B: 64 columns 0.515 ms, 32: 0.535, 128:
    // 0.525); SCC_DIST_COLS forces either (bit-identical).  Nontemporal stores
    // (SCC_DIST_NT=0: plain; B 0.51 vs 0.54 ms).  Removed after measuring slower
    // at B / D: unaligned row tiles (0.69 / 38.1 ms), barrier-free wave windows
    // (0.59 ms), 256-column tiles (0.78 / 36.2 ms).  Columns per LDS stage (DA_NB):
    // B 8: 0.57-0.58 ms, 4: 0.566, 16: 0.69.  Two entries per thread in one
    // 16-B store (SCC_DIST_V2, default; the store phase's address and bound
    // VALU work halves): 0.552 ms.
    const char* env = getenv("SCC_DIST_COLS");
    const int cols = (env && *env) ? atoi(env) : (N >= 65536 ? 128 : 64);
    const char* nte = getenv("SCC_DIST_NT");
    const bool nt = !(nte && *nte && atoi(nte) == 0);
    if (cols == 128)
        nt ? launch_dist_aligned<128, DA_NB, true>(P, N, c_lo, c_hi, out, f32, st)
           : launch_dist_aligned<128, DA_NB, false>(P, N, c_lo, c_hi, out, f32, st);
    else
        nt ? launch_dist_aligned<64, DA_NB, true>(P, N, c_lo, c_hi, out, f32, st)
           : launch_dist_aligned<64, DA_NB, false>(P, N, c_lo, c_hi, out, f32, st);
    return hipGetLastError();
}

// ------------------------------------------------------------ host output
// Device-to-host copy on the CUs into pinned (host-coherent) memory: loads
// from HBM, nontemporal stores that leave over PCIe.  A bounded grid (256
// workgroups, four 16-B loads in flight per lane) reaches the link rate (55 GB/s measured, scripts/d2h_overlap.hip;
// the SDMA engine hipMemcpyAsync picks in a plain process gives 30 GB/s, and
// the runtime's own blit kernel, picked in a torch process, 54 GB/s with a
// 131072-thread grid).  W = the widest unit src and dst share the alignment
// of; the head and tail bytes go one per thread in workgroup 0.
typedef unsigned int d2h_u32x4 __attribute__((ext_vector_type(4)));
template <class T>
__global__ void __launch_bounds__(256) k_d2h(const char* __restrict__ src, char* __restrict__ dst, size_t head,
                                             size_t units, size_t n)
{
    const T* s = reinterpret_cast<const T*>(src + head);
    T* d = reinterpret_cast<T*>(dst + head);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < units; i += 4 * stride) {  // four loads in flight per lane
        const T v0 = s[i], v1 = s[i + stride], v2 = s[i + 2 * stride], v3 = s[i + 3 * stride];
        __builtin_nontemporal_store(v0, d + i);
        __builtin_nontemporal_store(v1, d + i + stride);
        __builtin_nontemporal_store(v2, d + i + 2 * stride);
        __builtin_nontemporal_store(v3, d + i + 3 * stride);
    }
    for (; i < units; i += stride) __builtin_nontemporal_store(s[i], d + i);
    if (blockIdx.x == 0) {
        const size_t tail0 = head + units * sizeof(T);
        for (size_t b = threadIdx.x; b < head; b += blockDim.x) dst[b] = src[b];
        for (size_t b = tail0 + threadIdx.x; b < n; b += blockDim.x) dst[b] = src[b];
    }
}

static int env_int_d2h() { return 256; }  // workgroups of the copy (32-1024 measured 53-55 GB/s alike)

extern "C" hipError_t scc_launch_d2h(const void* src, void* dst, size_t n, hipStream_t st)
{
    if (!n) return hipSuccess;
    const uintptr_t a = (uintptr_t)src, b = (uintptr_t)dst;
    const size_t w = ((a ^ b) & 15) == 0 ? 16 : ((a ^ b) & 7) == 0 ? 8 : ((a ^ b) & 3) == 0 ? 4 : 1;
    const size_t head = std::min(n, (size_t)((w - (a & (w - 1))) & (w - 1)));
    const size_t units = (n - head) / w;
    const int grid = (int)std::max<size_t>(1, std::min<size_t>((size_t)env_int_d2h(), (units + 255) / 256));
    const char* s = (const char*)src;
    char* d = (char*)dst;
    if (w == 16)
        hipLaunchKernelGGL(k_d2h<d2h_u32x4>, dim3(grid), dim3(256), 0, st, s, d, head, units, n);
    else if (w == 8)
        hipLaunchKernelGGL(k_d2h<unsigned long long>, dim3(grid), dim3(256), 0, st, s, d, head, units, n);
    else if (w == 4)
        hipLaunchKernelGGL(k_d2h<unsigned int>, dim3(grid), dim3(256), 0, st, s, d, head, units, n);
    else
        hipLaunchKernelGGL(k_d2h<unsigned char>, dim3(grid), dim3(256), 0, st, s, d, head, units, n);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_zscore(const double* Xc, int N, int nu, int ld, float* Z, int ldz, hipStream_t st)
{
    hipLaunchKernelGGL(k_zscore, dim3((N + 3) / 4), dim3(256), 0, st, Xc, N, nu, ld, ldz, Z);
    return hipGetLastError();
}

// Z holds the z-scores (scc_launch_zscore); Xc / ld are not read
extern "C" hipError_t scc_launch_pearson(const double* Xc, int N, int nu, int ld, float* Z, int ldz, int c_lo,
                                         int c_hi, void* out, int f32, hipStream_t st)
{
    if (ldz % 8 != 0 || ldz < nu || N < 2) return hipErrorInvalidValue;  // Z: N * ldz + 32 floats
    (void)Xc;
    (void)ld;
    const int nt = (N + PT - 1) / PT;
    const long long ntri = (long long)nt * (nt + 1) / 2;
    const long long per = (ntri + 7) / 8;
    // persistent grid: 2 workgroups per CU (LDS: 72 KB each), at most one per tile
    const long long nwg_xcd = per < 64 ? per : 64;
    const long long obase = (long long)c_lo * (2LL * N - c_lo - 1) / 2;
    const char* ns = getenv("SCC_PEARSON_NOSTORE");
    const int nostore = ns && ns[0] == '1';
    // nontemporal epilogue stores: off by default (measured at B: WRITE_SIZE
    // 3.11 GB/launch with them, 2.79 GB = 1.03x the 2.70 GB output without —
    // the L2 merges the partial lines that neighbouring tiles of one XCD write —
    // and 2.287 vs 2.267 ms); SCC_PEARSON_NT=1 turns them on
    const char* nte = getenv("SCC_PEARSON_NT");
    const bool ntst = nte && *nte && atoi(nte) != 0;
    const dim3 grid((unsigned)(8 * nwg_xcd));
    const void* fn = f32 ? (ntst ? (const void*)k_pearson_mfma<true, true> : (const void*)k_pearson_mfma<true, false>)
                         : (ntst ? (const void*)k_pearson_mfma<false, true> : (const void*)k_pearson_mfma<false, false>);
    int nti = nt;
    void* args[] = {(void*)&Z, (void*)&N, (void*)&ldz, (void*)&nti, (void*)&ntri, (void*)&per, (void*)&c_lo,
                    (void*)&c_hi, (void*)&obase, (void*)&out, (void*)&nostore};
    const hipError_t e = hipLaunchKernel(fn, grid, dim3(256), args, 0, st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}
