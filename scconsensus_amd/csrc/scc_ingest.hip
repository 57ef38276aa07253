// scc_ingest.hip — boundary ingest: the R dgCMatrix (CSC over cells, row
// indices sorted inside each column) or a dense column-major matrix, plus the
// per-cell cluster codes, become a gene-major array of orderable 64-bit value
// keys of the kept nonzeros, resident in HBM.  Replaces the reference's
// per-pair `as.matrix(dataMatrix)` and name-indexed column subsets
// (R/reclusterDEConsensusFast.R:361-368).
//
// Cells are visited in cluster order (host permutation `perm`: kept cells by
// code, then the unkept ones), in "count chunks" of <= 32 cells that never
// straddle two clusters.  Inside every gene segment the keys are therefore
// grouped by cluster: cluster a of gene g occupies
//     [cnt[cl_cc[a]][g], cnt[cl_cc[a+1]][g])     (offsets inside the segment)
// so per-cluster statistics are contiguous reductions and no code array is
// stored.  A block-local counting sort, no global atomics:
//   k_ing_hist     one workgroup per count chunk: LDS histogram over genes (kept
//                  nonzeros), nodg per cell (Fast:440-443, x > 0 over ALL
//                  cells), optional sum of expm1 over all entries (slow:36),
//                  non-finite / bad-row / unsorted-row flags, and each cell's
//                  entry boundaries at every gene tile (bnd)
//   k_ing_colscan  per gene: exclusive prefix over count chunks (in place);
//                  row nc = per-gene totals
//   scan           gene starts gstart[G+1]
//   k_ing_scatter  one workgroup per (scatter chunk of <= 4 count chunks of one
//                  cluster, gene tile): the tile's entries are counting-sorted
//                  by gene in LDS, then written out as per-gene runs (~15
//                  consecutive keys each at PBMC density) instead of 8-byte
//                  scattered stores.
#include "scc_common.hpp"
#include <algorithm>
#include "scc_kernels.hpp"

#define ING_T 256
#define IH_T (64 * SCC_ING_HIST_WAVES)  // k_ing_hist: one cell per wave at a time

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

// first k in [lo, hi) with rows[k] >= v (hi if none), rows[lo, hi) sorted: a
// 64-way search (one probe per lane and a ballot per round), wave-uniform result
__device__ inline i64 wave_lower_bound(const int* __restrict__ rows, i64 lo, i64 hi, int v)
{
    const int lane = threadIdx.x & 63;
    while (hi - lo > 64) {
        const i64 step = (hi - lo + 63) / 64;
        const i64 k = lo + (i64)lane * step;
        const bool ge = k < hi ? rows[k] >= v : true;
        const u64 m = __ballot(ge);
        const int f = m ? __builtin_ctzll(m) : 64;
        const i64 nlo = f == 0 ? lo : lo + (i64)(f - 1) * step + 1;
        hi = min(hi, lo + (i64)f * step);
        lo = nlo;
    }
    const i64 k = lo + lane;
    const bool ge = k < hi ? rows[k] >= v : true;
    const u64 m = __ballot(ge);
    return lo + (m ? __builtin_ctzll(m) : 64);
}

// err bits: 1 non-finite value, 2 row index out of range, 4 rows not sorted
//
// The chunk's gene histogram lives in LDS as 8-bit counters (a count chunk has
// <= kCountChunk = 32 cells, so a (chunk, gene) count is <= 32): gene l of the
// window goes to byte l / nwq of word l % nwq (nwq = ceil(window / 4)), so the
// consecutive genes of one cell's entries hit consecutive words (no two lanes
// of a wave add to one word unless their genes are nwq apart).  One window
// holds up to 4 * 40960 genes in 160 KB; a larger G is counted in windows of
// `hw` genes: the first pass reads every entry (nodg, expm1, input checks,
// tile boundaries, counts of window 0), later passes read each cell's entries
// of their window only (two wave-parallel binary searches; dense: the range).
template <bool DENSE>
__global__ void __launch_bounds__(IH_T) k_ing_hist(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                    const double* __restrict__ vals, int G, const int* __restrict__ perm,
                                                    const int* __restrict__ cc_p0, const int* __restrict__ cc_code,
                                                    int gt, int ntile, u32* __restrict__ cnt, i64* __restrict__ bnd,
                                                    int* __restrict__ nodg, dd* __restrict__ wave_expm1,
                                                    int want_expm1, int glo, int ghi, int rng_in, int hw,
                                                    const i64* __restrict__ tbnd, int* __restrict__ err)
{
    // rng_in 1: a gene-shard range of a validated dataset (below); 2: the whole
    // range of a validated dataset with no explicit zeros (FAST): the counts
    // need only the row indices (4 of the 12 bytes per stored value), nodg
    // comes from the dataset's cache and the value checks were done by the
    // validating read -- the CSC is then read once in full (by the scatter)
    const bool rng = rng_in == 1, ro = rng_in == 2;
    // genes outside [glo, ghi) (a shard of the gene rows) are not counted; nodg
    // and the expm1 sum still see every entry -- unless rng (a validated CSC
    // dataset, FAST mode): then each cell's entries of the tiles covering
    // [glo, ghi) are found by two wave-parallel binary searches (rows sorted)
    // and only those are read; nodg comes from the dataset's cache
    extern __shared__ __attribute__((aligned(16))) u32 hist[];
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    const int ch = blockIdx.x;
    const int a = cc_code[ch];
    const int p0 = cc_p0[ch], p1 = cc_p0[ch + 1];
    const int t0r = glo / gt, t1r = min(ntile, (ghi + gt - 1) / gt);  // rng: the tiles [t0r, t1r) cover [glo, ghi)
    // rng: the count rows cover only the shard's tiles [gb, ge) (zero outside
    // [glo, ghi) inside them: the scatter reads its tiles' edge genes); the
    // column scan runs over the same range and the rest of the row is never read
    const int gb = rng ? t0r * gt : 0, ge = rng ? min(G, t1r * gt) : G;
    const int nwin = (ge - gb + hw - 1) / hw;
    dd se{0.0, 0.0};
    int bad = 0;
    for (int win = 0; win < nwin; ++win) {
        const int wlo = gb + win * hw, whi = min(ge, wlo + hw);
        const int clo = max(glo, wlo), chi = min(ghi, whi);  // genes this pass counts
        const u32 nwq = (u32)(whi - wlo + 3) >> 2;
        const u64 mq = ((1ull << 40) + nwq - 1) / nwq;  // l / nwq = (l * mq) >> 40 for l < 2^18
        if (win > 0 && (a < 0 || clo >= chi)) continue;  // block-uniform
        if (a >= 0)
            for (u32 q = threadIdx.x; q < nwq; q += IH_T) hist[q] = 0;
        __syncthreads();
        for (int p = p0 + wv; p < p1; p += IH_T / 64) {
            const int c = perm[p];
            i64 b, e;
            cell_range<DENSE>(indptr, c, G, b, e);
            u32 pos = 0;
            i64* bp = bnd + (size_t)p * (ntile + 1);
            i64 kb = b, ke = e;
            if (win > 0) {  // counting only: this window's entries
                if (DENSE) {
                    kb = b + clo;
                    ke = b + chi;
                } else {
                    kb = wave_lower_bound(rows, b, e, clo);
                    ke = wave_lower_bound(rows, kb, e, chi);
                }
            } else if (!DENSE && rng) {
                if (tbnd) {  // the dataset's tile starts: two loads (the scatter reads the cache itself)
                    const i64* tb = tbnd + (size_t)c * (ntile + 1);
                    kb = tb[t0r];
                    ke = tb[t1r];
                } else {
                    kb = wave_lower_bound(rows, b, e, t0r * gt);
                    ke = wave_lower_bound(rows, kb, e, t1r * gt);
                }
            }
            const bool tiles_known = tbnd != nullptr;  // (rng or ro: the dataset's cache, read by the scatter)
            for (i64 k0 = kb; k0 < ke; k0 += 4 * 64) {  // four loads in flight per lane
                double xs[4];
                int gs[4], gps[4];
                // clamped unconditional loads + select (a load under a lane
                // condition becomes a branch with its own wait, one load at a time)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const i64 k = k0 + u * 64 + lane;
                    const i64 kc = k < ke ? k : ke - 1;  // k0 < ke, so ke - 1 >= b
                    const double x = ro ? 1.0 : vals[kc];
                    xs[u] = k < ke ? x : 0.0;
                    if (DENSE) {
                        gs[u] = k < ke ? (int)(k - b) : -1;
                        gps[u] = -1;
                    } else {
                        const int r = rows[kc];
                        const int rp = tiles_known ? -1 : rows[kc > b ? kc - 1 : b];
                        gs[u] = k < ke ? r : -1;
                        gps[u] = (k < ke && k > b) ? rp : -1;
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const i64 k = k0 + u * 64 + lane;
                    if (k >= ke) break;
                    const double x = xs[u];
                    const int g = gs[u];
                    if (a >= 0 && x != 0.0 && g >= clo && g < chi) {
                        const u32 l = (u32)(g - wlo);
                        const u32 q = (u32)(((u64)l * mq) >> 40);
                        atomicAdd(&hist[l - q * nwq], 1u << (8 * q));
                    }
                    if (win > 0) continue;
                    const bool gok = (g >= 0) & (g < G);
                    if (!ro) {
                        bad |= (!(x - x == 0.0) ? 1 : 0) | (gok ? 0 : 2) | ((x == 0.0 && gok) ? 0x1000 : 0);
                        pos += (x > 0.0);
                        if (want_expm1) se = dd_add_d(se, expm1(x));
                    }
                    if (!DENSE && a >= 0 && !tiles_known) {
                        // tile boundaries: tiles t in (tile(prev), tile(g)] start at k
                        const int gp = gps[u];
                        if (k > b && gp >= g) bad |= 4;
                        const int tp = (gp < 0) ? -1 : min(gp / gt, ntile - 1);
                        const int tg = gok ? g / gt : (g < 0 ? -1 : ntile - 1);
                        for (int t = tp + 1; t <= tg; ++t) bp[t] = k;
                    }
                }
            }
            if (win > 0) continue;
            if (!DENSE && a >= 0 && !tiles_known) {
                // tiles after the last entry read (and every tile of an empty cell) end
                // at ke (= e, or in rng mode the first entry past tile t1r - 1)
                const int gl = (ke > b) ? rows[ke - 1] : -1;
                const int tl = (gl < 0) ? -1 : min(gl / gt, ntile - 1);
                const int tend = rng ? t1r : ntile;
                for (int t = tl + 1 + lane; t <= tend; t += 64) bp[t] = ke;
            }
            pos = u32_wave_sum(pos);
            if (lane == 0 && !rng && !ro) nodg[c] = (int)pos;
        }
        if (a < 0) break;  // unkept chunk: side work only (one pass)
        __syncthreads();
        u32* row = cnt + (size_t)ch * G;
        for (int g = wlo + threadIdx.x; g < whi; g += IH_T) {
            const u32 l = (u32)(g - wlo);
            const u32 q = (u32)(((u64)l * mq) >> 40);
            row[g] = (hist[l - q * nwq] >> (8 * q)) & 0xFFu;  // genes outside [glo, ghi) count 0
        }
        __syncthreads();
    }
    if (want_expm1) {
        se = dd_wave_sum(se);
        if (lane == 0) wave_expm1[blockIdx.x * (IH_T / 64) + wv] = se;
    }
    if (bad) atomicOr(err, bad);
}

// The counting pass of a validated, zero-free dataset over all genes (FAST):
// row indices only (4 of the 12 bytes per stored value), the cells' tile
// starts from the dataset's cache (the scatter reads them there), nodg from
// the dataset's cache -- so only the counts remain: no value, boundary or
// check logic (k_ing_hist's 81 registers left one workgroup per CU; this one
// runs two).  Same histogram layout and count rows as k_ing_hist.
// A gene shard [glo, ghi) (rng) counts the genes of its range over its gene
// tiles [gb, ge) (count rows zero elsewhere in them, as k_ing_hist), each
// cell's entries of those tiles found from the tile-start cache tbnd.
__global__ void __launch_bounds__(IH_T) k_ing_count_ro(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                       int G, const int* __restrict__ perm,
                                                       const int* __restrict__ cc_p0, const int* __restrict__ cc_code,
                                                       int hw, int glo, int ghi, int gt, int ntile,
                                                       const i64* __restrict__ tbnd, u32* __restrict__ cnt)
{
    extern __shared__ __attribute__((aligned(16))) u32 hist[];
    const int lane = threadIdx.x & 63, wv = scc_wave_id();
    const int ch = blockIdx.x;
    if (cc_code[ch] < 0) return;  // unkept cells: nothing to count (block-uniform)
    const int p0 = cc_p0[ch], p1 = cc_p0[ch + 1];
    const bool rng = glo > 0 || ghi < G;
    const int t0r = glo / gt, t1r = min(ntile, (ghi + gt - 1) / gt);
    const int gb = rng ? t0r * gt : 0, ge = rng ? min(G, t1r * gt) : G;
    for (int wlo = gb; wlo < ge; wlo += hw) {
        const int whi = min(ge, wlo + hw);
        const int clo = max(glo, wlo), chi = min(ghi, whi);  // genes this pass counts
        const u32 nwq = (u32)(whi - wlo + 3) >> 2;
        const u64 mq = ((1ull << 40) + nwq - 1) / nwq;
        for (u32 q = threadIdx.x; q < nwq; q += IH_T) hist[q] = 0;
        __syncthreads();
        for (int p = p0 + wv; p < p1; p += IH_T / 64) {
            const int c = perm[p];
            i64 kb, ke;
            if (rng) {
                const i64* tb = tbnd + (size_t)c * (ntile + 1);
                kb = tb[t0r];
                ke = tb[t1r];
            } else {
                kb = indptr[c];
                ke = indptr[c + 1];
            }
            if (wlo > gb || whi < ge) {
                kb = wave_lower_bound(rows, kb, ke, wlo);
                ke = wave_lower_bound(rows, kb, ke, whi);
            }
            for (i64 k0 = kb; k0 < ke; k0 += 4 * 64) {
                int gs[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {  // clamped unconditional loads, all in flight
                    const i64 k = k0 + u * 64 + lane;
                    gs[u] = rows[k < ke ? k : ke - 1];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (k0 + u * 64 + lane < ke && gs[u] >= clo && gs[u] < chi) {
                        const u32 l = (u32)(gs[u] - wlo);
                        const u32 q = (u32)(((u64)l * mq) >> 40);
                        atomicAdd(&hist[l - q * nwq], 1u << (8 * q));
                    }
                }
            }
        }
        __syncthreads();
        u32* row = cnt + (size_t)ch * G;
        for (int g = wlo + threadIdx.x; g < whi; g += IH_T) {
            const u32 l = (u32)(g - wlo);
            const u32 q = (u32)(((u64)l * mq) >> 40);
            row[g] = (hist[l - q * nwq] >> (8 * q)) & 0xFFu;  // genes outside [glo, ghi) count 0
        }
        __syncthreads();
    }
}

// per gene: exclusive prefix over the count chunks (in place); rows >= nc_kept
// (unkept cells) hold the total.  Three passes over [segment of CS_SEG
// chunks] x [256 genes] blocks so the whole chip works on it.
#define CS_SEG 32
__global__ void __launch_bounds__(256) k_ing_colsum(const u32* __restrict__ cnt, int nc_kept, int G, int gb, int ge,
                                                    u32* __restrict__ part)
{
    const int g = gb + blockIdx.y * 256 + threadIdx.x;
    if (g >= ge) return;
    const int w0 = blockIdx.x * CS_SEG, w1 = min(nc_kept, w0 + CS_SEG);
    u32 s = 0;
    for (int w = w0; w < w1; ++w) s += cnt[(size_t)w * G + g];
    part[(size_t)blockIdx.x * G + g] = s;
}

// 64 genes per workgroup (a lane per gene: coalesced rows), the segments cut
// into 16 runs, one per wave: each wave sums its run, the waves' sums are
// scanned in LDS, and each wave rewrites its run from its offset.  (A thread
// per gene walking every segment was a chain of nseg dependent loads: 48 us
// for a gene shard of config D; a wave per gene broke the chain but read each
// line for one 4-byte value, 15x the part array at config E.)
#define SS_T 1024
__global__ void __launch_bounds__(SS_T) k_ing_segscan(u32* __restrict__ part, int nseg, int G, int gb, int ge,
                                                      u32* __restrict__ total)
{
    __shared__ u32 ws[SS_T / 64][64];
    const int lane = threadIdx.x & 63, w = scc_wave_id();
    const int g = gb + blockIdx.x * 64 + lane;
    const bool ok = g < ge;
    const int per = (nseg + SS_T / 64 - 1) / (SS_T / 64);
    const int q0 = min(nseg, w * per), q1 = min(nseg, q0 + per);
    u32 s = 0;
    if (ok)
        for (int q = q0; q < q1; ++q) s += part[(size_t)q * G + g];
    ws[w][lane] = s;
    __syncthreads();
    u32 run = 0;
    for (int v = 0; v < w; ++v) run += ws[v][lane];
    if (ok) {
        for (int q = q0; q < q1; ++q) {
            const u32 v = part[(size_t)q * G + g];
            part[(size_t)q * G + g] = run;
            run += v;
        }
        if (w == SS_T / 64 - 1) total[g] = run;
    }
}

__global__ void __launch_bounds__(256) k_ing_colapply(u32* __restrict__ cnt, int nc, int nc_kept, int G, int gb,
                                                      int ge, const u32* __restrict__ part,
                                                      const u32* __restrict__ total)
{
    const int g = gb + blockIdx.y * 256 + threadIdx.x;
    if (g >= ge) return;
    const int w0 = blockIdx.x * CS_SEG;
    // Unkept chunks add nothing.  Of their rows only nc_kept (the end offset of
    // the last kept cluster, cl_cc[K]) and the totals row nc are ever read, so
    // only those two are written (at 1M cells with half the cells unkept the
    // rest would be > 1 GB of dead stores per run).
    if (w0 >= nc_kept) {
        const u32 tot = total[g];
        if (nc_kept >= w0 && nc_kept < w0 + CS_SEG) cnt[(size_t)nc_kept * G + g] = tot;
        if (nc != nc_kept && nc >= w0 && nc < w0 + CS_SEG) cnt[(size_t)nc * G + g] = tot;
        return;
    }
    u32 run = part[(size_t)blockIdx.x * G + g];
    const int w1 = min(nc_kept, w0 + CS_SEG);
    for (int w = w0; w < w1; ++w) {
        const u32 v = cnt[(size_t)w * G + g];
        cnt[(size_t)w * G + g] = run;
        run += v;
    }
    if (w1 == nc_kept) {
        const u32 tot = total[g];
        if (nc_kept < w0 + CS_SEG) cnt[(size_t)nc_kept * G + g] = tot;
        if (nc != nc_kept && nc < w0 + CS_SEG) cnt[(size_t)nc * G + g] = tot;
    }
}

#define SC_GT 256       // genes per tile
#define SC_CAP 4096     // default staged entries per round (u64 key + u16 gene = 10 B each): 3 blocks per CU
#define SC_CMAX 256     // cells per scatter chunk (kScatterCC * kCountChunk; <= ING_T: a thread per cell)
#define SC_RUN 8        // consecutive gene tiles of one chunk dealt to one XCD (SCC_SC_RUN)

template <bool DENSE, int U>
__global__ void __launch_bounds__(ING_T) k_ing_scatter(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                       const double* __restrict__ vals, int G,
                                                       const int* __restrict__ perm, const int* __restrict__ cc_p0,
                                                       const int* __restrict__ sc_cc0, const u32* __restrict__ cnt,
                                                       const i64* __restrict__ gstart, const i64* __restrict__ bnd,
                                                       const i64* __restrict__ tbnd, int ntile, int cap, int glo,
                                                       int ghi, int t0, int nsc, int ntl, int run,
                                                       u64* __restrict__ keys)
{
    __shared__ u32 loff[SC_GT + 1];
    __shared__ u32 cur[SC_GT];
    __shared__ u32 lcnt[SC_GT];
    __shared__ i64 gdst[SC_GT];
    __shared__ i64 ckb[SC_CMAX];
    __shared__ u32 cof[SC_CMAX + 1];
    __shared__ int rnd[SC_GT + 2];
    __shared__ int nrnd;
    __shared__ u32 wsum[ING_T / 64];
    __shared__ u32 csum[ING_T / 64];
    extern __shared__ __attribute__((aligned(16))) u64 skey[];  // [SC_CAP]
    unsigned short* sg = (unsigned short*)(skey + cap);        // [cap]
    const int tid = threadIdx.x, lane = tid & 63, wv = scc_wave_id();
    // dispatch slot -> (scatter chunk, gene tile): slot x runs on XCD x % 8, and
    // runs of SC_RUN consecutive tiles of one chunk share an XCD, so the cache
    // line a cell's entries of tiles t and t + 1 share is fetched once into
    // that XCD's L2 instead of twice from HBM
    const long long lin = blockIdx.x, kq = lin >> 3, xq = lin & 7;
    const long long L = ((kq / run) * 8 + xq) * run + kq % run;
    if (L >= (long long)nsc * ntl) return;
    const int s = (int)(L / ntl), t = t0 + (int)(L % ntl);  // gene tiles from t0 (a gene shard's tiles)
    const int g0 = t * SC_GT, g1 = min(G, g0 + SC_GT), ng = g1 - g0;
    const int cc0 = sc_cc0[s], cc1 = sc_cc0[s + 1];
    const int p0 = cc_p0[cc0], p1 = cc_p0[cc1];
    const int ncell = p1 - p0;  // <= SC_CMAX
    // ---- cell ranges inside this gene tile (all loads issued together)
    u32 clen = 0;
    if (tid < ncell) {
        const int c = perm[p0 + tid];
        i64 kb, ke;
        if (DENSE) {
            kb = (i64)c * G + g0;
            ke = kb + ng;
        } else {
            // clamp: bnd is only trustworthy when the hist pass saw sorted
            // rows (err bit 4 otherwise); reads must stay in bounds anyway
            // (the run's boundaries by cell order, or the dataset's cache by cell)
            const i64* bp = tbnd ? tbnd + (size_t)c * (ntile + 1) : bnd + (size_t)(p0 + tid) * (ntile + 1);
            const i64 cb = indptr[c], ce = indptr[c + 1];
            kb = min(max(bp[t], cb), ce);
            ke = min(max(bp[t + 1], kb), ce);
        }
        ckb[tid] = kb;
        clen = (u32)(ke - kb);
    }
    // ---- per gene counts and destinations of this (chunk, tile): 2 genes per thread
    u32 myc[2];
    for (int h = 0; h < 2; ++h) {
        const int gl = 2 * tid + h;
        myc[h] = 0;
        if (gl < ng) {
            const int g = g0 + gl;
            const u32 o0 = cnt[(size_t)cc0 * G + g];
            myc[h] = cnt[(size_t)cc1 * G + g] - o0;
            gdst[gl] = gstart[g] + o0;
        }
        if (gl < SC_GT) lcnt[gl] = myc[h];
    }
    // inclusive scans: gene counts (2 per thread) and cell lengths
    u32 inc = myc[0] + myc[1], cinc = clen;
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(inc, o, 64), z = __shfl_up(cinc, o, 64);
        if (lane >= o) {
            inc += y;
            cinc += z;
        }
    }
    if (lane == 63) {
        wsum[wv] = inc;
        csum[wv] = cinc;
    }
    __syncthreads();
    for (int v = 0; v < wv; ++v) {
        inc += wsum[v];
        cinc += csum[v];
    }
    if (2 * tid < SC_GT) {
        loff[2 * tid + 1] = inc - myc[1];
        loff[2 * tid + 2] = inc;
    }
    if (tid == 0) {
        loff[0] = 0;
        cof[0] = 0;
    }
    if (tid < ncell) cof[tid + 1] = cinc;
    __syncthreads();
    // rounds of <= cap entries over consecutive genes
    if (tid == 0) {
        const u32 tot = loff[ng];
        int nr = 0;
        rnd[0] = 0;
        if (tot <= (u32)cap) {
            nr = 1;
            rnd[1] = ng;
        } else {
            u32 acc = 0;
            for (int gl = 0; gl < ng; ++gl) {
                if (acc + lcnt[gl] > (u32)cap) {
                    rnd[++nr] = gl;
                    acc = 0;
                }
                acc += lcnt[gl];
            }
            rnd[++nr] = ng;
        }
        nrnd = nr;
    }
    __syncthreads();
    const int nr = nrnd;
    const u32 E = cof[ncell];  // stored entries of the tile (zeros included for dense input)
    for (int r = 0; r < nr; ++r) {
        const int r0 = rnd[r], r1 = rnd[r + 1];
        const u32 base = loff[r0];
        for (int gl = tid; gl < SC_GT; gl += ING_T) cur[gl] = 0;
        __syncthreads();
        // each wave takes 4 cells at a time, lanes over a cell's entries in the
        // tile (~60 at PBMC density); the 4 first chunks' loads are in flight together
        auto put = [&](double x, int gq) {
            if (x != 0.0 && gq >= r0 && gq < r1 && g0 + gq >= glo && g0 + gq < ghi) {
                const u32 o = atomicAdd(&cur[gq], 1u);
                if (o < lcnt[gq]) {  // always, for valid input
                    const u32 pos = loff[gq] - base + o;
                    skey[pos] = scc_key_of(x);
                    sg[pos] = (unsigned short)gq;
                }
            }
        };
        // lanes over the tile's entries as one flat range (entry e of the tile is
        // entry e - cof[c] of cell c, found by a binary search of cof): every
        // lane loads, however few entries a cell has in the tile (~8 at 1M-cell
        // density; a lane per cell entry left most lanes idle)
        for (u32 e0 = (u32)wv * (64 * U); e0 < E; e0 += U * ING_T) {
            double x[U];
            int gq[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                // clamped to the last entry (e0 < E) so the loads are
                // unconditional and all four stay in flight (as in k_ing_hist)
                const u32 e = e0 + (u32)(u * 64 + lane);
                const u32 ec = e < E ? e : E - 1;
                int lo = 0, hi = ncell;  // last cell c with cof[c] <= ec
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (cof[mid] <= ec) lo = mid;
                    else hi = mid;
                }
                const u32 j = ec - cof[lo];
                const i64 k = ckb[lo] + j;
                const double xv = vals[k];
                const int gv = DENSE ? (int)j : rows[k] - g0;
                x[u] = e < E ? xv : 0.0;
                gq[u] = e < E ? gv : -1;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) put(x[u], gq[u]);
        }
        __syncthreads();
        const int Er = (int)(loff[r1] - base);
        for (int i = tid; i < Er; i += ING_T) {
            const int gq = sg[i];
            keys[gdst[gq] + (i64)(i - (int)(loff[gq] - base))] = skey[i];
        }
        __syncthreads();
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

// ------------------------------------------------------------ per-run clears
// One launch for the DE run's small clears (error words, work counters), the
// rank accumulators and the first-occurrence keys (~0): four fill launches
// before, each ~5 us on the stream at config B.
__global__ void __launch_bounds__(256) k_de_clear(int* __restrict__ err, int* __restrict__ counts,
                                                  unsigned long long* __restrict__ acc, long long acc_n,
                                                  unsigned long long* __restrict__ first, int G, int glo, int ghi)
{
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x, stride = (long long)gridDim.x * 256;
    if (t < 4) err[t] = 0;
    if (t < SCC_NCOUNTS) counts[SCC_CNT_STRIDE * t] = 0;
    if (acc && glo == 0 && ghi == G) {
        typedef unsigned long long u2v __attribute__((ext_vector_type(2)));
        for (long long e = t; e < acc_n / 2; e += stride) ((u2v*)acc)[e] = u2v{0ull, 0ull};
        if ((acc_n & 1) && t == 0) acc[acc_n - 1] = 0ull;
    } else if (acc && ghi > glo) {
        // a gene shard: the accumulator rows' [glo, ghi) columns (the rank
        // stage and the test touch no other gene)
        const long long w = ghi - glo, n = (acc_n / G) * w;
        for (long long e = t; e < n; e += stride) acc[(e / w) * G + glo + e % w] = 0ull;
    }
    if (first)
        for (long long e = t; e < G; e += stride) first[e] = ~0ull;
}

extern "C" hipError_t scc_launch_de_clear(int* err, int* counts, unsigned long long* acc, long long acc_n,
                                          unsigned long long* first, int G, int glo, int ghi, hipStream_t st)
{
    const long long accw = !acc ? 0ll : (glo == 0 && ghi == G) ? acc_n / 2 : (acc_n / G) * std::max(0, ghi - glo);
    const long long work = std::max(accw, (long long)G);
    const int grid = (int)std::max(1ll, std::min(4096ll, (work + 255) / 256));
    hipLaunchKernelGGL(k_de_clear, dim3(grid), dim3(256), 0, st, err, counts, acc, acc_n, first, G, glo, ghi);
    return hipGetLastError();
}

// ------------------------------------------------------------ host launchers
extern "C" int scc_ingest_gene_tile(void) { return SC_GT; }

// genes per histogram window: 4 per LDS word, at most 160 KB of words
// (SCC_HIST_WINDOW overrides it, a test knob for the windowed path)
extern "C" int scc_ingest_hist_window(int G)
{
    const char* v = getenv("SCC_HIST_WINDOW");
    const int forced = (v && *v) ? atoi(v) : 0;
    const int cap = forced > 0 ? std::min(forced, 4 * 40960) : 4 * 40960;
    return std::max(1, std::min(G, cap));
}

// Every cell's gene-tile starts (tb[c][t] = first entry of cell c with row >=
// t * gt, tb[c][ntile] = the cell's end): a wave per cell over its row
// indices, the same rule k_ing_hist applies while it counts.
__global__ void __launch_bounds__(256) k_ing_tile_bounds(const i64* __restrict__ indptr, const int* __restrict__ rows,
                                                         int N, int gt, int ntile, i64* __restrict__ tbnd)
{
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + scc_wave_id();
    if (c >= N) return;
    const i64 b = indptr[c], e = indptr[c + 1];
    i64* tb = tbnd + (size_t)c * (ntile + 1);
    for (i64 k = b + lane; k < e; k += 64) {
        const int g = rows[k];
        const int gp = k > b ? rows[k - 1] : -1;
        const int tp = gp < 0 ? -1 : min(gp / gt, ntile - 1);
        const int tg = min(max(g, 0) / gt, ntile - 1);
        for (int t = tp + 1; t <= tg; ++t) tb[t] = k;
    }
    const int gl = e > b ? rows[e - 1] : -1;
    const int tl = gl < 0 ? -1 : min(max(gl, 0) / gt, ntile - 1);
    for (int t = tl + 1 + lane; t <= ntile; t += 64) tb[t] = e;
}

extern "C" hipError_t scc_launch_tile_bounds(const i64* indptr, const int* rows, int N, int gt, int ntile, i64* tbnd,
                                             hipStream_t st)
{
    if (N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ing_tile_bounds, dim3((N + 3) / 4), dim3(256), 0, st, indptr, rows, N, gt, ntile, tbnd);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_ingest_hist(const i64* indptr, const int* rows, const double* vals,
                                             const double* dense, int G, const int* perm, const int* cc_p0,
                                             const int* cc_code, int nc, int ntile, u32* cnt, i64* bnd, int* nodg,
                                             dd* wave_expm1, int want_expm1, int glo, int ghi, int rng,
                                             const i64* tbnd, int* err, hipStream_t st)
{
    const int hw = scc_ingest_hist_window(G);
    const size_t lds = sizeof(u32) * (size_t)((hw + 3) / 4);
    if (dense) {
        scc_set_lds((const void*)k_ing_hist<true>, (int)lds);
        hipLaunchKernelGGL((k_ing_hist<true>), dim3(nc), dim3(IH_T), lds, st, nullptr, nullptr, dense, G, perm, cc_p0,
                           cc_code, SC_GT, ntile, cnt, bnd, nodg, wave_expm1, want_expm1, glo, ghi, 0, hw, nullptr,
                           err);
    } else {
        scc_set_lds((const void*)k_ing_hist<false>, (int)lds);
        hipLaunchKernelGGL((k_ing_hist<false>), dim3(nc), dim3(IH_T), lds, st, indptr, rows, vals, G, perm, cc_p0,
                           cc_code, SC_GT, ntile, cnt, bnd, nodg, wave_expm1, want_expm1, glo, ghi, rng, hw, tbnd,
                           err);
    }
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_ingest_count_ro(const i64* indptr, const int* rows, int G, const int* perm,
                                                 const int* cc_p0, const int* cc_code, int nc, int glo, int ghi,
                                                 const i64* tbnd, u32* cnt, hipStream_t st)
{
    if ((glo > 0 || ghi < G) && !tbnd) return hipErrorInvalidValue;
    const int hw = scc_ingest_hist_window(G);
    const size_t lds = sizeof(u32) * (size_t)((hw + 3) / 4);
    const int ntile = (G + SC_GT - 1) / SC_GT;
    scc_set_lds((const void*)k_ing_count_ro, (int)lds);
    hipLaunchKernelGGL(k_ing_count_ro, dim3(nc), dim3(IH_T), lds, st, indptr, rows, G, perm, cc_p0, cc_code, hw, glo,
                       ghi, SC_GT, ntile, tbnd, cnt);
    return hipGetLastError();
}

extern "C" int scc_ingest_colscan_scratch(int nc, int G) { return ((nc + 1 + CS_SEG - 1) / CS_SEG + 1) * G; }

// genes [g0, g1) of the count rows (a gene shard's tiles in range mode,
// scc_ingest_count_range; all genes otherwise)
extern "C" hipError_t scc_launch_ingest_colscan(u32* cnt, int nc, int nc_kept, int G, int g0, int g1, u32* scratch,
                                                hipStream_t st)
{
    if (g1 <= g0) return hipSuccess;
    const int nseg_k = (nc_kept + CS_SEG - 1) / CS_SEG;
    const int nseg_all = (nc + 1 + CS_SEG - 1) / CS_SEG;
    u32* part = scratch;
    u32* total = scratch + (size_t)nseg_all * G;
    const int gbk = (g1 - g0 + 255) / 256;
    if (nseg_k > 0)
        hipLaunchKernelGGL(k_ing_colsum, dim3(nseg_k, gbk), dim3(256), 0, st, cnt, nc_kept, G, g0, g1, part);
    hipLaunchKernelGGL(k_ing_segscan, dim3((g1 - g0 + 63) / 64), dim3(SS_T), 0, st, part, nseg_k, G, g0, g1, total);
    hipLaunchKernelGGL(k_ing_colapply, dim3(nseg_all, gbk), dim3(256), 0, st, cnt, nc, nc_kept, G, g0, g1, part,
                       total);
    return hipGetLastError();
}

// the genes whose count rows a range-mode (rng) counting pass writes: the
// gene tiles covering [glo, ghi)
extern "C" void scc_ingest_count_range(int G, int glo, int ghi, int* g0, int* g1)
{
    const int ntile = (G + SC_GT - 1) / SC_GT;
    *g0 = (glo / SC_GT) * SC_GT;
    *g1 = std::min(G, std::min(ntile, (ghi + SC_GT - 1) / SC_GT) * SC_GT);
}

extern "C" hipError_t scc_launch_ingest_scatter(const i64* indptr, const int* rows, const double* vals,
                                                const double* dense, int G, const int* perm, const int* cc_p0,
                                                const int* sc_cc0, int ns, const u32* cnt, const i64* gstart,
                                                const i64* bnd, const i64* tbnd, int ntile, int glo, int ghi,
                                                u64* keys, hipStream_t st)
{
    if (ns <= 0 || ghi <= glo) return hipSuccess;
    const int t0 = glo / SC_GT, t1 = (ghi + SC_GT - 1) / SC_GT;  // the gene tiles of [glo, ghi)
    const int ntl = t1 - t0;
    static const int run = [] {
        const char* v = getenv("SCC_SC_RUN");
        return (v && *v) ? std::max(1, atoi(v)) : SC_RUN;
    }();
    const long long nrun = ((long long)ns * ntl + run - 1) / run;
    const dim3 grid((unsigned)(((nrun + 7) / 8) * 8 * run));
    static const int cap = [] {
        const char* v = getenv("SCC_SC_CAP");
        return (v && *v) ? std::max(SC_GT, atoi(v)) : SC_CAP;
    }();
    const size_t lds = (size_t)cap * (8 + 2);
    // (4 loads in flight per lane: 8 and 16 measured slower at config B)
    scc_set_lds((const void*)k_ing_scatter<true, 4>, (int)lds);
    scc_set_lds((const void*)k_ing_scatter<false, 4>, (int)lds);
    if (dense)
        hipLaunchKernelGGL((k_ing_scatter<true, 4>), grid, dim3(ING_T), lds, st, nullptr, nullptr, dense, G, perm,
                           cc_p0, sc_cc0, cnt, gstart, bnd, nullptr, ntile, cap, glo, ghi, t0, ns, ntl, run, keys);
    else
        hipLaunchKernelGGL((k_ing_scatter<false, 4>), grid, dim3(ING_T), lds, st, indptr, rows, vals, G, perm, cc_p0,
                           sc_cc0, cnt, gstart, bnd, tbnd, ntile, cap, glo, ghi, t0, ns, ntl, run, keys);
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
