// scc_csr.hip — gene-major CSR input (genes x cells, per gene strictly
// ascending cell columns: scipy.sparse.csr_matrix / an AnnData .X transposed,
// R's dgRMatrix; BASELINE config E's "1M-cell sparse CSR input") turned into
// the engine's resident layout, the dgCMatrix CSC over cells that R hands the
// reference (R/reclusterDEConsensusFast.R:368 `as.matrix(dataMatrix)` consumes
// it).  Run once when the dataset is created.
//
// A sparse transpose is a stable sort of the entries by cell.  Done in one
// scatter, every (gene tile, cell) run is a few entries long and lands at its
// own place in the output: at config E (1M cells, 20k genes, 3.3 % dense) the
// round-5 kernel moved 56 GB of partial-line writes for a 7.8 GB CSC.  Here
// the transpose is two coalesced passes through an intermediate:
//   k_ct_bounds  the columns streamed once (a wave per 8192 entries):
//                validated (in [0, N), strictly ascending within a gene), and
//                where each superblock of SB cells starts in each row (u32,
//                row-relative; k_ct_btail fills the superblocks past a row's end)
//   k_ct_tiles   per tile of 256 genes: entries per (tile, superblock), their
//                scan (a region's offset inside the tile's output), tile sums
//   k_ct_pass1   one workgroup per (tile, superblock) region: the 256 genes'
//                row pieces in the superblock read as one flattened,
//                coalesced stream into registers, ranked inside each cell by a
//                256-bit gene mask per cell in LDS (popcounts: the gene order),
//                and written cell-major into the region's contiguous slot of
//                the intermediate (10 B per entry: the value and a u16 of (cell
//                in its output group, gene in tile)); each output group's start
//                inside the tile is recorded (OFF), each cell's entries added
//                to its total (one atomic per (region, cell))
//   scan         cell totals -> the CSC indptr
//   k_ct_pass2   one workgroup per output group of CG cells: the group's run
//                from every tile (contiguous, in tile order) read into
//                registers; per (tile, cell) counts in LDS give each entry its
//                slot (the cell's entries in earlier tiles + its place in its
//                tile's cell segment), and the group's stretch of the CSC
//                (rows, values: contiguous) is written from the registers
// Within a cell the rows come out ascending (tiles in order, genes of a tile
// in order): exactly the dgCMatrix R would hold.  Minimum traffic: the CSR read
// (12 B per entry) and the CSC written (12 B); these passes move ~48 B per
// entry (the columns read twice, the 10-B intermediate written and read), in
// whole-line runs (XCD-contiguous workgroup orders keep a region's neighbours
// on one L2; a workgroup's scattered stores fill a stretch of a few tens of KB
// within its lifetime).
#include "scc_common.hpp"
#include "scc_kernels.hpp"

#include <algorithm>

#define CT_TG 256          // genes per tile (pass 1: one thread per gene, a 4 x 64-bit gene mask per cell)
#define CT_T1 256          // pass-1 threads
#define CT_KPT1 12         // pass-1 entries per thread per piece (held in registers)
#define CT_WMAX 1024       // widest superblock (cells)
#define CT_T2 256          // pass-2 threads
#define CT_KPT2 16         // pass-2 entries per thread per chunk (held in registers)
#define CT_TCMAX 1024      // pass-2 (tile, cell) counters in LDS
#define CT_GMAX (CT_TG * CT_TCMAX)  // genes the transpose takes (262,144)

typedef unsigned short u16;

struct CtArgs {
    int G, N, SB, NS, T, CG, NG;
    const u32* bnd;  // [G][NS + 1]
    const u32* rs;   // [T][NS]
    const i64* ts;   // [T + 1]
    u32* off;        // [T][NG + 1]
    u16* meta;       // [nnz]
    double* ival;    // [nnz]
};

static CtArgs ct_args(const ScCsrPlan* P, void* scratch)
{
    char* b = (char*)scratch;
    CtArgs A;
    A.G = (int)P->G;
    A.N = (int)P->N;
    A.SB = P->SB;
    A.NS = P->NS;
    A.T = P->T;
    A.CG = P->CG;
    A.NG = P->NG;
    A.bnd = (const u32*)(b + P->off_bnd);
    A.rs = (const u32*)(b + P->off_rs);
    A.ts = (const i64*)(b + P->off_ts);
    A.off = (u32*)(b + P->off_off);
    A.meta = (u16*)(b + P->off_meta);
    A.ival = (double*)(b + P->off_ival);
    return A;
}

// exclusive scan of one u32 per thread over the workgroup (NT threads); every
// thread must call it; `sh` holds NT / 64 words
template <int NT>
__device__ inline u32 ct_block_scan(u32 v, u32& total, u32* sh)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32 x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = (u32)__shfl_up((int)x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    u32 before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
        const u32 s = sh[i];
        before += i < w ? s : 0u;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return before + x - v;
}

// workgroup b of an XCD-contiguous order: the dispatcher deals workgroups to
// the 8 XCDs round robin, so XCD x runs items [x * per, (x + 1) * per) in order
__device__ inline int ct_xcd_item(int nitems)
{
    const int per = (nitems + 7) >> 3;
    return (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
}

// ---------------------------------------------------------------- validation + bounds
// One wave per CT_BCH consecutive stored entries of the whole CSR (a gene's
// boundaries may fall inside: each lane tracks its own gene), so a gene of a
// million entries does not serialise on one wave.  Superblock s of gene g
// starts at the first entry whose column is >= s * SB: written by that entry
// (s > the last superblock of the gene: k_ct_btail).
#define CT_BCH 8192
__global__ void __launch_bounds__(256) k_ct_bounds(const i64* __restrict__ indptr, const int* __restrict__ cols,
                                                   int G, int N, int SB, int NS, long long nnz,
                                                   u32* __restrict__ bnd, int* __restrict__ err)
{
    const int lane = threadIdx.x & 63;
    const long long e0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * CT_BCH;
    if (e0 >= nnz) return;
    const long long e1 = min(nnz, e0 + (long long)CT_BCH);
    // the gene holding entry e0: indptr[g] <= e0 < indptr[g + 1]
    int lo = 0, hi = G;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (indptr[mid] <= e0)
            lo = mid;
        else
            hi = mid;
    }
    int g = lo;
    while (g < G - 1 && indptr[g + 1] <= e0) ++g;  // (empty genes at e0)
    i64 gs = indptr[g], ge = indptr[g + 1];
    bool bad = false;
    int prev = e0 > 0 ? cols[e0 - 1] : -1;  // the previous entry's column (wave-uniform)
    for (long long b0 = e0; b0 < e1; b0 += 256) {
        int c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // four loads in flight (clamped index, then masked)
            const long long e = b0 + q * 64 + lane;
            c[q] = cols[e < e1 ? e : e1 - 1];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const long long e = b0 + q * 64 + lane;
            int p = __shfl_up(c[q], 1, 64);
            if (lane == 0) p = prev;
            prev = __shfl(c[q], 63, 64);
            if (e >= e1) continue;
            while (e >= ge) {  // this lane's gene (boundaries are rare: a few steps at most)
                ++g;
                gs = ge;
                ge = indptr[g + 1];
            }
            if (e == gs) p = -1;  // a gene's first entry
            const int cq = c[q];
            if (cq < 0 || cq >= N || cq <= p) {
                bad = true;
            } else {
                // superblocks (p / SB, c / SB] start at this entry
                u32* B = bnd + (size_t)g * (NS + 1);
                const int sp = p < 0 ? -1 : p / SB;
                for (int s = sp + 1; s <= cq / SB; ++s) B[s] = (u32)(e - gs);
            }
        }
    }
    if (__ballot(bad) && lane == 0) atomicOr(err, 2);
}

// superblocks past a gene's last entry start at its end (all of them for an
// empty gene): one thread per (gene, superblock)
__global__ void __launch_bounds__(256) k_ct_btail(const i64* __restrict__ indptr, const int* __restrict__ cols,
                                                  int G, int N, int SB, int NS, u32* __restrict__ bnd)
{
    const long long x = (long long)blockIdx.x * 256 + threadIdx.x;
    if (x >= (long long)G * (NS + 1)) return;
    const int g = (int)(x / (NS + 1)), s = (int)(x - (long long)g * (NS + 1));
    const i64 r0 = indptr[g], len = indptr[g + 1] - r0;
    const int last = len > 0 ? cols[r0 + len - 1] : -1;
    const int sl = (last >= 0 && last < N) ? last / SB : -1;
    if (s > sl) bnd[x] = (u32)len;
}

// ---------------------------------------------------------------- per-tile region offsets
__global__ void __launch_bounds__(256) k_ct_tiles(CtArgs A, u32* __restrict__ rs, u32* __restrict__ tt)
{
    __shared__ u32 sh[4];
    const int t = blockIdx.x;
    const int g0 = t * CT_TG, g1 = min(A.G, g0 + CT_TG);
    u32 carry = 0;
    for (int s0 = 0; s0 < A.NS; s0 += 256) {
        const int s = s0 + (int)threadIdx.x;
        u32 n = 0;
        if (s < A.NS) {
            int g = g0;
            for (; g + 8 <= g1; g += 8) {  // eight rows' loads in flight
                u32 d[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const u32* B = A.bnd + (size_t)(g + u) * (A.NS + 1);
                    d[u] = B[s + 1] - B[s];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) n += d[u];
            }
            for (; g < g1; ++g) {
                const u32* B = A.bnd + (size_t)g * (A.NS + 1);
                n += B[s + 1] - B[s];
            }
        }
        u32 tot;
        const u32 ex = ct_block_scan<256>(n, tot, sh);
        if (s < A.NS) rs[(size_t)t * A.NS + s] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        tt[t] = carry;
        A.off[(size_t)t * (A.NG + 1) + A.NG] = carry;
    }
}

// ---------------------------------------------------------------- pass 1
template <int KPT>
__global__ void __launch_bounds__(CT_T1) k_ct_pass1(const i64* __restrict__ indptr, const int* __restrict__ cols,
                                                    const double* __restrict__ vals, CtArgs A,
                                                    u32* __restrict__ cell_tot)
{
    extern __shared__ u64 ct_dyn[];   // SB cells: the masks, then the slots
    u64(*mask)[4] = (u64(*)[4])ct_dyn;    // per cell: which of the tile's genes hold an entry there
    u32* cst = (u32*)(ct_dyn + 4 * A.SB); // per cell: its first slot in the region's cell-major order
    double* sval = (double*)(ct_dyn + 4 * A.SB + (A.SB + 1) / 2);  // the region, cell-major (one chunk)
    u16* smeta = (u16*)(sval + KPT * CT_T1);
    __shared__ u32 gofs[CT_TG + 1];   // per gene: its first entry in the region's flattened stream
    __shared__ i64 gsrc[CT_TG];       // per gene: the region's first entry (absolute)
    __shared__ u32 sh[CT_T1 / 64];
    const int nreg = A.T * A.NS;
    const int L = ct_xcd_item(nreg);
    if (L >= nreg) return;
    const int t = L / A.NS, s = L - t * A.NS;
    const int tid = threadIdx.x;
    const int g = t * CT_TG + tid;
    const bool gv = g < A.G;
    const i64 rb = gv ? indptr[g] : 0;
    const u32* B = A.bnd + (size_t)(gv ? g : 0) * (A.NS + 1);
    const u32 pos = gv ? B[s] : 0u;
    const u32 pend = gv ? B[s + 1] : 0u;
    const int a = s * A.SB, w = min(A.N, a + A.SB) - a;
    const i64 tbase = A.ts[t];
    const u32 orel = A.rs[(size_t)t * A.NS + s];  // this region's offset inside the tile's output
    const int CGm = A.CG - 1;
    u32* offt = A.off + (size_t)t * (A.NG + 1);
    for (int i = tid; i < w * 4; i += CT_T1) (&mask[0][0])[i] = 0ull;
    u32 cnt;
    gofs[tid] = ct_block_scan<CT_T1>(pend - pos, cnt, sh);
    gsrc[tid] = rb + pos;
    if (tid == 0) gofs[CT_TG] = cnt;
    __syncthreads();
    // the region's row pieces as one flattened stream: entry i = i0 + tid + q * 256
    // of chunk i0 (the searches advance together; every load is issued before
    // the LDS work; indices clamped, then masked).  One chunk: held in
    // registers from the mask build to the placement; more: a sweep building
    // the masks, then one placing (columns read twice).
    u32 kc[KPT];
    double kv[KPT];
    auto load_chunk = [&](u32 i0, bool with_vals) {
        int lo[KPT];
#pragma unroll
        for (int q = 0; q < KPT; ++q) lo[q] = 0;
#pragma unroll
        for (int st = 7; st >= 0; --st)  // gofs[lo] <= i < gofs[lo + 1]: a step of every search at once
#pragma unroll
            for (int q = 0; q < KPT; ++q) {
                const u32 i = min(i0 + tid + (u32)q * CT_T1, cnt - 1);
                lo[q] += gofs[lo[q] + (1 << st)] <= i ? (1 << st) : 0;
            }
#pragma unroll
        for (int q = 0; q < KPT; ++q) {
            const u32 i = min(i0 + tid + (u32)q * CT_T1, cnt - 1);
            const i64 e = gsrc[lo[q]] + (i - gofs[lo[q]]);
            kc[q] = (u32)cols[e];
            if (with_vals) kv[q] = vals[e];
        }
#pragma unroll
        for (int q = 0; q < KPT; ++q) {
            const int cl = min(max((int)kc[q] - a, 0), w - 1);  // (validated by k_ct_bounds)
            kc[q] = ((u32)cl << 8) | (u32)lo[q];
        }
    };
    auto mark = [&](u32 i0) {
#pragma unroll
        for (int q = 0; q < KPT; ++q)
            if (i0 + tid + (u32)q * CT_T1 < cnt)
                atomicOr(&mask[kc[q] >> 8][(kc[q] & 255u) >> 6], 1ull << (kc[q] & 63u));
    };
    // staged: the slot inside the region in LDS (then written out linearly);
    // otherwise straight to the intermediate
    auto place = [&](u32 i0, bool staged) {
#pragma unroll
        for (int q = 0; q < KPT; ++q) {
            if (i0 + tid + (u32)q * CT_T1 >= cnt) continue;
            const int cl = (int)(kc[q] >> 8), j = (int)(kc[q] & 255u);
            const int qq = j >> 6;
            u32 r = (u32)__popcll(mask[cl][qq] & ((1ull << (j & 63)) - 1ull));
            r += qq > 0 ? (u32)__popcll(mask[cl][0]) : 0u;
            r += qq > 1 ? (u32)__popcll(mask[cl][1]) : 0u;
            r += qq > 2 ? (u32)__popcll(mask[cl][2]) : 0u;
            const u32 d = cst[cl] + r;
            const u16 m = (u16)((((a + cl) & CGm) << 8) | j);
            if (staged) {
                smeta[d] = m;
                sval[d] = kv[q];
            } else {
                A.meta[tbase + orel + d] = m;
                A.ival[tbase + orel + d] = kv[q];
            }
        }
    };
    const u32 CAP = (u32)(KPT * CT_T1);
    const bool one = cnt <= CAP;
    for (u32 i0 = 0; i0 < cnt; i0 += CAP) {
        load_chunk(i0, one);
        mark(i0);
    }
    __syncthreads();
    // per-cell counts (4 cells a thread) and their scan: the cell-major slots
    u32 c4[4], ln = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int cl = tid * 4 + q;
        c4[q] = 0;
        if (cl < w)
            c4[q] = (u32)(__popcll(mask[cl][0]) + __popcll(mask[cl][1]) + __popcll(mask[cl][2]) +
                          __popcll(mask[cl][3]));
        ln += c4[q];
    }
    u32 tot2;
    u32 cx = ct_block_scan<CT_T1>(ln, tot2, sh);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int cl = tid * 4 + q;
        if (cl < w) {
            cst[cl] = cx;
            if (((a + cl) & CGm) == 0) offt[(a + cl) / A.CG] = orel + cx;  // an output group starts here
            if (c4[q]) atomicAdd(&cell_tot[a + cl], c4[q]);
        }
        cx += c4[q];
    }
    __syncthreads();
    // cell-major placement: a cell's rank of gene j = the tile's genes below j there
    if (one) {
        if (cnt > 0) {
            place(0, true);
            __syncthreads();
            u16* dm = A.meta + tbase + orel;
            double* dv = A.ival + tbase + orel;
            for (u32 i = tid; i < cnt; i += CT_T1) {
                dm[i] = smeta[i];
                dv[i] = sval[i];
            }
        }
    } else {
        for (u32 i0 = 0; i0 < cnt; i0 += CAP) {
            load_chunk(i0, true);
            place(i0, false);
        }
    }
}

// ---------------------------------------------------------------- pass 2
// Entry i of the group's flattened runs (tile order, a run cell-major, a cell's
// entries gene-ordered) goes to slot  cb[c] + P[t][c] + (i - S[t][c]):  P the
// cell's entries in earlier tiles, S where the cell's segment of run t starts.
// The KPT entries of a thread are searched together (a step of every search,
// then the next step: the LDS reads of one step are in flight together) and
// all their loads are issued before any is used.
template <int KPT>
__device__ inline void ct_runs_of(const u32* F, int nsteps, u32 i0, u32 n, int (&lo)[KPT])
{
#pragma unroll
    for (int q = 0; q < KPT; ++q) lo[q] = 0;
    for (int st = nsteps - 1; st >= 0; --st) {  // F[lo] <= i < F[lo + 1] (F past nt: 0xffffffff)
#pragma unroll
        for (int q = 0; q < KPT; ++q) {
            const u32 i = min(i0 + (u32)q * CT_T2, n - 1);
            lo[q] += F[lo[q] + (1 << st)] <= i ? (1 << st) : 0;
        }
    }
}

template <int KPT>
__global__ void __launch_bounds__(CT_T2) k_ct_pass2(CtArgs A, const long long* __restrict__ csc_indptr,
                                                   int* __restrict__ rows_out, double* __restrict__ vals_out)
{
    __shared__ u32 F[CT_TCMAX + 1];      // the batch's runs: flattened starts (padded to a power of two)
    __shared__ i64 rbase[CT_TCMAX];      // the batch's runs: first entry in the intermediate
    __shared__ u32 tc[CT_TCMAX];         // per (tile of the batch, cell): count, then P
    __shared__ u32 sg[CT_TCMAX];         // per (tile of the batch, cell): S
    __shared__ u32 cb[257];              // per cell: first slot inside the group
    __shared__ u32 carry[256];           // per cell: entries in earlier batches
    __shared__ u32 lastm[KPT][CT_T2 / 64 + 1];
    __shared__ u32 sh[CT_T2 / 64];
    const int k = ct_xcd_item(A.NG);
    if (k >= A.NG) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int CG = A.CG;
    const int c0 = k * CG, nc = min(CG, A.N - c0);
    const i64 gbase = csc_indptr[c0];
    for (int c = tid; c <= nc; c += CT_T2) cb[c] = (u32)(csc_indptr[c0 + c] - gbase);  // (nc may be 256)
    if (tid < 256) carry[tid] = 0;
    const int TB = CT_TCMAX / CG;  // tiles per batch
    for (int tb0 = 0; tb0 < A.T; tb0 += TB) {
        const int nt = min(TB, A.T - tb0);
        int nsteps = 0;
        while ((1 << nsteps) < nt) ++nsteps;
        // the runs of this batch's tiles and their flattened starts
        u32 carryl = 0;
        for (int i0 = 0; i0 < nt; i0 += CT_T2) {
            const int i = i0 + tid;
            u32 l = 0;
            if (i < nt) {
                const u32* o = A.off + (size_t)(tb0 + i) * (A.NG + 1);
                const u32 o0 = o[k];
                rbase[i] = A.ts[tb0 + i] + o0;
                l = o[k + 1] - o0;
            }
            u32 tot;
            const u32 x = ct_block_scan<CT_T2>(l, tot, sh);
            if (i < nt) F[i] = carryl + x;
            carryl += tot;
        }
        const u32 Mb = carryl;
        for (int i = nt + tid; i <= (1 << nsteps); i += CT_T2) F[i] = i == nt ? Mb : 0xffffffffu;
        for (int i = tid; i < nt * CG; i += CT_T2) sg[i] = 0xffffffffu;
        if (tid == 0) lastm[0][CT_T2 / 64] = 0xffffffffu;  // the entry before the group: none
        __syncthreads();
        // sweep 1: every entry's run and meta (registers); where each (tile,
        // cell) segment starts: an entry whose predecessor is in another run or
        // another cell (lane - 1 holds entry i - 1; lane 0 reads the previous
        // wave's last entry from LDS)
        u32 km[KPT];  // meta | run << 16
        double kv[KPT];
        const bool one = Mb <= (u32)(KPT * CT_T2);
        auto load_chunk = [&](u32 q0) {
            int lo[KPT];
            ct_runs_of<KPT>(F, nsteps, q0 + tid, Mb, lo);
#pragma unroll
            for (int q = 0; q < KPT; ++q) {
                const u32 i = min(q0 + tid + (u32)q * CT_T2, Mb - 1);
                const i64 src = rbase[lo[q]] + (i - F[lo[q]]);
                km[q] = (u32)A.meta[src] | ((u32)lo[q] << 16);
                kv[q] = A.ival[src];
            }
        };
        for (u32 q0 = 0; q0 < Mb; q0 += KPT * CT_T2) {
            load_chunk(q0);
#pragma unroll
            for (int q = 0; q < KPT; ++q)
                if (lane == 63) lastm[q][wv] = km[q] & 0xffffu;
            __syncthreads();
#pragma unroll
            for (int q = 0; q < KPT; ++q) {
                const u32 i = q0 + tid + (u32)q * CT_T2;
                const u32 m = km[q] & 0xffffu;
                const int lo = (int)(km[q] >> 16);
                u32 pm = (u32)__shfl_up((int)m, 1, 64);
                if (lane == 0) pm = wv > 0 ? lastm[q][wv - 1] : (q > 0 ? lastm[q - 1][CT_T2 / 64 - 1]
                                                                         : lastm[0][CT_T2 / 64]);
                const int c = (int)(m >> 8);
                const bool start = i == F[lo] || (pm >> 8) != (m >> 8);
                if (i < Mb && start && c < nc) sg[lo * CG + c] = i;
            }
            __syncthreads();
            if (tid == 0) lastm[0][CT_T2 / 64] = lastm[KPT - 1][CT_T2 / 64 - 1];  // for the next chunk
            __syncthreads();
        }
        // a thread per tile: counts from the segment starts (an empty segment
        // starts where the next one does); S stays in sg
        for (int tl = tid; tl < nt; tl += CT_T2) {
            u32 nxt = F[tl + 1];
            for (int c = CG - 1; c >= 0; --c) {
                u32 st = sg[tl * CG + c];
                if (st == 0xffffffffu) st = nxt;
                sg[tl * CG + c] = st;
                tc[tl * CG + c] = nxt - st;
                nxt = st;
            }
        }
        __syncthreads();
        // P: a wave per cell, the prefix over tiles 64 at a time
        for (int c = wv; c < nc; c += CT_T2 / 64) {
            u32 run = carry[c];
            for (int j0 = 0; j0 < nt; j0 += 64) {
                const int tl = j0 + lane;
                const u32 x = tl < nt ? tc[tl * CG + c] : 0u;
                u32 y = x;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const u32 z = (u32)__shfl_up((int)y, o, 64);
                    if (lane >= o) y += z;
                }
                if (tl < nt) tc[tl * CG + c] = run + y - x;
                run += (u32)__shfl((int)y, 63, 64);
            }
            if (lane == 0) carry[c] = run;
        }
        __syncthreads();
        // sweep 2: place (one chunk: from the registers; more: reloaded)
        for (u32 q0 = 0; q0 < Mb; q0 += KPT * CT_T2) {
            if (!one) load_chunk(q0);
#pragma unroll
            for (int q = 0; q < KPT; ++q) {
                const u32 i = q0 + tid + (u32)q * CT_T2;
                const int lo = (int)(km[q] >> 16);
                const int c = (int)((km[q] & 0xffffu) >> 8);
                if (i >= Mb || c >= nc) continue;  // (c >= nc cannot happen on a consistent intermediate)
                const u32 d = cb[c] + tc[lo * CG + c] + (i - sg[lo * CG + c]);
                if (d >= cb[nc]) continue;
                rows_out[gbase + d] = (tb0 + lo) * CT_TG + (int)(km[q] & 255u);
                vals_out[gbase + d] = kv[q];
            }
        }
        __syncthreads();  // (the batch's tables are rebuilt next)
    }
}

// ---------------------------------------------------------------- host
static size_t ct_align(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" int scc_csr_plan(long long G, long long N, long long nnz, ScCsrPlan* P)
{
    if (G <= 0 || N <= 0 || nnz < 0 || !P || G > CT_GMAX) return -1;
    ScCsrPlan p{};
    p.G = G;
    p.N = N;
    p.nnz = nnz;
    // superblock: a region of 256 genes x SB cells holds about half a register chunk
    // (one sweep; a larger region takes two)
    const double rho = std::max(1e-9, (double)nnz / ((double)G * (double)N));
    const double want = 0.5 * (CT_KPT1 * CT_T1) / (CT_TG * rho);
    int sb = 64;
    while (sb < CT_WMAX && 2.0 * sb <= want * 1.414) sb *= 2;
    p.SB = sb;
    p.NS = (int)((N + sb - 1) / sb);
    p.T = (int)((G + CT_TG - 1) / CT_TG);
    // output group: whole cells, about 3/4 of a register chunk (CT_KPT2 x CT_T2) of
    // entries, and one batch of tiles' (tile, cell) counters in LDS
    const double per_cell = std::max(1.0, (double)nnz / (double)N);
    const int tmax = std::min(p.T, CT_TCMAX);
    int cg = 1;
    while (cg < 256 && 2.0 * cg * per_cell <= 0.75 * (CT_KPT2 * CT_T2) * 1.414 && 2 * cg * tmax <= CT_TCMAX) cg *= 2;
    p.CG = cg;
    p.NG = (int)((N + cg - 1) / cg);
    size_t o = 0;
    p.off_bnd = o;
    o = ct_align(o + sizeof(u32) * (size_t)G * (p.NS + 1));
    p.off_rs = o;
    o = ct_align(o + sizeof(u32) * (size_t)p.T * p.NS);
    p.off_tt = o;
    o = ct_align(o + sizeof(u32) * (size_t)p.T);
    p.off_ts = o;
    o = ct_align(o + sizeof(i64) * (size_t)(p.T + 1));
    p.off_off = o;
    o = ct_align(o + sizeof(u32) * (size_t)p.T * (p.NG + 1));
    p.off_gm = o;  // per-cell totals
    o = ct_align(o + sizeof(u32) * (size_t)N);
    p.off_gb = o;  // (unused)
    p.off_scan = o;
    o = ct_align(o + sizeof(i64) * (size_t)(scc_scan_scratch_blocks(std::max<long long>(N, p.T)) + 1));
    p.off_meta = o;
    o = ct_align(o + sizeof(u16) * (size_t)nnz);
    p.off_ival = o;
    o = ct_align(o + sizeof(double) * (size_t)nnz);
    p.bytes = o;
    *P = p;
    return 0;
}

extern "C" hipError_t scc_launch_csr_check(const ScCsrPlan* P, const long long* indptr, const int* cols,
                                           void* scratch, int* err, hipStream_t st)
{
    u32* bnd = (u32*)((char*)scratch + P->off_bnd);
    const long long nw = (P->nnz + CT_BCH - 1) / CT_BCH;
    if (nw > 0)
        hipLaunchKernelGGL(k_ct_bounds, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, st, indptr, cols, (int)P->G,
                           (int)P->N, P->SB, P->NS, P->nnz, bnd, err);
    const long long nb = (long long)P->G * (P->NS + 1);
    hipLaunchKernelGGL(k_ct_btail, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, indptr, cols, (int)P->G,
                       (int)P->N, P->SB, P->NS, bnd);
    return hipGetLastError();
}

extern "C" hipError_t scc_launch_csr_to_csc(const ScCsrPlan* P, const long long* indptr, const int* cols,
                                            const double* vals, void* scratch, long long* csc_indptr,
                                            int* csc_rows, double* csc_vals, hipStream_t st)
{
    CtArgs A = ct_args(P, scratch);
    char* b = (char*)scratch;
    u32* rs = (u32*)(b + P->off_rs);
    u32* tt = (u32*)(b + P->off_tt);
    i64* ts = (i64*)(b + P->off_ts);
    u32* tot = (u32*)(b + P->off_gm);
    i64* scan = (i64*)(b + P->off_scan);
    hipLaunchKernelGGL(k_ct_tiles, dim3(P->T), dim3(256), 0, st, A, rs, tt);
    hipError_t e = scc_launch_scan(tt, P->T, ts, scan, ts + P->T, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(tot, 0, sizeof(u32) * (size_t)P->N, st);
    if (e != hipSuccess) return e;
    const long long nreg = (long long)P->T * P->NS;
    const size_t lds1 = (size_t)P->SB * 4 * sizeof(u64) + (size_t)(P->SB + 1) / 2 * sizeof(u64) +
                        (size_t)CT_KPT1 * CT_T1 * (sizeof(double) + sizeof(u16));
    hipLaunchKernelGGL(k_ct_pass1<CT_KPT1>, dim3((unsigned)(8 * ((nreg + 7) / 8))), dim3(CT_T1), lds1, st, indptr,
                       cols, vals, A, tot);
    e = scc_launch_scan(tot, P->N, csc_indptr, scan, csc_indptr + P->N, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_ct_pass2<CT_KPT2>, dim3((unsigned)(8 * ((P->NG + 7) / 8))), dim3(CT_T2), 0, st, A,
                       (const long long*)csc_indptr, csc_rows, csc_vals);
    return hipGetLastError();
}
