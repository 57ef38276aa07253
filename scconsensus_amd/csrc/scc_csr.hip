// scc_csr.hip — gene-major CSR input (genes x cells, per gene ascending cell
// columns: scipy.sparse.csr_matrix / an AnnData .X transposed, BASELINE config
// E's "1M-cell sparse CSR input") turned into the engine's resident layout,
// the dgCMatrix CSC over cells that R hands the reference
// (R/reclusterDEConsensusFast.R:368 `as.matrix(dataMatrix)` consumes it).
//
// A deterministic device transpose, run once when the dataset is created
// (the dataset is reused by every scc_de_run / scc_distance call):
//   k_csr_count    one workgroup per gene row: per (gene tile of CSR_TG
//                  genes, cell) counts, column indices range-checked
//   k_csr_colscan  one thread per cell: counts -> offsets over the tiles
//                  (in place), cell totals
//   scan           totals -> CSC indptr
//   k_csr_scatter  one workgroup per gene tile: its genes in ascending order,
//                  a gene's entries in parallel (distinct cells, so the
//                  per-(tile, cell) cursors need no atomics)
// Within a cell the rows come out ascending (tiles, then genes of a tile, in
// order), exactly the dgCMatrix the same matrix would have in R.
#include "scc_common.hpp"
#include "scc_kernels.hpp"

__global__ void __launch_bounds__(256) k_csr_count(const long long* __restrict__ indptr,
                                                   const int* __restrict__ cols, int N, int tg,
                                                   uint32_t* __restrict__ cnt, int* __restrict__ err)
{
    const int g = blockIdx.x;
    const long long e0 = indptr[g], e1 = indptr[g + 1];
    uint32_t* row = cnt + (size_t)(g / tg) * N;
    bool bad = e1 < e0;
    for (long long e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int c = cols[e];
        if (c < 0 || c >= N) {
            bad = true;
            continue;
        }
        atomicAdd(&row[c], 1u);
    }
    if (bad) atomicOr(err, 2);
}

__global__ void __launch_bounds__(256) k_csr_colscan(uint32_t* __restrict__ cnt, int ntile, int N,
                                                     uint32_t* __restrict__ total)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= N) return;
    uint32_t run = 0;
    for (int t = 0; t < ntile; ++t) {
        const uint32_t v = cnt[(size_t)t * N + c];
        cnt[(size_t)t * N + c] = run;
        run += v;
    }
    total[c] = run;
}

__global__ void __launch_bounds__(256) k_csr_scatter(const long long* __restrict__ indptr,
                                                     const int* __restrict__ cols,
                                                     const double* __restrict__ vals, int G, int N, int tg,
                                                     uint32_t* __restrict__ cur,
                                                     const long long* __restrict__ cptr,
                                                     int* __restrict__ rows_out, double* __restrict__ vals_out)
{
    const int t = blockIdx.x;
    uint32_t* row = cur + (size_t)t * N;
    const int g1 = min(G, (t + 1) * tg);
    for (int g = t * tg; g < g1; ++g) {
        const long long e0 = indptr[g], e1 = indptr[g + 1];
        for (long long e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
            const int c = cols[e];
            const uint32_t k = row[c];
            row[c] = k + 1;
            const long long pos = cptr[c] + k;
            rows_out[pos] = g;
            vals_out[pos] = vals[e];
        }
        __syncthreads();  // the next gene may hit the same cells
    }
}

extern "C" size_t scc_csr_scratch_words(long long G, long long N)
{
    const long long ntile = (G + SCC_CSR_TG - 1) / SCC_CSR_TG;
    return (size_t)(ntile * N + N);
}

extern "C" hipError_t scc_launch_csr_to_csc(const long long* indptr, const int* cols, const double* vals, int G,
                                            int N, uint32_t* scratch, long long* scan_scratch,
                                            long long* csc_indptr, int* csc_rows, double* csc_vals, int* err,
                                            int check_only, hipStream_t st)
{
    const int tg = SCC_CSR_TG, ntile = (G + tg - 1) / tg;
    uint32_t* cnt = scratch;
    uint32_t* total = scratch + (size_t)ntile * N;
    if (check_only == 1) {
        hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (size_t)ntile * N, st);
        hipLaunchKernelGGL(k_csr_count, dim3(G), dim3(256), 0, st, indptr, cols, N, tg, cnt, err);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_csr_colscan, dim3((N + 255) / 256), dim3(256), 0, st, cnt, ntile, N, total);
    hipError_t e = scc_launch_scan(total, N, csc_indptr, scan_scratch, csc_indptr + N, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_csr_scatter, dim3(ntile), dim3(256), 0, st, indptr, cols, vals, G, N, tg, cnt, csc_indptr,
                       csc_rows, csc_vals);
    return hipGetLastError();
}
