// scc_sil.hip — silhouette widths on the HBM-resident distance vector.
//
// Reference: cluster::silhouette(dynamicGroups, dmatrix = as.matrix(d)) and
// mean(summary(.)$clus.avg.widths) per deepSplit value
// (R/reclusterDEConsensusFast.R:433), SURVEY §8(f)-2.  R materialises the
// N x N matrix (as.matrix) and sums per cluster on the host; here the packed
// R `dist` vector stays in HBM and is read once per (row, column) pair.
//
// k_sil_sums   S[i][c] = sum_{j in cluster c} d(i, j) as the product of the
//              full symmetric matrix (read from the packed lower triangle,
//              mirrored) and the one-hot cluster matrix, on fp64 MFMA
//              16x16x4: a wave owns 16 rows x one of SIL_JCH column chunks,
//              up to 4 cluster tiles of 16 in its accumulators.  Partial sums
//              per chunk go to a scratch and are added in chunk order
//              (deterministic).
// k_sil_widths cluster's sildist rule: a = S[own] / (n_own - 1),
//              b = min_{c != own} S[c] / n_c, s = 1 - a/b (a < b), b/a - 1
//              (a > b), 0 (a == b or a singleton cluster).
#include "scc_common.hpp"

typedef double d4 __attribute__((ext_vector_type(4)));

#define SIL_JCH 8    // column chunks per 16-row block (waves in flight)
#define SIL_CT 4     // cluster tiles of 16 per pass (64 clusters)

template <class T>
__device__ inline double sil_d(const T* __restrict__ D, long long N, long long i, long long j)
{
    if (i == j || i >= N || j >= N) return 0.0;
    const long long c = i < j ? i : j, r = i < j ? j : i;  // column c < row r in the packed lower triangle
    return (double)D[c * (2 * N - c - 1) / 2 + (r - c - 1)];
}

// grid: (row blocks of 64 = 4 waves x 16 rows, SIL_JCH, cluster passes)
template <class T>
__global__ void __launch_bounds__(256) k_sil_sums(const T* __restrict__ D, int N, const int* __restrict__ lab, int C,
                                                  double* __restrict__ part)
{
    const int lane = threadIdx.x & 63, w = scc_wave_id();
    const int I0 = (blockIdx.x * 4 + w) * 16;
    if (I0 >= N) return;
    const int ch = blockIdx.y, c0 = blockIdx.z * 16 * SIL_CT;
    const int per = ((N + SIL_JCH - 1) / SIL_JCH + 3) & ~3;
    const int J0 = ch * per, J1 = min(N, J0 + per);
    const int i = I0 + (lane & 15), kq = lane >> 4, cl = lane & 15;
    d4 acc[SIL_CT];
#pragma unroll
    for (int t = 0; t < SIL_CT; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    for (int j0 = J0; j0 < J1; j0 += 16) {
        double dv[4];
        int lj[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {  // 4 k-steps: loads first
            const int j = j0 + 4 * u + kq;
            const bool ok = j < J1;
            dv[u] = ok ? sil_d(D, N, i, j) : 0.0;
            lj[u] = ok ? lab[j] : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int t = 0; t < SIL_CT; ++t) {
                const double b = (lj[u] == c0 + 16 * t + cl) ? 1.0 : 0.0;
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(dv[u], b, acc[t], 0, 0, 0);
            }
        }
    }
    // accumulator register r of tile t: S[row = I0 + kq + 4 r][cluster c0 + 16 t + cl]
#pragma unroll
    for (int t = 0; t < SIL_CT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = I0 + kq + 4 * r, c = c0 + 16 * t + cl;
            if (row < N && c < C) part[((size_t)ch * N + row) * C + c] = acc[t][r];
        }
}

__global__ void __launch_bounds__(256) k_sil_widths(const double* __restrict__ part, int N, int C,
                                                    const int* __restrict__ lab, const int* __restrict__ cnt,
                                                    double* __restrict__ width)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int own = lab[i];
    double a = 0.0, b = INFINITY;
    for (int c = 0; c < C; ++c) {
        double s = 0.0;
        for (int ch = 0; ch < SIL_JCH; ++ch) s += part[((size_t)ch * N + i) * C + c];  // chunk order
        if (c == own)
            a = s;
        else if (cnt[c] > 0)
            b = fmin(b, s / cnt[c]);
    }
    double w = 0.0;
    if (cnt[own] > 1) {
        a /= (cnt[own] - 1);
        w = (a < b) ? 1.0 - a / b : ((a > b) ? b / a - 1.0 : 0.0);
    }
    width[i] = w;
}

extern "C" size_t scc_sil_scratch_doubles(int N, int C) { return (size_t)SIL_JCH * N * C; }

extern "C" hipError_t scc_launch_silhouette(const void* D, int f32, int N, const int* lab, const int* cnt, int C,
                                            double* part, double* width, hipStream_t st)
{
    const dim3 grid((N + 63) / 64, SIL_JCH, (C + 16 * SIL_CT - 1) / (16 * SIL_CT));
    if (f32)
        hipLaunchKernelGGL(k_sil_sums<float>, grid, dim3(256), 0, st, (const float*)D, N, lab, C, part);
    else
        hipLaunchKernelGGL(k_sil_sums<double>, grid, dim3(256), 0, st, (const double*)D, N, lab, C, part);
    hipLaunchKernelGGL(k_sil_widths, dim3((N + 255) / 256), dim3(256), 0, st, part, N, C, lab, cnt, width);
    return hipGetLastError();
}
