// Streaming-store bandwidth on MI355X for the packed-distance write pattern
// (2.7 GB, the config-B fp64 output): which store shape reaches the HBM write
// ceiling.  hipcc --offload-arch=gfx950 -O3 -o store_bw store_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
            return 1;                                                           \
        }                                                                       \
    } while (0)

// grid-stride, one double per lane per instruction (512 B per wave-instruction)
__global__ void k_x2(double* out, long long n)
{
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
        out[e] = (double)e;
}
// two doubles per lane (1 KB per wave-instruction)
__global__ void k_x4(double* out, long long n)
{
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2* o = (d2*)out;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n / 2; e += (long long)gridDim.x * blockDim.x)
        o[e] = d2{(double)e, (double)e};
}
// non-temporal stores
__global__ void k_nt(double* out, long long n)
{
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((double)e, out + e);
}
// per-block contiguous chunk (each workgroup writes its own 64 KB run)
__global__ void k_chunk(double* out, long long n, int per)
{
    const long long base = (long long)blockIdx.x * per;
    for (int k = threadIdx.x; k < per; k += blockDim.x) {
        const long long e = base + k;
        if (e < n) out[e] = (double)e;
    }
}
// the distance tile shape: 256 threads = 256 rows, 64 columns, column j's run
// starts at an arbitrary (unaligned) offset off + j * stride
__global__ void k_tile(double* out, long long n, long long stride)
{
    const long long t = blockIdx.x;
    const long long base = t * 64 * stride + (t * 8) % 16;
    for (int j = 0; j < 64; ++j) {
        const long long e = base + (long long)j * stride + threadIdx.x;
        if (e < n) out[e] = (double)e;
    }
}

// column-major square layout like the packed dist (column stride N): tile t
// = (column block cb, row block rb), rows dealt consecutively; optional
// per-element arithmetic of the distance kernel (15 sub + 15 FMA + sqrt)
template <bool COMPUTE>
__global__ void k_colmajor(double* out, long long n, int N, int nrb, const double* P)
{
    const long long t = blockIdx.x;
    const int cb = (int)(t / nrb), rb = (int)(t % nrb);
    const int i = rb * 256 + threadIdx.x;
    double pi[15];
    if (COMPUTE)
        for (int q = 0; q < 15; ++q) pi[q] = P[(i % 4096) * 16 + q];
    for (int jj = 0; jj < 64; ++jj) {
        const int j = cb * 64 + jj;
        const long long e = ((long long)j * N + i) % n;
        double v = (double)e;
        if (COMPUTE) {
            double s = 0.0;
            for (int q = 0; q < 15; ++q) {
                const double dv = pi[q] - P[(j % 4096) * 16 + q];
                s = fma(dv, dv, s);
            }
            v = __builtin_amdgcn_sqrt(s);
        }
        out[e] = v;
    }
}

int main()
{
    const long long n = 26000LL * 25999 / 2;
    double* d;
    CHK(hipMalloc(&d, n * sizeof(double)));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto run = [&](const char* name, auto launch) {
        for (int r = 0; r < 2; ++r) launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 10; ++r) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        ms /= 10;
        printf("%-28s %.3f ms  %.2f TB/s\n", name, ms, n * 8.0 / ms / 1e9);
        fflush(stdout);
    };
    for (int wpc : {4, 8, 16, 32}) {
        char nm[64];
        snprintf(nm, sizeof nm, "x2 grid %d/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL(k_x2, dim3(cus * wpc), dim3(256), 0, 0, d, n); });
        snprintf(nm, sizeof nm, "x4 grid %d/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL(k_x4, dim3(cus * wpc), dim3(256), 0, 0, d, n); });
        snprintf(nm, sizeof nm, "nt grid %d/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL(k_nt, dim3(cus * wpc), dim3(256), 0, 0, d, n); });
    }
    for (int per : {8192, 16384, 65536}) {
        char nm[64];
        snprintf(nm, sizeof nm, "chunk %d doubles", per);
        run(nm, [&] { hipLaunchKernelGGL(k_chunk, dim3((unsigned)((n + per - 1) / per)), dim3(256), 0, 0, d, n, per); });
    }
    run("tile 256x64 unaligned", [&] {
        hipLaunchKernelGGL(k_tile, dim3((unsigned)((n + 64 * 256 - 1) / (64 * 256))), dim3(256), 0, 0, d, n, 256LL);
    });
    {
        const int N = 26000, nrb = (N + 255) / 256;
        double* P;
        CHK(hipMalloc(&P, 4096 * 16 * sizeof(double)));
        hipMemset(P, 0, 4096 * 16 * sizeof(double));
        const unsigned ntile = (unsigned)(n / (64LL * 256));
        run("colmajor stride N", [&] { hipLaunchKernelGGL(k_colmajor<false>, dim3(ntile), dim3(256), 0, 0, d, n, N, nrb, P); });
        run("colmajor stride N + math", [&] { hipLaunchKernelGGL(k_colmajor<true>, dim3(ntile), dim3(256), 0, 0, d, n, N, nrb, P); });
    }
    run("hipMemsetAsync", [&] { hipMemsetAsync(d, 0, n * sizeof(double)); });
    CHK(hipFree(d));
    return 0;
}
