// D2H copy engines vs a concurrent store-bound kernel (streamed
// tiles).  Times a streaming-store kernel alone, a 512 MB device-to-pinned-host
// copy alone, and the two together on two streams, for each copy kind:
//   0 hipMemcpyDeviceToHost, 1 hipMemcpyDeviceToDeviceNoCU (dst = pinned host),
//   2 hipMemcpyDefault.
// hipcc --offload-arch=gfx950 -O2 scripts/d2h_overlap.hip -o /tmp/d2h && /tmp/d2h [kind]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

__global__ void k_store(double* __restrict__ out, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x * 2;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += stride) {
        double2 v = {(double)i, (double)(i + 1)};
        *reinterpret_cast<double2*>(out + i) = v;
    }
}

__global__ void k_marker(int) {}

// a device-to-host copy on the CUs with a bounded grid: 16-B loads from HBM,
// 16-B stores into the pinned (host-coherent) destination over PCIe
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_copy_h(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n16)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        __builtin_nontemporal_store(src[i], dst + i);
}
static const int kWg[] = {32, 64, 128, 256, 1024};

static const char* kname(int k)
{
    static char b[32];
    if (k >= 3) {
        std::snprintf(b, sizeof b, "kernel_%dwg", kWg[k - 3]);
        return b;
    }
    return k == 0 ? "D2H" : k == 1 ? "D2D_NoCU" : "Default";
}

int main(int argc, char** argv)
{
    const int only = argc > 1 ? std::atoi(argv[1]) : -1;
    if (only == 9) {  // sweep: size x offset, a k_marker<<<id>>> before each (which engine copies shows in a trace)
        const size_t big = (size_t)512 << 20;
        char *d, *hh;
        CK(hipMalloc(&d, big + 4096));
        CK(hipHostMalloc(&hh, big + 4096, hipHostMallocDefault));
        CK(hipMemset(d, 1, big + 4096));
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const size_t mbs[] = {1, 8, 32, 64, 128, 512};
        const size_t offs[] = {0, 8, 4096};
        int id = 1;
        for (size_t mb : mbs)
            for (size_t off : offs) {
                const size_t nb = (mb << 20) - (off ? 24 : 0);
                k_marker<<<id, 64, 0, s>>>(id);
                CK(hipMemcpyAsync(hh + off, d + off, nb, hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(e0, s));
                CK(hipMemcpyAsync(hh + off, d + off, nb, hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                std::printf("marker %d: %zu MB off %zu: %.3f ms %.1f GB/s\n", id, mb, off, t, nb / t / 1e6);
                ++id;
            }
        return 0;
    }
    const size_t bytes = (size_t)512 << 20, n = bytes / 8;
    double *dk, *dsrc, *h;
    CK(hipMalloc(&dk, bytes));
    CK(hipMalloc(&dsrc, bytes));
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    CK(hipMemset(dsrc, 1, bytes));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t a0, b0, a1, b1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&b0));
    CK(hipEventCreate(&a1));
    CK(hipEventCreate(&b1));
    const int grid = 256 * 8, reps = 8;
    auto kern = [&](int r) {
        for (int i = 0; i < r; ++i) k_store<<<grid, 256, 0, s0>>>(dk, n);
    };
    kern(2);
    CK(hipStreamSynchronize(s0));
    float ms;
    CK(hipEventRecord(a0, s0));
    kern(reps);
    CK(hipEventRecord(b0, s0));
    CK(hipEventSynchronize(b0));
    CK(hipEventElapsedTime(&ms, a0, b0));
    const double k_alone = ms / reps;
    std::printf("kernel alone: %.3f ms/launch, %.0f GB/s\n", k_alone, bytes / k_alone / 1e6);
    for (int kind = 0; kind < 8; ++kind) {
        if (only >= 0 && kind != only) continue;
        const hipMemcpyKind mk0 = kind == 0 ? hipMemcpyDeviceToHost
                                  : kind == 1 ? hipMemcpyDeviceToDeviceNoCU
                                              : hipMemcpyDefault;
        auto hipMemcpyAsync = [&](void* dst, const void* src, size_t nb, hipMemcpyKind mk, hipStream_t st) {
            if (kind < 3) return ::hipMemcpyAsync(dst, src, nb, mk, st);
            k_copy_h<<<kWg[kind - 3], 256, 0, st>>>((const u32x4*)src, (u32x4*)dst, nb / 16);
            return hipGetLastError();
        };
        const hipMemcpyKind mk = mk0;
        hipError_t e = hipMemcpyAsync(h, dsrc, bytes, mk, s1);  // warm + check the kind is accepted
        if (e != hipSuccess) {
            std::printf("%s: rejected (%s)\n", kname(kind), hipGetErrorString(e));
            (void)hipGetLastError();
            continue;
        }
        CK(hipStreamSynchronize(s1));
        CK(hipEventRecord(a1, s1));
        CK(hipMemcpyAsync(h, dsrc, bytes, mk, s1));
        CK(hipEventRecord(b1, s1));
        CK(hipEventSynchronize(b1));
        CK(hipEventElapsedTime(&ms, a1, b1));
        const double c_alone = ms;
        // together: the copy on s1 while s0 runs kernels back to back
        const int rt = 96;  // about as long as the copy
        CK(hipEventRecord(a0, s0));
        kern(rt);
        CK(hipEventRecord(b0, s0));
        CK(hipEventRecord(a1, s1));
        CK(hipMemcpyAsync(h, dsrc, bytes, mk, s1));
        CK(hipEventRecord(b1, s1));
        CK(hipDeviceSynchronize());
        float mk_ms, mc_ms;
        CK(hipEventElapsedTime(&mk_ms, a0, b0));
        CK(hipEventElapsedTime(&mc_ms, a1, b1));
        std::printf("%s: copy alone %.3f ms (%.1f GB/s); together: kernels %.3f ms/launch (x%.2f), copy %.3f ms (%.1f GB/s)\n",
                    kname(kind), c_alone, bytes / c_alone / 1e6, mk_ms / rt, mk_ms / rt / k_alone, mc_ms,
                    bytes / mc_ms / 1e6);
        std::fflush(stdout);
    }
    CK(hipHostFree(h));
    CK(hipFree(dk));
    CK(hipFree(dsrc));
    return 0;
}
