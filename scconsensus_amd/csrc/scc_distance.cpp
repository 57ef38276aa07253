// scc_distance.cpp — C ABI for stage 3 (include/scc.h: scc_distance).
//
// PCA path (parity default, reference Fast:398-400): gather X[U, ] for ALL
// cells, centre columns (R colMeans), fp64 MFMA Gram C = Xc^T Xc, top-k
// eigenpairs of the |U| x |U| Gram (Householder + multisection + inverse
// iteration, exact to fp64 backward error), scores
// P = Xc V_k, then the packed Euclidean `dist`.  The eigensolve is this
// engine's own multi-workgroup dense solver (scc_eigen.hip), no vendor BLAS.  The exact truncated SVD is
// the deterministic quantity irlba approximates.
// Pearson path (reference Fast:403, commented out there): per-cell z-scores
// over U and an FP32 MFMA Gram with the 1 - r epilogue fused into the store.
#include "scc_internal.hpp"

#include <chrono>
#include <functional>
#include <thread>

using namespace scc_rt;

extern "C" {
hipError_t scc_launch_union_map(int* umap, int G, const int* genes, int nu, hipStream_t st);
int scc_gather_writes_rows(int ld);
hipError_t scc_launch_gather(const long long* indptr, const int* rows, const double* vals, const double* dense,
                             int G, int N, int Npad, int* umap, const int* genes, int nu, int ld, double* Xc,
                             hipStream_t st);
hipError_t scc_launch_center(double* Xc, int N, int nu, int ld, dd* part, int nchunk, double* mean, int apply,
                             hipStream_t st);
hipError_t scc_launch_gram(const double* Xc, int Npad, int ld, int nchunk, double* slabs, double* C, const double* mean,
                           int nval, hipStream_t st);

int scc_gram_tile_width(int ld);
hipError_t scc_launch_scores(const double* Xc, int N, int nu, int ld, const double* Z16, int k, double* P,
                             const double* mean,
                             hipStream_t st);
size_t scc_sil_scratch_doubles(int N, int C);
hipError_t scc_launch_silhouette(const void* D, int f32, int N, const int* lab, const int* cnt, int C, double* part,
                                 double* width, hipStream_t st);
hipError_t scc_launch_dist_euclid(const double* P, int N, int c_lo, int c_hi, void* out, int f32, hipStream_t st);
hipError_t scc_launch_zscore(const double* Xc, int N, int nu, int ld, float* Z, int ldz, hipStream_t st);
hipError_t scc_launch_pearson(const double* Xc, int N, int nu, int ld, float* Z, int ldz, int c_lo, int c_hi,
                              void* out, int f32, hipStream_t st);
hipError_t scc_launch_d2h(const void* src, void* dst, size_t n, hipStream_t st);
}

extern "C" void scc_distance_release(scc_ctx*) {}

// cell chunks of the split-K Gram (slabs reduced in a fixed order); SCC_GRAM_CHUNKS overrides
static int gram_chunks(int npad)
{
    static const int forced = [] {
        const char* e = getenv("SCC_GRAM_CHUNKS");
        return (e && *e) ? atoi(e) : 0;
    }();
    const int cap = forced > 0 ? std::min(forced, 64) : 32;
    return std::max(1, std::min(cap, npad / 512));
}

namespace {

// host copy of one staged chunk, split over a few threads (a single core
// copies pageable memory at ~10 GB/s, well below the PCIe rate)
void parallel_copy(char* dst, const char* src, size_t n)
{
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>(std::min(8u, hw), std::max<size_t>(1, n >> 22));
    if (nt <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t part = (n / nt + 4095) & ~(size_t)4095;
    for (size_t t = 0; t < nt; ++t) {
        const size_t a = std::min(n, t * part), b = std::min(n, a + part);
        if (a < b) th.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
    }
    for (auto& x : th) x.join();
}

}  // namespace

// Stream the packed distance slice to the caller's host buffer (north_star:
// "the distance tiles stream back through pinned" memory).  The output kernel
// runs once over the slice on s0 (≈1% of the PCIe time: 0.55 ms against 50 ms
// at config B), then the bytes leave in chunks, copied on the CUs by
// k_d2h (scc_dist.hip) in stream order behind it.  A pinned caller buffer
// (hipHostMalloc / hipHostRegister / torch pin_memory) is written directly; a
// pageable one goes through a 2-slot pinned staging ring (2 x 32 MB: its
// allocation is a context's first-call cost, ~25 ms at 2 x 64 MB; 2 x 16 MB
// chunks are slower, profiles/r05_streamed_tiles.md) whose host-side copy of
// slot s overlaps the device copy into the other slot.
// Why not column tiles overlapped with hipMemcpyAsync on a second stream (the
// round-1..4 design): in a torch process the runtime ran each copy as its own
// 131072-thread blit kernel, and a tile kernel sharing the CUs with it ran 24x
// slower (1.18 ms against 49 us per 128 MB tile, profiles/r05_streamed_tiles.md);
// in a plain process it picked the SDMA engine at 30 GB/s.  k_d2h gives the
// link rate (55 GB/s) in either process.  SCC_D2H_KERNEL=0: hipMemcpyAsync
// (the runtime's choice of engine), same stream order.
template <class Emit>
static int stream_to_host(scc_ctx* c, int64_t N, int64_t col_lo, int64_t col_hi, size_t es, char* d_out,
                          char* host, Emit emit)
{
    hipStream_t s0 = c->s0;
    auto colbase = [&](int64_t j) { return (size_t)j * (2 * (size_t)N - j - 1) / 2; };
    const size_t total = (colbase(col_hi) - colbase(col_lo)) * es;
    HIPCHK(c, emit(col_lo, col_hi, d_out));
    const bool kern = env_int("SCC_D2H_KERNEL", 1) != 0;
    auto copy = [&](char* dst, char* dst_dev, const char* src, size_t n) -> hipError_t {
        if (kern && dst_dev) return scc_launch_d2h(src, dst_dev, n, s0);
        return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s0);
    };
    auto dev_ptr = [](char* h) -> char* {  // the device address of pinned host memory
        void* p = nullptr;
        if (hipHostGetDevicePointer(&p, h, 0) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return (char*)p;
    };
    hipPointerAttribute_t pa{};
    bool pinned = hipPointerGetAttributes(&pa, host) == hipSuccess && pa.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    const auto t0 = std::chrono::steady_clock::now();
    // SCC_DIST_REGISTER=1: a large pageable buffer (R's allocVector) is
    // registered with the runtime for the call (page-locked in place, mapped
    // for k_d2h) instead of going through the staging ring and a host memcpy.
    // Off by default: on a freshly allocated buffer (what R hands over) the
    // registration faults in and locks every page first, and the cold call at
    // config B took 164 ms against ~64 ms through the ring (round 6 bench,
    // cold_call_ms)
    bool registered = false;
    if (!pinned && total >= ((size_t)256 << 20) && env_int("SCC_DIST_REGISTER", 0) != 0) {
        registered = hipHostRegister(host, total, hipHostRegisterMapped) == hipSuccess;
        if (!registered) (void)hipGetLastError();
        pinned = registered;
    }
    if (pinned) {  // straight into the caller's buffer
        char* hd = dev_ptr(host);
        const size_t C = (size_t)std::max(1, env_int("SCC_DIST_CHUNK_MB", 1024)) << 20;
        hipError_t e = hipSuccess;
        for (size_t a = 0; a < total && e == hipSuccess; a += C)
            e = copy(host + a, hd ? hd + a : nullptr, d_out + a, std::min(C, total - a));
        if (e == hipSuccess) e = hipStreamSynchronize(s0);
        if (registered && hipHostUnregister(host) != hipSuccess) (void)hipGetLastError();
        HIPCHK(c, e);
    } else {
        const size_t S = (size_t)std::max(1, env_int("SCC_DIST_STAGE_MB", 32)) << 20;
        if (c->dstage_bytes < S) {
            if (c->h_dstage) (void)hipHostFree(c->h_dstage);
            c->h_dstage = nullptr;
            c->dstage_bytes = 0;
            if (hipHostMalloc((void**)&c->h_dstage, 2 * S, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                c->h_dstage = nullptr;
                return fail(c, SCC_ERR_OOM, "pinned distance staging allocation failed");
            }
            c->dstage_bytes = S;
        }
        char* sd = dev_ptr(c->h_dstage);
        const size_t nch = (total + S - 1) / S;
        hipEvent_t done[2] = {ev_take(c), ev_take(c)};
        auto enqueue = [&](size_t ch) -> hipError_t {
            const size_t a = ch * S, b = std::min(total, a + S), slot = (ch & 1) * S;
            hipError_t e = copy(c->h_dstage + slot, sd ? sd + slot : nullptr, d_out + a, b - a);
            if (e == hipSuccess) e = hipEventRecord(done[ch & 1], s0);
            return e;
        };
        hipError_t e = nch ? enqueue(0) : hipSuccess;
        for (size_t ch = 0; ch < nch && e == hipSuccess; ++ch) {
            if (ch + 1 < nch) e = enqueue(ch + 1);  // the next chunk's device copy overlaps this chunk's host copy
            if (e == hipSuccess) e = hipEventSynchronize(done[ch & 1]);
            if (e == hipSuccess) {
                const size_t a = ch * S, b = std::min(total, a + S);
                parallel_copy(host + a, c->h_dstage + (ch & 1) * S, b - a);
            }
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s0);
        c->ev_pool.push_back(done[0]);
        c->ev_pool.push_back(done[1]);
        HIPCHK(c, e);
    }
    if (c->profile) {  // wall time of the streamed output (output kernel + PCIe + host copy)
        auto& tm = c->timers[registered ? "d2h_registered" : (pinned ? "d2h_pinned" : "d2h")];
        tm.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        tm.n += 1;
    }
    return SCC_OK;
}

// Device list (scc_opts.n_devices > 1): the packed columns [col_lo, col_hi)
// cut into one slice of equal entry count per device (distance
// row/column blocks per GPU).  Every device gets the N x 16 scores (xGMI peer
// copy) and writes its slice with the same kernel, so the output is the
// one-device output bit for bit: straight into the caller's host buffer
// (each device streams its own slice through its own staging), or into the
// device output on devices[0] (peer copies of the other slices).  With host
// output devices[0] keeps only its own slice of the engine-kept copy; the
// others stay on their devices until scc_silhouette needs them
// (last_dist_pending).
// The payload a device needs to write its slice: the N x 16 scores (PCA +
// Euclid) or the N x ldz fp32 z-scores (Pearson); `launch(payload, a, b, dst,
// stream)` emits columns [a, b) at dst.
using SliceLaunch = std::function<hipError_t(const void*, int64_t, int64_t, void*, hipStream_t)>;
static int dist_multi(scc_ctx* c, const void* d_pay, size_t pay_bytes, const SliceLaunch& launch, const char* scope,
                      int N, int64_t col_lo, int64_t col_hi, void* d_out, void* dist_out, int32_t out_kind,
                      int32_t out_f32)
{
    const int D = 1 + (int)c->peers.size();
    const size_t es = out_f32 ? 4 : 8;
    auto colbase = [&](int64_t j) { return (size_t)j * (2 * (size_t)N - j - 1) / 2; };
    const size_t base0 = colbase(col_lo), total = colbase(col_hi) - base0;
    std::vector<int64_t> cut(D + 1, col_lo);
    cut[D] = col_hi;
    for (int d = 1; d < D; ++d) {  // first column whose packed start reaches d/D of the entries
        int64_t j = cut[d - 1];
        while (j < col_hi && colbase(j) - base0 < total * d / D) ++j;
        cut[d] = j;
    }
    HIPCHK(c, hipStreamSynchronize(c->s0));  // the scores exist before the peers copy them
    std::vector<int> rcs(D, SCC_OK);
    std::vector<void*> slice(D, nullptr);
    std::vector<std::thread> th;
    for (int d = 0; d < D; ++d)
        th.emplace_back([&, d] {
            scc_ctx* x = d ? c->peers[d - 1] : c;
            hipSetDevice(x->device);
            const int64_t a = cut[d], b = cut[d + 1];
            const size_t off = colbase(a) - base0, n = colbase(b) - colbase(a);
            const void* P = d_pay;
            auto run = [&]() -> int {
                int rc;
                if (d) {  // the payload on this device
                    void* xp = nullptr;
                    if ((rc = ws_get(x, "d_pay", pay_bytes, &xp))) return rc;
                    if (x->device == c->device)
                        HIPCHK(x, hipMemcpyAsync(xp, d_pay, pay_bytes, hipMemcpyDeviceToDevice, x->s0));
                    else
                        HIPCHK(x, hipMemcpyPeerAsync(xp, x->device, d_pay, c->device, pay_bytes, x->s0));
                    P = xp;
                }
                if (a == b) return SCC_OK;
                auto emit = [&](int64_t ca, int64_t cb, void* dst) { return launch(P, ca, cb, dst, x->s0); };
                Scope sc(x, scope, x->s0);
                void* mine = (char*)d_out + off * es;  // devices[0]: straight into the output / kept copy
                if (d) {
                    if ((rc = ws_get(x, "d_dist", std::max<size_t>(n, 1) * es, &mine))) return rc;
                    slice[d] = mine;
                }
                if (out_kind == SCC_PTR_HOST)
                    return stream_to_host(x, N, a, b, es, (char*)mine, (char*)dist_out + off * es, emit);
                HIPCHK(x, emit(a, b, mine));
                if (d) {  // device output on devices[0]
                    if (x->device == c->device)
                        HIPCHK(x, hipMemcpyAsync((char*)d_out + off * es, mine, n * es, hipMemcpyDeviceToDevice, x->s0));
                    else
                        HIPCHK(x, hipMemcpyPeerAsync((char*)d_out + off * es, c->device, mine, x->device, n * es, x->s0));
                }
                HIPCHK(x, hipStreamSynchronize(x->s0));
                return SCC_OK;
            };
            rcs[d] = run();
        });
    for (auto& t : th) t.join();
    scc_enter(c);
    for (int d = 0; d < D; ++d)
        if (rcs[d]) return d ? fail(c, rcs[d], c->peers[d - 1]->err) : rcs[d];
    if (out_kind == SCC_PTR_HOST)
        for (int d = 1; d < D; ++d)
            if (cut[d + 1] > cut[d])
                c->last_dist_pending.push_back({c->peers[d - 1]->device, slice[d], colbase(cut[d]) - base0,
                                                colbase(cut[d + 1]) - colbase(cut[d])});
    return SCC_OK;
}

// columns [col_lo, col_hi) of the packed output (the whole matrix: [0, N))

// the gene list through a pinned buffer: an asynchronous DMA instead of the
// staged copy a pageable source takes
static int genes_h2d(scc_ctx* c, int* d_genes, const int32_t* genes, int nu, hipStream_t s0)
{
    if (c->h_genes_n < (size_t)nu) {
        if (c->h_genes) hipHostFree(c->h_genes);
        c->h_genes = nullptr;
        c->h_genes_n = 0;
        if (hipHostMalloc((void**)&c->h_genes, sizeof(int) * std::max(nu, 1024), hipHostMallocDefault) != hipSuccess) {
            hipGetLastError();
            c->h_genes = nullptr;
            HIPCHK(c, hipMemcpyAsync(d_genes, genes, sizeof(int) * nu, hipMemcpyHostToDevice, s0));
            return SCC_OK;
        }
        c->h_genes_n = (size_t)std::max(nu, 1024);
    }
    if (!c->ev_genes) HIPCHK(c, hipEventCreateWithFlags(&c->ev_genes, hipEventDisableTiming));
    HIPCHK(c, hipEventSynchronize(c->ev_genes));  // the previous copy out of h_genes has completed
    std::memcpy(c->h_genes, genes, sizeof(int) * nu);
    HIPCHK(c, hipMemcpyAsync(d_genes, c->h_genes, sizeof(int) * nu, hipMemcpyHostToDevice, s0));
    HIPCHK(c, hipEventRecord(c->ev_genes, s0));
    return SCC_OK;
}

// set by scc_de_distance around its distance call: the DE's device union
static thread_local const int* t_dev_union = nullptr;

static int dist_impl(scc_ctx* c, const scc_dataset* ds, const int32_t* genes, int32_t nu, int32_t metric,
                     int32_t ncomp, int64_t col_lo, int64_t col_hi, void* dist_out, int32_t out_kind, int32_t out_f32)
{
    if (!c || !ds || !genes) return fail(c, SCC_ERR_INVALID, "scc_distance: null argument");
    if (!dist_out && out_kind != SCC_PTR_DEVICE) return fail(c, SCC_ERR_INVALID, "scc_distance: null output");
    if (ds->ctx != c) return fail(c, SCC_ERR_INVALID, "dataset belongs to another context");
    if (nu < 1) return fail(c, SCC_ERR_INVALID, "empty gene union");
    if (metric != SCC_DIST_PCA_EUCLID && metric != SCC_DIST_PEARSON) return fail(c, SCC_ERR_INVALID, "bad metric");
    const int G = (int)ds->G, N = (int)ds->N;
    if (N < 2) return fail(c, SCC_ERR_INVALID, "need at least two cells");
    for (int u = 0; u < nu; ++u)
        if (genes[u] < 0 || genes[u] >= G) return fail(c, SCC_ERR_INVALID, "gene index out of range");
    int k = ncomp > 0 ? ncomp : std::min(nu, 15);
    if (k > 16 || k > nu) return fail(c, SCC_ERR_UNSUPPORTED, "ncomp must be <= min(16, |U|)");
    scc_enter(c);
    hipStream_t s0 = c->s0;
    c->d_last_dist = nullptr;  // set again only when this call succeeds (the workspace may move)
    c->last_dist_pending.clear();
    const int ld = (nu + 63) & ~63;
    const int Npad = (N + 15) & ~15;
    if (col_lo < 0 || col_hi > N || col_lo > col_hi) return fail(c, SCC_ERR_INVALID, "column slice out of range");
    auto colbase = [&](int64_t j) { return (size_t)j * (2 * (size_t)N - j - 1) / 2; };
    const size_t npairs = colbase(col_hi) - colbase(col_lo);  // the slice's packed entries
    int rc;
    int *d_genes, *d_umap;
    double *d_X, *d_mean;
    void* d_part;
#define WS(name, n, ptr)                                       \
    do {                                                       \
        if ((rc = ws(c, name, (size_t)(n), &(ptr)))) return rc; \
    } while (0)
    WS("d_genes", nu, d_genes);
    WS("d_umap", G, d_umap);
    WS("d_X", (size_t)Npad * ld, d_X);
    WS("d_mean", ld, d_mean);
    const int nchunk_mean = 512;  // 2 x 512 workgroups over the column sums
    if ((rc = ws_get(c, "d_part", sizeof(double) * 2 * (size_t)nchunk_mean * ld, &d_part))) return rc;
    void* d_out = dist_out;
    if (out_kind == SCC_PTR_HOST || !dist_out) {  // NULL device output: keep it in the workspace
        if ((rc = ws_get(c, "d_dist", npairs * (out_f32 ? 4 : 8), &d_out))) return rc;
    }
    // scc_de_distance: the DE's union is still in the workspace, on this device
    // and in this order: used in place of an upload of the host copy
    if (t_dev_union && c->peers.empty())
        d_genes = const_cast<int*>(t_dev_union);
    else if ((rc = genes_h2d(c, d_genes, genes, nu, s0)))
        return rc;
    {
        Scope sc(c, "gather", s0);
        // (the union map and the padding rows' clear included)
        HIPCHK(c, scc_launch_gather(ds->d_indptr, ds->d_rows, ds->d_vals, ds->d_dense, G, N, Npad, d_umap, d_genes, nu,
                                    ld, d_X, s0));
    }
    unsigned int* d_eig_err = nullptr;  // the hand-off's time-out flag, read back after the last launch
    if (metric == SCC_DIST_PCA_EUCLID) {
        double *d_slabs, *d_C, *d_W, *d_Z, *d_P, *d_escr;
        const bool fused = scc_gram_tile_width(ld) == 64;  // centring folded into the 64-wide Gram and the scores
        const int nchunk = gram_chunks(Npad);
        WS("d_slabs", (size_t)nchunk * ld * ld, d_slabs);
        WS("d_C", (size_t)ld * ld, d_C);
        WS("d_W", ld, d_W);
        WS("d_Z", (size_t)ld * 16, d_Z);
        WS("d_P", (size_t)N * 16, d_P);
        WS("d_escr", scc_eigen_scratch_doubles(nu, ld, k), d_escr);
        {
            Scope sc(c, "center", s0);
            // the means only: the Gram and the scores centre on the fly (SCC_CENTER_FUSED=0: a centring pass)
            HIPCHK(c, scc_launch_center(d_X, N, nu, ld, (dd*)d_part, nchunk_mean, d_mean, fused ? 0 : 1, s0));
        }
        {
            Scope sc(c, "gram", s0);
            HIPCHK(c, scc_launch_gram(d_X, Npad, ld, nchunk, d_slabs, d_C, fused ? d_mean : nullptr, fused ? N : Npad,
                                      s0));
        }
        {
            Scope sc(c, "eigen", s0);
            hipEvent_t mk[6];
            hipEvent_t* marks = nullptr;
            static const char* const mk_names[3] = {"eig_tridiag", "eig_vec", "eig_fin"};
            for (int q = 0; q < 3; ++q) {  // per-kernel split of the eigensolve
                mk[2 * q] = mk[2 * q + 1] = nullptr;
                if (stage_timed(c, mk_names[q])) {
                    mk[2 * q] = ev_take(c);
                    mk[2 * q + 1] = ev_take(c);
                    marks = mk;
                }
            }
            unsigned long long* st_buf = nullptr;
            if (env_int("SCC_STAMPS", 0)) WS("d_estamps", 24, st_buf);
            int nwg_used = 0;
            HIPCHK(c, scc_launch_eigen_topk(d_C, nu, ld, k, d_escr, d_Z, d_W, &d_eig_err, &nwg_used, marks, st_buf,
                                            eig_graph_key(c), s0));
            if (st_buf) {
                unsigned long long h[24];
                HIPCHK(c, hipMemcpyAsync(h, st_buf, sizeof(h), hipMemcpyDeviceToHost, s0));
                HIPCHK(c, hipStreamSynchronize(s0));
                fprintf(stderr, "[scc stamps] tridiag n=%d nwg=%d: phase B %llu (wave 0 rows %llu), hand-off wait %llu, "
                        "phase C %llu cycles\n", nu, nwg_used, h[0], h[7], h[1], h[2]);
                fprintf(stderr, "[scc stamps] vectors (eigenpair 0): bisection %llu, LU %llu, inverse iteration %llu, "
                        "back-transform %llu cycles\n", h[3], h[4], h[5], h[6]);
                fprintf(stderr, "[scc stamps] twisted (eigenpair 0): chains %llu, vector %llu, second pass %llu cycles\n",
                        h[8], h[9], h[10]);
                fprintf(stderr, "[scc stamps] block back-transform: stage %llu, V^T Y %llu, T W %llu, Y update %llu, "
                        "load %llu cycles\n", h[12], h[13], h[14], h[15], h[16]);
            }
            for (int q = 0; q < 3; ++q)
                if (mk[2 * q]) c->pending.push_back({mk_names[q], mk[2 * q], mk[2 * q + 1]});
        }
        if (env_int("SCC_EIG_DUMP", 0)) {  // debug: eigenvalues and vectors on stderr
            HIPCHK(c, hipMemcpyAsync(&c->eig_err, d_eig_err, sizeof(unsigned int), hipMemcpyDeviceToHost, s0));
            std::vector<double> w(k), z((size_t)nu * 16);
            HIPCHK(c, hipMemcpyAsync(w.data(), d_W, sizeof(double) * k, hipMemcpyDeviceToHost, s0));
            HIPCHK(c, hipMemcpyAsync(z.data(), d_Z, sizeof(double) * z.size(), hipMemcpyDeviceToHost, s0));
            HIPCHK(c, hipStreamSynchronize(s0));
            fprintf(stderr, "[scc eig] n=%d k=%d err=%u W:", nu, k, c->eig_err);
            for (int q = 0; q < k; ++q) fprintf(stderr, " %.6g", w[q]);
            fprintf(stderr, "\n");
            for (int u = 0; u < std::min(nu, 8); ++u) {
                fprintf(stderr, "[scc eig] Z[%d]:", u);
                for (int q = 0; q < k; ++q) fprintf(stderr, " %.4g", z[(size_t)u * 16 + q]);
                fprintf(stderr, "\n");
            }
        }
        {
            Scope sc(c, "scores", s0);
            HIPCHK(c, scc_launch_scores(d_X, N, nu, ld, d_Z, k, d_P, fused ? d_mean : nullptr, s0));
        }
        auto emit = [&](int64_t a, int64_t b, void* dst) {
            return scc_launch_dist_euclid(d_P, N, (int)a, (int)b, dst, out_f32, s0);
        };
        if (!c->peers.empty()) {
            const SliceLaunch launch = [&](const void* pay, int64_t a, int64_t b, void* dst, hipStream_t st) {
                return scc_launch_dist_euclid((const double*)pay, N, (int)a, (int)b, dst, out_f32, st);
            };
            if ((rc = dist_multi(c, d_P, sizeof(double) * (size_t)N * 16, launch, "dist", N, col_lo, col_hi, d_out,
                                 dist_out, out_kind, out_f32)))
                return rc;
        } else {
            Scope sc(c, "dist", s0);
            if (out_kind == SCC_PTR_HOST) {
                if ((rc = stream_to_host(c, N, col_lo, col_hi, out_f32 ? 4 : 8, (char*)d_out, (char*)dist_out, emit)))
                    return rc;
            } else {
                HIPCHK(c, emit(col_lo, col_hi, d_out));
            }
        }
        c->d_last_scores = d_P;
        c->last_n = N;
        c->last_ncomp = k;
    } else {
        float* d_Zp;
        // rows padded to 8 floats (k_pearson_mfma's fragment group); its 32-float
        // staging reads run up to 24 floats past a row, so the last row has slack
        const int ldz = (nu + 7) & ~7;
        WS("d_Zp", (size_t)N * ldz + 32, d_Zp);
        {
            Scope sz(c, "zscore", s0);
            HIPCHK(c, scc_launch_zscore(d_X, N, nu, ld, d_Zp, ldz, s0));
        }
        auto emit = [&](int64_t a, int64_t b, void* dst) {
            return scc_launch_pearson(d_X, N, nu, ld, d_Zp, ldz, (int)a, (int)b, dst, out_f32, s0);
        };
        if (!c->peers.empty()) {
            // device list: column slices of 1 - r, each device with its own copy
            // of the z-scores (the same kernel per slice: bit-identical to one device)
            const SliceLaunch launch = [&](const void* pay, int64_t a, int64_t b, void* dst, hipStream_t st) {
                return scc_launch_pearson(nullptr, N, nu, ld, (float*)pay, ldz, (int)a, (int)b, dst, out_f32, st);
            };
            if ((rc = dist_multi(c, d_Zp, sizeof(float) * ((size_t)N * ldz + 32), launch, "pearson", N, col_lo, col_hi,
                                 d_out, dist_out, out_kind, out_f32)))
                return rc;
        } else {
        Scope sc(c, "pearson", s0);
        if (out_kind == SCC_PTR_HOST) {
            if ((rc = stream_to_host(c, N, col_lo, col_hi, out_f32 ? 4 : 8, (char*)d_out, (char*)dist_out, emit)))
                return rc;
        } else {
            HIPCHK(c, emit(col_lo, col_hi, d_out));
        }
        }
    }
    // what scc_silhouette(dist = NULL) reads: only an output the engine owns
    // (a caller's device buffer may be freed or reused after this call).  The
    // eigensolver's flag is read here, after the last launch (a copy between
    // the eigensolve and the scores left the GPU idle ~30 us per call).
    c->eig_err = 0;
    unsigned int* hflag_dev = nullptr;
    if (d_eig_err) {
        if (!c->h_flag) {
            // a page, not 4 bytes: a tiny pinned allocation came back without a
            // device mapping (hipHostGetDevicePointer: "Cannot get amd_mem_obj")
            if (hipHostMalloc((void**)&c->h_flag, 4096, hipHostMallocMapped) == hipSuccess)
                *c->h_flag = 0;
            else {
                hipGetLastError();
                c->h_flag = nullptr;
            }
        }
        if (c->h_flag && hipHostGetDevicePointer((void**)&hflag_dev, c->h_flag, 0) != hipSuccess) {
            hipGetLastError();
            hflag_dev = nullptr;
        }
        if (hflag_dev)
            HIPCHK(c, scc_launch_flag_copy(d_eig_err, hflag_dev, s0));
        else
            HIPCHK(c, hipMemcpyAsync(&c->eig_err, d_eig_err, sizeof(unsigned int), hipMemcpyDeviceToHost, s0));
    }
    const bool own = out_kind == SCC_PTR_HOST || !dist_out;
    c->d_last_dist = (own && col_lo == 0 && col_hi == N) ? d_out : nullptr;
    c->last_dist_n = N;
    c->last_dist_f32 = out_f32 ? 1 : 0;
    if (hflag_dev && out_kind == SCC_PTR_DEVICE && !dist_out && c->peers.empty()) {
        // the engine keeps the output (HBM-resident, read only by later calls
        // on this context's stream): return once the work is queued, so the
        // caller's next host work overlaps the distance kernels; the hand-off
        // flag waits in h_flag for the next synchronising call (scc_de_run,
        // scc_ctx_synchronize, a host- or caller-buffer scc_distance)
        c->eig_flag_pending = true;
        return SCC_OK;
    }
    HIPCHK(c, hipStreamSynchronize(s0));
    if (hflag_dev) {
        c->eig_flag_pending = true;
        int rc2 = check_pending_eig(c);
        if (rc2) {
            c->d_last_dist = nullptr;
            return rc2;
        }
    } else if (metric == SCC_DIST_PCA_EUCLID && c->eig_err) {
        c->d_last_dist = nullptr;
        return fail(c, SCC_ERR_HIP, "scc_distance: eigensolver workgroup hand-off timed out");
    }
    return SCC_OK;
#undef WS
}

extern "C" int scc_distance(scc_ctx* c, const scc_dataset* ds, const int32_t* genes, int32_t nu, int32_t metric,
                            int32_t ncomp, void* dist_out, int32_t out_kind, int32_t out_f32)
{
    return dist_impl(c, ds, genes, nu, metric, ncomp, 0, ds ? ds->N : 0, dist_out, out_kind, out_f32);
}

extern "C" int scc_de_distance(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K,
                               const scc_de_params* prm, int32_t metric, int32_t ncomp, void* dist_out,
                               int32_t out_kind, int32_t out_f32, scc_de_result** out)
{
    if (!out) return fail(c, SCC_ERR_INVALID, "scc_de_distance: null result pointer");
    *out = nullptr;
    const int rc = scc_de_run(c, ds, code, K, prm, out);
    if (rc != SCC_OK) return rc;
    const scc_de_result* r = *out;
    if (r->union_genes.empty()) return fail(c, SCC_ERR_INVALID, "empty gene union");
    // the DE's device union (a workspace view, valid while nothing else ran)
    t_dev_union = (c->peers.empty() && r->generation == c->generation && env_int("SCC_DEVICE_UNION", 1)) ? r->d_union
                                                                                                     : nullptr;
    const int drc = dist_impl(c, ds, r->union_genes.data(), (int32_t)r->union_genes.size(), metric, ncomp, 0, ds->N,
                              dist_out, out_kind, out_f32);
    t_dev_union = nullptr;
    return drc;
}

extern "C" int scc_distance_cols(scc_ctx* c, const scc_dataset* ds, const int32_t* genes, int32_t nu, int32_t metric,
                                 int32_t ncomp, int64_t col_lo, int64_t col_hi, void* dist_out, int32_t out_kind,
                                 int32_t out_f32)
{
    return dist_impl(c, ds, genes, nu, metric, ncomp, col_lo, col_hi, dist_out, out_kind, out_f32);
}

// ====================================================================== sharded PCA
// (include/scc.h: scc_pca_shard_*; SURVEY 8e "per-GPU partial Gram over cell
// shards, then an all-reduce of the |U| x |U| fp64 Gram")
extern "C" hipError_t scc_launch_colsum_dd(const double* Xc, int n, int ld, int nu, dd* part, int nchunk, dd* out,
                                           hipStream_t st);
extern "C" hipError_t scc_launch_center_parts(double* Xc, int n, int nu, int ld, const dd* parts, int nparts, double N,
                                              double* mean, hipStream_t st);

extern "C" int scc_pca_shard_colsum(scc_ctx* c, const scc_dataset* ds, const int32_t* genes, int32_t nu,
                                    int64_t cell_lo, int64_t cell_hi, void* part)
{
    if (!c || !ds || !genes || !part) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_colsum: null argument");
    if (ds->ctx != c) return fail(c, SCC_ERR_INVALID, "dataset belongs to another context");
    const int G = (int)ds->G, N = (int)ds->N;
    if (nu < 1) return fail(c, SCC_ERR_INVALID, "empty gene union");
    if (cell_lo < 0 || cell_hi > N || cell_lo > cell_hi) return fail(c, SCC_ERR_INVALID, "cell shard out of range");
    for (int u = 0; u < nu; ++u)
        if (genes[u] < 0 || genes[u] >= G) return fail(c, SCC_ERR_INVALID, "gene index out of range");
    scc_enter(c);
    hipStream_t s0 = c->s0;
    const int ld = (nu + 63) & ~63;
    const int n = (int)(cell_hi - cell_lo);
    const int npad = std::max(16, (n + 15) & ~15);
    int rc;
    int *d_genes, *d_umap;
    double* d_X;
    void* d_part;
    if ((rc = ws(c, "d_genes", nu, &d_genes))) return rc;
    if ((rc = ws(c, "d_umap", G, &d_umap))) return rc;
    if ((rc = ws(c, "d_X", (size_t)npad * ld, &d_X))) return rc;
    const int nchunk_mean = 512;
    if ((rc = ws_get(c, "d_part", sizeof(double) * 2 * (size_t)nchunk_mean * ld, &d_part))) return rc;
    if ((rc = genes_h2d(c, d_genes, genes, nu, s0))) return rc;
    {
        Scope sc(c, "gather", s0);
        HIPCHK(c, scc_launch_gather(ds->dense ? nullptr : ds->d_indptr + cell_lo, ds->d_rows, ds->d_vals,
                                    ds->dense ? ds->d_dense + (size_t)cell_lo * G : nullptr, G, n, npad, d_umap,
                                    d_genes, nu, ld, d_X, s0));
    }
    {
        Scope sc(c, "center", s0);
        HIPCHK(c, scc_launch_colsum_dd(d_X, n, ld, nu, (dd*)d_part, nchunk_mean, (dd*)part, s0));
    }
    c->pca_nu = nu;
    c->pca_ld = ld;
    c->pca_N = N;
    c->pca_clo = cell_lo;
    c->pca_chi = cell_hi;
    c->pca_stage = 1;
    HIPCHK(c, hipStreamSynchronize(s0));  // the caller's collective reads `part` on its own stream
    return SCC_OK;
}

extern "C" int scc_pca_shard_gram(scc_ctx* c, const void* parts, int32_t world, void* gram)
{
    if (!c || !parts || !gram || world < 1) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_gram: bad argument");
    if (c->pca_stage < 1) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_gram: call scc_pca_shard_colsum first");
    scc_enter(c);
    hipStream_t s0 = c->s0;
    const int nu = c->pca_nu, ld = c->pca_ld;
    const int n = (int)(c->pca_chi - c->pca_clo);
    const int npad = std::max(16, (n + 15) & ~15);
    int rc;
    double *d_X, *d_mean, *d_slabs, *d_C;
    if ((rc = ws(c, "d_X", (size_t)npad * ld, &d_X))) return rc;
    if ((rc = ws(c, "d_mean", ld, &d_mean))) return rc;
    const int nchunk = gram_chunks(npad);
    if ((rc = ws(c, "d_slabs", (size_t)nchunk * ld * ld, &d_slabs))) return rc;
    if ((rc = ws(c, "d_C", (size_t)ld * ld, &d_C))) return rc;
    {
        Scope sc(c, "center", s0);
        HIPCHK(c, scc_launch_center_parts(d_X, n, nu, ld, (const dd*)parts, world, (double)c->pca_N, d_mean, s0));
    }
    {
        Scope sc(c, "gram", s0);
        HIPCHK(c, scc_launch_gram(d_X, npad, ld, nchunk, d_slabs, d_C, nullptr, npad, s0));
    }
    HIPCHK(c, hipMemcpy2DAsync(gram, sizeof(double) * nu, d_C, sizeof(double) * ld, sizeof(double) * nu, nu,
                               hipMemcpyDeviceToDevice, s0));
    c->pca_stage = 2;
    HIPCHK(c, hipStreamSynchronize(s0));
    return SCC_OK;
}

// The eigensolve of the summed Gram (Fast:398): top-k eigenvectors as [n_union][16]
// doubles (columns >= k zero) in `vecs` (device).  Run on ONE rank and broadcast:
// the hand-off kernel's workgroup count depends on arrival order, so two ranks
// could differ in the last bits (scc_pca_shard_project then scores every cell
// block with the same vectors).
extern "C" int scc_pca_shard_eigen(scc_ctx* c, const void* gram_sum, int32_t ncomp, void* vecs)
{
    if (!c || !gram_sum || !vecs) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_eigen: null argument");
    if (c->pca_stage < 2) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_eigen: call scc_pca_shard_gram first");
    const int nu = c->pca_nu, ld = c->pca_ld;
    const int k = ncomp > 0 ? ncomp : std::min(nu, 15);
    if (k > 16 || k > nu) return fail(c, SCC_ERR_UNSUPPORTED, "ncomp must be <= min(16, |U|)");
    scc_enter(c);
    hipStream_t s0 = c->s0;
    int rc;
    double *d_C, *d_W, *d_Z, *d_escr;
    if ((rc = ws(c, "d_C", (size_t)ld * ld, &d_C))) return rc;
    if ((rc = ws(c, "d_W", ld, &d_W))) return rc;
    if ((rc = ws(c, "d_Z", (size_t)ld * 16, &d_Z))) return rc;
    if ((rc = ws(c, "d_escr", scc_eigen_scratch_doubles(nu, ld, k), &d_escr))) return rc;
    HIPCHK(c, hipMemsetAsync(d_C, 0, sizeof(double) * (size_t)ld * ld, s0));
    HIPCHK(c, hipMemcpy2DAsync(d_C, sizeof(double) * ld, gram_sum, sizeof(double) * nu, sizeof(double) * nu, nu,
                               hipMemcpyDeviceToDevice, s0));
    unsigned int* d_eig_err = nullptr;
    {
        Scope sc(c, "eigen", s0);
        int nwg_used = 0;
        HIPCHK(c, scc_launch_eigen_topk(d_C, nu, ld, k, d_escr, d_Z, d_W, &d_eig_err, &nwg_used, nullptr, nullptr,
                                        eig_graph_key(c), s0));
    }
    HIPCHK(c, hipMemcpyAsync(vecs, d_Z, sizeof(double) * (size_t)nu * 16, hipMemcpyDeviceToDevice, s0));
    HIPCHK(c, hipMemcpyAsync(&c->eig_err, d_eig_err, sizeof(unsigned int), hipMemcpyDeviceToHost, s0));
    HIPCHK(c, hipStreamSynchronize(s0));
    c->last_ncomp = k;
    if (c->eig_err) return fail(c, SCC_ERR_HIP, "scc_pca_shard_eigen: eigensolver workgroup hand-off timed out");
    return SCC_OK;
}

// Scores of this rank's cell block from eigenvectors [n_union][16] (device).
extern "C" int scc_pca_shard_project(scc_ctx* c, const void* vecs, int32_t ncomp, void* scores)
{
    if (!c || !vecs || !scores) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_project: null argument");
    if (c->pca_stage < 2) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_project: call scc_pca_shard_gram first");
    const int nu = c->pca_nu, ld = c->pca_ld;
    const int k = ncomp > 0 ? ncomp : std::min(nu, 15);
    if (k > 16 || k > nu) return fail(c, SCC_ERR_UNSUPPORTED, "ncomp must be <= min(16, |U|)");
    scc_enter(c);
    hipStream_t s0 = c->s0;
    const int n = (int)(c->pca_chi - c->pca_clo);
    const int npad = std::max(16, (n + 15) & ~15);
    int rc;
    double* d_X;
    if ((rc = ws(c, "d_X", (size_t)npad * ld, &d_X))) return rc;
    if (n > 0) {
        Scope sc(c, "scores", s0);
        HIPCHK(c, scc_launch_scores(d_X, n, nu, ld, (const double*)vecs, k, (double*)scores + (size_t)c->pca_clo * 16,
                                    nullptr, s0));
    }
    HIPCHK(c, hipStreamSynchronize(s0));
    c->last_ncomp = k;
    return SCC_OK;
}

extern "C" int scc_pca_shard_scores(scc_ctx* c, const void* gram_sum, int32_t ncomp, void* scores)
{
    if (!c || !gram_sum || !scores) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_scores: null argument");
    if (c->pca_stage < 2) return fail(c, SCC_ERR_INVALID, "scc_pca_shard_scores: call scc_pca_shard_gram first");
    const int nu = c->pca_nu;
    int rc;
    double* d_V;
    if ((rc = ws(c, "d_V", (size_t)std::max(nu, 1) * 16, &d_V))) return rc;
    if ((rc = scc_pca_shard_eigen(c, gram_sum, ncomp, d_V))) return rc;
    return scc_pca_shard_project(c, d_V, ncomp, scores);
}

extern "C" int scc_distance_scores(scc_ctx* c, const void* scores, int64_t N64, int64_t col_lo, int64_t col_hi,
                                   void* dist_out, int32_t out_kind, int32_t out_f32)
{
    if (!c || !scores) return fail(c, SCC_ERR_INVALID, "scc_distance_scores: null argument");
    if (!dist_out && out_kind != SCC_PTR_DEVICE) return fail(c, SCC_ERR_INVALID, "scc_distance_scores: null output");
    if (N64 < 2 || N64 > INT32_MAX) return fail(c, SCC_ERR_INVALID, "scc_distance_scores: bad cell count");
    const int N = (int)N64;
    if (col_lo < 0 || col_hi > N || col_lo > col_hi) return fail(c, SCC_ERR_INVALID, "column slice out of range");
    scc_enter(c);
    hipStream_t s0 = c->s0;
    c->d_last_dist = nullptr;  // set again only when this call succeeds
    c->last_dist_pending.clear();
    auto colbase = [&](int64_t j) { return (size_t)j * (2 * (size_t)N - j - 1) / 2; };
    const size_t npairs = colbase(col_hi) - colbase(col_lo);
    const size_t es = out_f32 ? 4 : 8;
    void* d_out = dist_out;
    int rc;
    if (out_kind == SCC_PTR_HOST || !dist_out)
        if ((rc = ws_get(c, "d_dist", npairs * es, &d_out))) return rc;
    const double* P = (const double*)scores;
    auto emit = [&](int64_t a, int64_t b, void* dst) { return scc_launch_dist_euclid(P, N, (int)a, (int)b, dst, out_f32, s0); };
    {
        Scope sc(c, "dist", s0);
        if (out_kind == SCC_PTR_HOST) {
            if ((rc = stream_to_host(c, N, col_lo, col_hi, es, (char*)d_out, (char*)dist_out, emit))) return rc;
        } else {
            HIPCHK(c, emit(col_lo, col_hi, d_out));
        }
    }
    HIPCHK(c, hipStreamSynchronize(s0));
    const bool own = out_kind == SCC_PTR_HOST || !dist_out;
    c->d_last_dist = (own && col_lo == 0 && col_hi == N) ? d_out : nullptr;
    c->last_dist_n = N;
    c->last_dist_f32 = out_f32 ? 1 : 0;
    return SCC_OK;
}

extern "C" int scc_silhouette(scc_ctx* c, int64_t n_cells, const int32_t* groups, const void* dist, int32_t dist_f32,
                              double* widths, double* clus_avg, int32_t* n_groups)
{
    if (!c || !groups) return fail(c, SCC_ERR_INVALID, "scc_silhouette: null argument");
    const int N = (int)n_cells;
    if (N < 2) return fail(c, SCC_ERR_INVALID, "scc_silhouette: need at least two cells");
    const void* D = dist;
    int f32 = dist_f32 ? 1 : 0;
    if (!D) {
        if (!c->d_last_dist || c->last_dist_n != N)
            return fail(c, SCC_ERR_INVALID, "scc_silhouette: no full scc_distance output of this size is kept");
        D = c->d_last_dist;
        f32 = c->last_dist_f32;
        const size_t es = f32 ? 4 : 8;
        hipSetDevice(c->device);
        for (const auto& sl : c->last_dist_pending) {  // peer slices of a device-list distance
            char* dst = (char*)c->d_last_dist + sl.off * es;
            if (sl.dev == c->device)
                HIPCHK(c, hipMemcpyAsync(dst, sl.ptr, sl.n * es, hipMemcpyDeviceToDevice, c->s0));
            else
                HIPCHK(c, hipMemcpyPeerAsync(dst, c->device, sl.ptr, sl.dev, sl.n * es, c->s0));
        }
        c->last_dist_pending.clear();
    }
    // cluster codes in increasing id order (silhouette's sorted clusters)
    std::vector<int32_t> ids(groups, groups + N);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const int C = (int)ids.size();
    if (n_groups) *n_groups = C;
    if (C < 2 || C >= N) return fail(c, SCC_ERR_INVALID, "silhouette needs 2 <= clusters < cells (R returns NA)");
    std::vector<int> lab(N), cnt(C, 0);
    for (int i = 0; i < N; ++i) {
        lab[i] = (int)(std::lower_bound(ids.begin(), ids.end(), groups[i]) - ids.begin());
        cnt[lab[i]]++;
    }
    scc_enter(c);
    hipStream_t s0 = c->s0;
    int rc;
    int *d_lab, *d_cnt;
    double *d_part, *d_w;
    if ((rc = ws(c, "sil_lab", N, &d_lab))) return rc;
    if ((rc = ws(c, "sil_cnt", C, &d_cnt))) return rc;
    if ((rc = ws(c, "sil_part", scc_sil_scratch_doubles(N, C), &d_part))) return rc;
    if ((rc = ws(c, "sil_w", N, &d_w))) return rc;
    HIPCHK(c, hipMemcpyAsync(d_lab, lab.data(), sizeof(int) * N, hipMemcpyHostToDevice, s0));
    HIPCHK(c, hipMemcpyAsync(d_cnt, cnt.data(), sizeof(int) * C, hipMemcpyHostToDevice, s0));
    {
        Scope sc(c, "silhouette", s0);
        HIPCHK(c, scc_launch_silhouette(D, f32, N, d_lab, d_cnt, C, d_part, d_w, s0));
    }
    std::vector<double> w(N);
    HIPCHK(c, hipMemcpyAsync(w.data(), d_w, sizeof(double) * N, hipMemcpyDeviceToHost, s0));
    HIPCHK(c, hipStreamSynchronize(s0));
    // widths read from an engine-kept distance whose eigensolve failed are
    // not an answer: report the flag that distance left (and drop it)
    if (!dist && (rc = check_pending_eig(c))) {
        c->d_last_dist = nullptr;
        return rc;
    }
    if (widths) std::copy(w.begin(), w.end(), widths);
    if (clus_avg) {  // summary(.)$clus.avg.widths: mean width per cluster (long double sums, R mean)
        std::vector<long double> sum(C, 0.0L);
        for (int i = 0; i < N; ++i) sum[lab[i]] += w[i];
        for (int k = 0; k < C; ++k) clus_avg[k] = (double)(sum[k] / cnt[k]);
    }
    return SCC_OK;
}

extern "C" int scc_last_pca_scores(const scc_ctx* c, double* scores, int32_t* ncomp)
{
    if (!c) return SCC_ERR_INVALID;
    if (ncomp) *ncomp = c->last_ncomp;
    if (scores && c->last_ncomp > 0 && c->d_last_scores) {
        scc_ctx* cc = const_cast<scc_ctx*>(c);
        hipSetDevice(c->device);
        std::vector<double> buf((size_t)c->last_n * 16);
        HIPCHK(cc, hipMemcpy(buf.data(), c->d_last_scores, sizeof(double) * buf.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < (size_t)c->last_n; ++i)
            for (int q = 0; q < c->last_ncomp; ++q) scores[i * c->last_ncomp + q] = buf[i * 16 + q];
    }
    return SCC_OK;
}
