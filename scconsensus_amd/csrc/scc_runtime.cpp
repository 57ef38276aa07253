// scc_runtime.cpp — host runtime behind the C ABI (include/scc.h).
//
// Owns the HIP device, two streams, a grow-only HBM workspace, the exact
// Wilcoxon count table, and optional HIP-event kernel timers.  The whole DE
// stage is one stream-ordered launch sequence (the bigger genes run on a side
// stream concurrently with the LDS-resident ones); the host synchronises once
// per call to read the union size.  No CPU fallback exists: without a HIP
// device every entry point returns SCC_ERR_HIP.
#include "scc_internal.hpp"

#include <atomic>
#include <cstring>
#include <memory>
#include <thread>

using namespace scc_rt;

// ====================================================================== ctx
static int ctx_create_one(int device, bool profile, scc_ctx** out)
{
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        hipGetLastError();
        return SCC_ERR_HIP;
    }
    if (device < 0 || device >= ndev) return SCC_ERR_INVALID;
    static std::atomic<uint64_t> next_serial{1};
    scc_ctx* c = new scc_ctx();
    c->serial = next_serial.fetch_add(1);
    c->device = device;
    c->profile = profile;
    if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->s0, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s1, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&c->sw[0], hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->sw[1], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_wj[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_wj[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_wfork, hipEventDisableTiming) != hipSuccess) {
        hipGetLastError();
        delete c;
        return SCC_ERR_HIP;
    }
    c->own_s0 = c->s0;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) {
        hipGetLastError();
        c->n_cu = 256;
    }
    *out = c;
    return SCC_OK;
}

extern "C" int scc_ctx_create(const scc_opts* opts, scc_ctx** out)
{
    if (!out) return SCC_ERR_INVALID;
    *out = nullptr;
    const bool profile = opts ? (opts->profile != 0) : false;
    const int nd = (opts && opts->n_devices > 1) ? opts->n_devices : 1;
    if (nd > 1 && !opts->devices) return SCC_ERR_INVALID;
    const int dev0 = nd > 1 ? opts->devices[0] : (opts ? opts->device : 0);
    scc_ctx* c = nullptr;
    int rc = ctx_create_one(dev0, profile, &c);
    if (rc) return rc;
    for (int i = 1; i < nd; ++i) {
        scc_ctx* p = nullptr;
        if ((rc = ctx_create_one(opts->devices[i], profile, &p))) {
            scc_ctx_destroy(c);
            return rc;
        }
        c->peers.push_back(p);
        if (p->device != c->device) {  // xGMI peer access both ways (already enabled is fine)
            hipSetDevice(c->device);
            if (hipDeviceEnablePeerAccess(p->device, 0) != hipSuccess) hipGetLastError();
            hipSetDevice(p->device);
            if (hipDeviceEnablePeerAccess(c->device, 0) != hipSuccess) hipGetLastError();
        }
    }
    scc_enter(c);
    *out = c;
    return SCC_OK;
}

extern "C" int scc_device_count(int32_t* n)
{
    if (!n) return SCC_ERR_INVALID;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess) {
        hipGetLastError();
        nd = 0;
    }
    *n = nd;
    return SCC_OK;
}

extern "C" void scc_distance_release(scc_ctx* c);

extern "C" void scc_ctx_destroy(scc_ctx* c)
{
    if (!c) return;
    for (scc_ctx* p : c->peers) scc_ctx_destroy(p);
    c->peers.clear();
    scc_enter(c);
    scc_distance_release(c);
    hipStreamSynchronize(c->s0);
    hipStreamSynchronize(c->s1);
    for (auto& kv : c->ws) {
        scc_fsi_forget(kv.second.first, kv.second.second);
        hipFree(kv.second.first);
    }
    for (auto& pe : c->pending) {
        hipEventDestroy(pe.a);
        hipEventDestroy(pe.b);
    }
    for (auto e : c->ev_pool) hipEventDestroy(e);
    if (c->h_stage) hipHostFree(c->h_stage);
    if (c->h_tab) hipHostFree(c->h_tab);
    if (c->h_flag) hipHostFree(c->h_flag);
    if (c->ev_genes) hipEventSynchronize(c->ev_genes), hipEventDestroy(c->ev_genes);
    if (c->h_genes) hipHostFree(c->h_genes);
    if (c->h_dstage) hipHostFree(c->h_dstage);
    hipEventDestroy(c->ev_fork);
    hipEventDestroy(c->ev_join);
    for (int i = 0; i < 2; ++i) {
        hipStreamSynchronize(c->sw[i]);
        hipStreamDestroy(c->sw[i]);
        hipEventDestroy(c->ev_wj[i]);
    }
    hipEventDestroy(c->ev_wfork);
    hipStreamSynchronize(c->s0);
    hipStreamDestroy(c->own_s0);
    hipStreamDestroy(c->s1);
    delete c;
}

extern "C" const char* scc_ctx_last_error(const scc_ctx* c) { return c ? c->err.c_str() : "null context"; }

namespace scc_rt {
void scc_enter(const scc_ctx* c)
{
    hipSetDevice(c->device);
    (void)hipGetLastError();
}

int check_pending_eig(scc_ctx* c)
{
    if (!c->eig_flag_pending || !c->h_flag) return SCC_OK;
    c->eig_flag_pending = false;
    const unsigned int v = *(volatile unsigned int*)c->h_flag;
    *(volatile unsigned int*)c->h_flag = 0;
    c->eig_err = v;
    if (v) return fail(c, SCC_ERR_HIP, "scc_distance: eigensolver workgroup hand-off timed out");
    return SCC_OK;
}

}  // namespace scc_rt

extern "C" int scc_ctx_synchronize(scc_ctx* c)
{
    if (!c) return SCC_ERR_INVALID;
    scc_enter(c);
    HIPCHK(c, hipStreamSynchronize(c->s0));
    HIPCHK(c, hipStreamSynchronize(c->s1));
    for (scc_ctx* p : c->peers) {
        int rc = scc_ctx_synchronize(p);
        if (rc) return fail(c, rc, p->err);
    }
    scc_enter(c);
    return check_pending_eig(c);
}

extern "C" int scc_ctx_set_stream(scc_ctx* c, void* stream, int32_t external)
{
    if (!c) return SCC_ERR_INVALID;
    scc_enter(c);
    HIPCHK(c, hipStreamSynchronize(c->s0));  // work already queued on the old stream first
    c->s0 = external ? (hipStream_t)stream : c->own_s0;
    return SCC_OK;
}

extern "C" int scc_ctx_kernel_time(const scc_ctx* cc, const char* name, double* total_ms, int64_t* launches)
{
    scc_ctx* c = const_cast<scc_ctx*>(cc);
    if (!c || !name) return SCC_ERR_INVALID;
    scc_enter(c);
    resolve_timers(c);
    auto it = c->timers.find(name);
    if (total_ms) *total_ms = it == c->timers.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == c->timers.end() ? 0 : it->second.n;
    return SCC_OK;
}

extern "C" void scc_ctx_reset_timers(scc_ctx* c)
{
    if (!c) return;
    scc_enter(c);
    resolve_timers(c);
    c->timers.clear();
}

// ====================================================================== dataset
// device list: the dataset's replica on every peer engine (the same device:
// its buffers borrowed; another device: owned copies over xGMI)
static int replicate(scc_ctx* c, scc_dataset* d)
{
    for (scc_ctx* p : c->peers) {
        scc_dataset* r = new scc_dataset();
        r->ctx = p;
        r->device = p->device;
        r->G = d->G;
        r->N = d->N;
        r->nnz = d->nnz;
        r->dense = d->dense;
        d->reps.push_back(r);
        if (p->device == c->device) {
            r->d_indptr = d->d_indptr;
            r->d_rows = d->d_rows;
            r->d_vals = d->d_vals;
            r->d_dense = d->d_dense;
            r->owned = false;
            continue;
        }
        r->owned = true;
        hipSetDevice(p->device);
        auto peer = [&](void** dst, const void* src, size_t bytes) {
            if (hipMalloc(dst, std::max<size_t>(bytes, 8)) != hipSuccess) {
                hipGetLastError();
                *dst = nullptr;
                return false;
            }
            if (bytes && hipMemcpyPeerAsync(*dst, p->device, src, c->device, bytes, p->s0) != hipSuccess) {
                hipGetLastError();
                return false;
            }
            return true;
        };
        bool ok = true;
        if (d->dense) {
            ok = peer((void**)&r->d_dense, d->d_dense, sizeof(double) * (size_t)d->G * d->N);
        } else {
            ok = peer((void**)&r->d_indptr, d->d_indptr, sizeof(long long) * (d->N + 1)) &&
                 peer((void**)&r->d_rows, d->d_rows, sizeof(int) * d->nnz) &&
                 peer((void**)&r->d_vals, d->d_vals, sizeof(double) * d->nnz);
        }
        if (!ok || hipStreamSynchronize(p->s0) != hipSuccess) {
            hipGetLastError();
            hipSetDevice(c->device);
            return fail(c, SCC_ERR_OOM, "dataset replication to a peer device failed");
        }
    }
    scc_enter(c);
    return SCC_OK;
}

static int finish_create(scc_ctx* c, scc_dataset* d, scc_dataset** out)
{
    int rc = replicate(c, d);
    if (rc) {
        scc_dataset_destroy(d);
        return rc;
    }
    *out = d;
    return SCC_OK;
}

extern "C" int scc_dataset_create_csc(scc_ctx* c, const int64_t* indptr, const int32_t* rows, const double* vals,
                                      int64_t G, int64_t N, int64_t nnz, int32_t kind, scc_dataset** out)
{
    if (!c || !out || !indptr || G <= 0 || N <= 0 || nnz < 0 || (nnz > 0 && (!rows || !vals)))
        return fail(c, SCC_ERR_INVALID, "scc_dataset_create_csc: bad arguments");
    if (G > INT32_MAX || N > INT32_MAX) return fail(c, SCC_ERR_UNSUPPORTED, "dimensions exceed int32");
    scc_enter(c);
    scc_dataset* d = new scc_dataset();
    d->ctx = c;
    d->device = c->device;
    d->G = G;
    d->N = N;
    d->nnz = nnz;
    if (kind == SCC_PTR_DEVICE) {
        d->d_indptr = (long long*)indptr;
        d->d_rows = (int*)rows;
        d->d_vals = (double*)vals;
        d->owned = false;
    } else {
        d->owned = true;
        if (hipMalloc(&d->d_indptr, sizeof(long long) * (N + 1)) != hipSuccess ||
            hipMalloc(&d->d_rows, sizeof(int) * std::max<int64_t>(nnz, 1)) != hipSuccess ||
            hipMalloc(&d->d_vals, sizeof(double) * std::max<int64_t>(nnz, 1)) != hipSuccess) {
            hipGetLastError();
            scc_dataset_destroy(d);
            return fail(c, SCC_ERR_OOM, "dataset allocation failed");
        }
        hipMemcpyAsync(d->d_indptr, indptr, sizeof(long long) * (N + 1), hipMemcpyHostToDevice, c->s0);
        if (nnz > 0) {
            hipMemcpyAsync(d->d_rows, rows, sizeof(int) * nnz, hipMemcpyHostToDevice, c->s0);
            hipMemcpyAsync(d->d_vals, vals, sizeof(double) * nnz, hipMemcpyHostToDevice, c->s0);
        }
        if (hipStreamSynchronize(c->s0) != hipSuccess) {
            hipGetLastError();
            scc_dataset_destroy(d);
            return fail(c, SCC_ERR_HIP, "dataset upload failed");
        }
    }
    return finish_create(c, d, out);
}

extern "C" int scc_dataset_create_csr(scc_ctx* c, const int64_t* indptr, const int32_t* cols, const double* vals,
                                      int64_t G, int64_t N, int64_t nnz, int32_t kind, scc_dataset** out)
{
    if (!c || !out || !indptr || G <= 0 || N <= 0 || nnz < 0 || (nnz > 0 && (!cols || !vals)))
        return fail(c, SCC_ERR_INVALID, "scc_dataset_create_csr: bad arguments");
    if (G > INT32_MAX || N > INT32_MAX) return fail(c, SCC_ERR_UNSUPPORTED, "dimensions exceed int32");
    if (nnz > UINT32_MAX) return fail(c, SCC_ERR_UNSUPPORTED, "more than 2^32 stored values");
    scc_enter(c);
    hipStream_t s0 = c->s0;
    // the CSR on the device (borrowed, or a temporary upload)
    long long* d_ip = nullptr;
    int* d_cols = nullptr;
    double* d_vals = nullptr;
    std::vector<void*> tmp;
    auto cleanup = [&]() {
        hipStreamSynchronize(s0);
        for (void* p : tmp) hipFree(p);
    };
    auto dalloc = [&](void** p, size_t bytes) {
        if (hipMalloc(p, std::max<size_t>(bytes, 8)) != hipSuccess) {
            hipGetLastError();
            *p = nullptr;
            return false;
        }
        tmp.push_back(*p);
        return true;
    };
    if (kind == SCC_PTR_DEVICE) {
        d_ip = (long long*)indptr;
        d_cols = (int*)cols;
        d_vals = (double*)vals;
    } else {
        if (!dalloc((void**)&d_ip, sizeof(long long) * (G + 1)) || !dalloc((void**)&d_cols, sizeof(int) * nnz) ||
            !dalloc((void**)&d_vals, sizeof(double) * nnz)) {
            cleanup();
            return fail(c, SCC_ERR_OOM, "CSR upload allocation failed");
        }
        hipMemcpyAsync(d_ip, indptr, sizeof(long long) * (G + 1), hipMemcpyHostToDevice, s0);
        if (nnz > 0) {
            hipMemcpyAsync(d_cols, cols, sizeof(int) * nnz, hipMemcpyHostToDevice, s0);
            hipMemcpyAsync(d_vals, vals, sizeof(double) * nnz, hipMemcpyHostToDevice, s0);
        }
    }
    // host-side shape checks on the row pointer (G+1 words)
    std::vector<long long> hip_(G + 1);
    if (hipMemcpyAsync(hip_.data(), d_ip, sizeof(long long) * (G + 1), hipMemcpyDeviceToHost, s0) != hipSuccess ||
        hipStreamSynchronize(s0) != hipSuccess) {
        hipGetLastError();
        cleanup();
        return fail(c, SCC_ERR_HIP, "CSR upload failed");
    }
    if (hip_[0] != 0 || hip_[G] != nnz) {
        cleanup();
        return fail(c, SCC_ERR_INVALID, "CSR indptr must start at 0 and end at nnz");
    }
    for (int64_t g = 0; g < G; ++g)
        if (hip_[g + 1] < hip_[g]) {
            cleanup();
            return fail(c, SCC_ERR_INVALID, "CSR indptr is not non-decreasing");
        }
    // the transpose's plan and scratch (scc_csr.hip: bounds, region and group
    // offsets, the 10-B-per-entry intermediate)
    ScCsrPlan plan;
    if (scc_csr_plan(G, N, nnz, &plan) != 0) {
        cleanup();
        return fail(c, SCC_ERR_UNSUPPORTED, "scc_dataset_create_csr: more than 262,144 genes");
    }
    void* scratch = nullptr;
    int* d_err = nullptr;
    if (!dalloc(&scratch, plan.bytes) || !dalloc((void**)&d_err, sizeof(int))) {
        cleanup();
        return fail(c, SCC_ERR_OOM, "CSR transpose scratch allocation failed");
    }
    scc_dataset* d = new scc_dataset();
    d->ctx = c;
    d->device = c->device;
    d->G = G;
    d->N = N;
    d->nnz = nnz;
    d->owned = true;
    if (hipMalloc(&d->d_indptr, sizeof(long long) * (N + 1)) != hipSuccess ||
        hipMalloc(&d->d_rows, sizeof(int) * std::max<int64_t>(nnz, 1)) != hipSuccess ||
        hipMalloc(&d->d_vals, sizeof(double) * std::max<int64_t>(nnz, 1)) != hipSuccess) {
        hipGetLastError();
        cleanup();
        scc_dataset_destroy(d);
        return fail(c, SCC_ERR_OOM, "dataset allocation failed");
    }
    // validation first (columns in range, strictly ascending per gene), then
    // the transpose only over a valid matrix
    int herr = 0;
    hipError_t e = hipMemsetAsync(d_err, 0, sizeof(int), s0);
    if (e == hipSuccess) e = scc_launch_csr_check(&plan, d_ip, d_cols, scratch, d_err, s0);
    if (e == hipSuccess) e = hipMemcpyAsync(&herr, d_err, sizeof(int), hipMemcpyDeviceToHost, s0);
    if (e == hipSuccess) e = hipStreamSynchronize(s0);
    if (e == hipSuccess && herr) {
        cleanup();
        scc_dataset_destroy(d);
        return fail(c, SCC_ERR_INVALID, "CSR column index out of range or not strictly ascending within a gene");
    }
    if (e == hipSuccess)
        e = scc_launch_csr_to_csc(&plan, d_ip, d_cols, d_vals, scratch, d->d_indptr, d->d_rows, d->d_vals, s0);
    if (e == hipSuccess) e = hipStreamSynchronize(s0);
    cleanup();
    if (e != hipSuccess) {
        hipGetLastError();
        scc_dataset_destroy(d);
        return fail(c, SCC_ERR_HIP, std::string("CSR transpose failed: ") + hipGetErrorString(e));
    }
    return finish_create(c, d, out);
}

extern "C" int scc_dataset_create_dense(scc_ctx* c, const double* x, int64_t G, int64_t N, int32_t kind,
                                        scc_dataset** out)
{
    if (!c || !out || !x || G <= 0 || N <= 0) return fail(c, SCC_ERR_INVALID, "scc_dataset_create_dense: bad arguments");
    if (G > INT32_MAX || N > INT32_MAX) return fail(c, SCC_ERR_UNSUPPORTED, "dimensions exceed int32");
    scc_enter(c);
    scc_dataset* d = new scc_dataset();
    d->ctx = c;
    d->device = c->device;
    d->G = G;
    d->N = N;
    d->nnz = G * N;
    d->dense = true;
    if (kind == SCC_PTR_DEVICE) {
        d->d_dense = (double*)x;
    } else {
        d->owned = true;
        if (hipMalloc(&d->d_dense, sizeof(double) * G * N) != hipSuccess) {
            hipGetLastError();
            delete d;
            return fail(c, SCC_ERR_OOM, "dataset allocation failed");
        }
        if (hipMemcpy(d->d_dense, x, sizeof(double) * G * N, hipMemcpyHostToDevice) != hipSuccess) {
            hipGetLastError();
            scc_dataset_destroy(d);
            return fail(c, SCC_ERR_HIP, "dataset upload failed");
        }
    }
    return finish_create(c, d, out);
}

extern "C" int scc_dataset_read_csc(scc_dataset* d, int64_t* indptr, int32_t* rows, double* vals)
{
    if (!d || !indptr || (!rows != !vals))
        return fail(d ? d->ctx : nullptr, SCC_ERR_INVALID, "scc_dataset_read_csc: bad arguments");
    if (d->dense || !d->d_indptr) return fail(d->ctx, SCC_ERR_INVALID, "scc_dataset_read_csc: not a sparse dataset");
    scc_enter(d->ctx);
    hipStream_t s0 = d->ctx->s0;
    hipError_t e = hipMemcpyAsync(indptr, d->d_indptr, sizeof(int64_t) * (d->N + 1), hipMemcpyDeviceToHost, s0);
    if (e == hipSuccess && d->nnz > 0 && rows)
        e = hipMemcpyAsync(rows, d->d_rows, sizeof(int32_t) * d->nnz, hipMemcpyDeviceToHost, s0);
    if (e == hipSuccess && d->nnz > 0 && vals)
        e = hipMemcpyAsync(vals, d->d_vals, sizeof(double) * d->nnz, hipMemcpyDeviceToHost, s0);
    if (e == hipSuccess) e = hipStreamSynchronize(s0);
    if (e != hipSuccess) {
        hipGetLastError();
        return fail(d->ctx, SCC_ERR_HIP, std::string("scc_dataset_read_csc: ") + hipGetErrorString(e));
    }
    return SCC_OK;
}

extern "C" void scc_dataset_destroy(scc_dataset* d)
{
    if (!d) return;
    for (scc_dataset* r : d->reps) scc_dataset_destroy(r);
    d->reps.clear();
    if (d->owned || d->d_nodg || d->d_tbnd) {
        hipSetDevice(d->device);
        hipDeviceSynchronize();
    }
    if (d->owned) {
        hipFree(d->d_indptr);
        hipFree(d->d_rows);
        hipFree(d->d_vals);
        hipFree(d->d_dense);
    }
    hipFree(d->d_nodg);
    hipFree(d->d_tbnd);
    delete d;
}

// ====================================================================== DE
// stage DE_FULL: the whole DE for genes [glo, ghi) (all genes: scc_de_run).
// stage DE_SHARD: the per-(pair, gene) stage for the gene shard [glo, ghi),
//   packed into `shard` (zero outside the shard, so the shards of all ranks
//   combine by an integer sum: scc_de_shard_bytes layout) -- no selection.
// stage DE_FINISH: `shard` holds every gene's (pair, gene) cells (the sum of
//   all ranks' shards); per-pair BH, filters, top-N and the union, on the
//   context that ran this rank's DE_SHARD for the same inputs.
// stage DE_SHARD_REC / DE_FINISH_REC: the same with the compact exchange
//   (scc_de_record per tested (pair, gene) cell; scc_exchange.hip).
enum { DE_FULL = 0, DE_SHARD = 1, DE_FINISH = 2, DE_SHARD_REC = 3, DE_FINISH_REC = 4 };

extern "C" {
int scc_rec_blocks(long long cells);
hipError_t scc_launch_rec_count(const uint8_t* flags, int G, int P, int glo, int ghi, int all, uint32_t* cnt,
                                hipStream_t st);
hipError_t scc_launch_rec_pack(const uint8_t* flags, int G, int P, int glo, int ghi, int all, const long long* off,
                               const double* p, const double* lfc, const double* pct1, const double* pct2,
                               const long long* u2, const long long* t, scc_de_record* out, hipStream_t st);
hipError_t scc_launch_rec_scatter(const scc_de_record* rec, long long n, int G, int P, double* p, double* lfc,
                                  double* pct1, double* pct2, long long* u2, long long* t, uint8_t* flags, int* err,
                                  int plo, int phi, hipStream_t st);
}

struct RecIO {  // the compact exchange's buffers (DE_SHARD_REC out, DE_FINISH_REC in)
    void* out = nullptr;
    int64_t cap = 0;
    int64_t* n_out = nullptr;
    const void* in = nullptr;
    const int64_t* counts = nullptr;
    int nblocks = 0;
    int64_t stride = 0;
    // DE_FINISH_REC for pairs [pair_lo, pair_hi) only: the per-gene first
    // occurrence keys go to first_out (device u64 [G]) and no result is built
    int pair_lo = 0, pair_hi = 0;
    void* first_out = nullptr;
};

static int de_run_body(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K, const scc_de_params* prm,
                       int stage, int64_t glo64, int64_t ghi64, void* shard, scc_de_result** out,
                       const RecIO* rio);
extern "C" void scc_rank_split_diag(hipStream_t st, int ngenes);

static int de_run_impl(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K, const scc_de_params* prm,
                       int stage, int64_t glo64, int64_t ghi64, void* shard, scc_de_result** out,
                       const RecIO* rio = nullptr)
{
    return de_run_body(c, ds, code, K, prm, stage, glo64, ghi64, shard, out, rio);
}

static int de_run_body(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K, const scc_de_params* prm,
                       int stage, int64_t glo64, int64_t ghi64, void* shard, scc_de_result** out,
                       const RecIO* rio)
{
    const bool shard_stage = stage == DE_SHARD || stage == DE_SHARD_REC;
    const bool finish_stage = stage == DE_FINISH || stage == DE_FINISH_REC;
    if (!c || !ds || !code || !prm || (!shard_stage && !out && !(rio && rio->first_out)) || ((stage == DE_SHARD || stage == DE_FINISH) && !shard) ||
        ((stage == DE_SHARD_REC || stage == DE_FINISH_REC) && !rio))
        return fail(c, SCC_ERR_INVALID, "scc_de_run: null argument");
    if (out) *out = nullptr;
    if (ds->ctx != c) return fail(c, SCC_ERR_INVALID, "dataset belongs to another context");
    if (prm->mode != SCC_DE_FAST && prm->mode != SCC_DE_SLOW) return fail(c, SCC_ERR_INVALID, "bad mode");
    if (prm->test != SCC_TEST_WILCOX && (prm->test != SCC_TEST_T || prm->mode != SCC_DE_FAST))
        return fail(c, SCC_ERR_INVALID, "test: SCC_TEST_WILCOX, or SCC_TEST_T with SCC_DE_FAST");
    if (K < 2) return fail(c, SCC_ERR_INVALID, "need at least two clusters");
    if (K > kMaxK)
        return fail(c, SCC_ERR_UNSUPPORTED,
                    "K > 128 clusters: one engine run holds 128 (scc_de_run cuts larger K into group-pair runs; "
                    "the gene-shard entry points do not)");
    scc_enter(c);
    const int G = (int)ds->G, N = (int)ds->N, P = K * (K - 1) / 2;
    const bool fast = prm->mode == SCC_DE_FAST;
    // cluster sizes (host: the codes are a host array at the R boundary)
    std::vector<int> nclu(K, 0);
    for (int i = 0; i < N; ++i) {
        const int a = code[i];
        if (a < -1 || a >= K) return fail(c, SCC_ERR_INVALID, "code out of range");
        if (a >= 0) nclu[a]++;
    }
    for (int a = 0; a < K; ++a) {
        if (nclu[a] == 0) return fail(c, SCC_ERR_INVALID, "empty cluster");
        // ComputePairWiseDE: min.cells.group = 3 (Fast:76,208-213)
        if (fast && nclu[a] < 3) return fail(c, SCC_ERR_RSTOP, "cluster has fewer than 3 cells (R stop())");
    }
    if (glo64 < 0 || ghi64 > G || glo64 > ghi64) return fail(c, SCC_ERR_INVALID, "gene shard out of range");
    const int glo = (int)glo64, ghi = (int)ghi64;
    const int64_t GK = (int64_t)G * K;
    const size_t PG = (size_t)P * G;
    // Cells in cluster order: kept cells by code, then unkept ones.  Count
    // chunks of <= kCountChunk cells never straddle clusters; scatter chunks
    // group <= kScatterCC count chunks of one cluster.
    std::vector<int>& H = c->host_tables;
    std::vector<int> start(K + 1, 0);
    for (int a = 0; a < K; ++a) start[a + 1] = start[a] + nclu[a];
    const int nkept = start[K];
    // (a finish stage reads no cell order: the records carry every statistic)
    std::vector<int> perm(finish_stage ? 0 : N), fill(start.begin(), start.end() - 1);
    if (!finish_stage) {
        int u = nkept;
        for (int i = 0; i < N; ++i) perm[code[i] >= 0 ? fill[code[i]]++ : u++] = i;
    }
    std::vector<int> cc_p0, cc_code, sc_cc0, cl_cc(K + 1);
    // scatter chunks of 2 count chunks (64 cells) when a cell has >= 16 stored
    // values per gene tile (config B / D: ~29; ingest B 0.45 -> 0.40 ms, D 5.97
    // -> 5.79), else 8 (config E: ~8 per tile, where small chunks leave the
    // workgroups too little work for their fixed cost: 64 cells 16.5 ms, 128
    // cells 12.0-12.2, 192 cells 11.0, 256 cells 10.4-10.5, round 6); SCC_SC_CC overrides
    const int64_t ntile_h = (ds->G + scc_ingest_gene_tile() - 1) / scc_ingest_gene_tile();
    const bool dense_tiles = ds->nnz >= 16 * (int64_t)std::max(1, N) * std::max<int64_t>(1, ntile_h);
    const int scatter_cc =
        std::min(kScatterCC, std::max(1, env_int("SCC_SC_CC", dense_tiles ? 2 : kScatterCC)));
    for (int a = 0; a < K; ++a) {
        cl_cc[a] = (int)cc_code.size();
        for (int p = start[a]; p < start[a + 1]; p += kCountChunk) {
            cc_p0.push_back(p);
            cc_code.push_back(a);
        }
    }
    const int nc_kept = (int)cc_code.size();
    cl_cc[K] = nc_kept;
    for (int a = 0; a < K; ++a)
        for (int q = cl_cc[a]; q < cl_cc[a + 1]; q += scatter_cc) sc_cc0.push_back(q);
    const int ns = (int)sc_cc0.size();
    sc_cc0.push_back(nc_kept);
    for (int p = nkept; p < N; p += kCountChunk) {
        cc_p0.push_back(p);
        cc_code.push_back(-1);
    }
    const int nc = (int)cc_code.size();
    cc_p0.push_back(N);
    const int gt = scc_ingest_gene_tile();
    const int ntile = (G + gt - 1) / gt;
    H.clear();
    H.insert(H.end(), perm.begin(), perm.end());
    const size_t o_ccp0 = H.size();
    H.insert(H.end(), cc_p0.begin(), cc_p0.end());
    const size_t o_cccode = H.size();
    H.insert(H.end(), cc_code.begin(), cc_code.end());
    const size_t o_sccc0 = H.size();
    H.insert(H.end(), sc_cc0.begin(), sc_cc0.end());
    const size_t o_clcc = H.size();
    H.insert(H.end(), cl_cc.begin(), cl_cc.end());
    const size_t o_nclu = H.size();
    H.insert(H.end(), nclu.begin(), nclu.end());

    int rc;
    int *d_tab, *d_nodg, *d_splitg, *d_counts, *d_err, *d_tested, *d_union, *d_nu;
    uint32_t *d_cnt, *d_cntpos, *d_cntneg, *d_gix, *d_gwin;
    long long *d_gstart, *d_scan, *d_rowoff, *d_bnd;
    unsigned long long* d_keys;
    uint8_t *d_gcode, *d_gsc, *d_codes2;
    unsigned long long *d_keys2, *d_acc;
    ScRankItem* d_items;
    dd* d_wexp;
    dd* d_gexp;
    double *d_mx, *d_me;
    long long *d_u2, *d_t;
    unsigned long long* d_first;
    double *d_p, *d_lfc, *d_pct1, *d_pct2;
    uint8_t* d_flags;
    const int nwaves = nc * SCC_ING_HIST_WAVES;
    const int64_t nnz1 = std::max<int64_t>(ds->nnz, 1);
#define WS(name, n, ptr)                                  \
    do {                                                  \
        if ((rc = ws(c, name, (size_t)(n), &(ptr)))) return rc; \
    } while (0)
    WS("tables", H.size(), d_tab);
    WS("nodg", N, d_nodg);
    WS("cnt", (size_t)(nc + 1) * G, d_cnt);
    WS("bnd", ds->dense ? 1 : (size_t)N * (ntile + 1), d_bnd);
    WS("gstart", G + 1, d_gstart);
    WS("scan", scc_scan_scratch_blocks(G) + 1, d_scan);
    WS("keys", nnz1, d_keys);
    WS("gix", 2 * (size_t)nnz1, d_gix);
    WS("gcode", nnz1, d_gcode);
    WS("gwin", nnz1, d_gwin);
    WS("gsc", nnz1, d_gsc);
    WS("keys2", nnz1, d_keys2);
    WS("codes2", nnz1, d_codes2);
    {
        void* p;
        if ((rc = ws_get(c, "wexp", sizeof(double) * 2 * (nwaves + 1), &p))) return rc;
        d_wexp = (dd*)p;
        d_gexp = (dd*)((char*)p + sizeof(double) * 2 * nwaves);
    }
    WS("splitg", (size_t)G, d_splitg);
    WS("counts", SCC_NCOUNTS * SCC_CNT_STRIDE, d_counts);
    WS("err", 4, d_err);
    WS("mx", GK, d_mx);
    WS("me", GK, d_me);
    WS("cntpos", GK, d_cntpos);
    WS("cntneg", GK, d_cntneg);
    const bool ttest = fast && prm->test == SCC_TEST_T;  // DiffTTest (Fast:185-196): no rank stage
    double* d_vx;
    WS("vx", ttest ? GK : 1, d_vx);
    // rank accumulators: S, E, X per (pair, gene), F per (cluster, gene)
    const size_t acc_n = 3 * PG + (size_t)GK;
    WS("acc", acc_n, d_acc);
    // rank work items (LDS capacities depend on the tested-pair list size)
    const bool all_pairs = !fast || prm->test_all;
    const int ntp_max = P;
    // small items: 4 workgroups per CU; medium: 2 per CU (LDS budget per workgroup)
    const int cap_s = scc_rank_item_cap(0, env_int("SCC_CAP_SMALL", kCapSmall), ntp_max, K, 40 * 1024);
    const int cap_m = std::max(cap_s, scc_rank_item_cap(1, env_int("SCC_CAP_MEDIUM", kCapMedium), ntp_max, K, 80 * 1024));
    const int wave_target = 32;  // value buckets of < 64 elements: one wave each
    const int bucket_cap = (int)std::min<int64_t>(3 * nnz1 / wave_target + 2 * (int64_t)G + 64, 1 << 29);
    const int item_cap = bucket_cap;
    const int bucket_target = std::max(64, cap_m / 2);
    WS("items", 3 * (size_t)item_cap, d_items);
    ScRankItem* d_sbk;
    unsigned int* d_hbg;
    int* d_genebk;
    WS("sbuckets", (size_t)bucket_cap, d_sbk);
    WS("hbg", (size_t)bucket_cap * K, d_hbg);
    WS("genebk", 2 * (size_t)G, d_genebk);
    unsigned long long* d_gkmin;
    WS("gkmin", (size_t)G, d_gkmin);
    WS("p", PG, d_p);
    WS("lfc", PG, d_lfc);
    WS("pct1", fast ? PG : 1, d_pct1);
    WS("pct2", fast ? PG : 1, d_pct2);
    WS("u2", PG, d_u2);
    WS("t", PG, d_t);
    WS("flags", PG, d_flags);
    WS("tested", P, d_tested);
    WS("rowoff", P + 1, d_rowoff);
    WS("first", G, d_first);
    WS("union", G, d_union);
    WS("nu", 4, d_nu);
    if ((rc = ensure_wtab(c, exact_test_max_size(nclu)))) return rc;
    hipStream_t s0 = c->s0, s1 = c->s1;
    // the rank stage's work counters on the host (diagnostics; synchronises s0)
    auto read_counts = [&](int* h) -> hipError_t {
        int t[SCC_NCOUNTS * SCC_CNT_STRIDE];
        hipError_t e = hipMemcpyAsync(t, d_counts, sizeof(t), hipMemcpyDeviceToHost, s0);
        if (e == hipSuccess) e = hipStreamSynchronize(s0);
        for (int i = 0; i < SCC_NCOUNTS; ++i) h[i] = t[i * SCC_CNT_STRIDE];
        return e;
    };
    c->generation++;
    const int* d_perm = d_tab;
    const int* d_ccp0 = d_tab + o_ccp0;
    const int* d_cccode = d_tab + o_cccode;
    const int* d_sccc0 = d_tab + o_sccc0;
    const int* d_clcc = d_tab + o_clcc;
    const int* d_nclu = d_tab + o_nclu;

    const int64_t sig[6] = {G, N, K, prm->mode, ds->nnz, (int64_t)(intptr_t)ds};
    double log_thr = 0.0;
    bool hist_rng = false, hist_full = false;
    bool de_cleared = false;  // the per-run clears ran (scc_launch_de_clear at the ingest)
    // after an error-free run whose ingest read every entry: the dataset is
    // validated and its nodg cached (for later gene-shard runs)
    auto note_validated = [&](int err_bits) -> int {
        if (!hist_full || ds->validated || ds->dense) return SCC_OK;
        ds->no_zeros = !(err_bits & 0x1000);  // the full read saw no explicit zero
        if (!ds->d_nodg && hipMalloc((void**)&ds->d_nodg, sizeof(int) * N) != hipSuccess) {
            hipGetLastError();
            ds->d_nodg = nullptr;
            return SCC_OK;  // no cache: later shards keep reading everything
        }
        HIPCHK(c, hipMemcpyAsync(ds->d_nodg, d_nodg, sizeof(int) * N, hipMemcpyDeviceToDevice, s0));
        HIPCHK(c, hipStreamSynchronize(s0));
        ds->validated = true;
        return SCC_OK;
    };
    if (finish_stage) {
        if (!std::equal(sig, sig + 6, c->shard_sig))
            return fail(c, SCC_ERR_INVALID, "scc_de_finish: this context ran no scc_de_run_shard for these inputs");
        log_thr = c->shard_log_thr;
    } else {
    // the tables through a pinned buffer (an asynchronous DMA; every earlier
    // DE call ended with a synchronisation, so no copy out of it is pending)
    const int* tab_src = H.data();
    if (c->h_tab_n < H.size()) {
        if (c->h_tab) hipHostFree(c->h_tab);
        c->h_tab = nullptr;
        c->h_tab_n = 0;
        if (hipHostMalloc((void**)&c->h_tab, sizeof(int) * H.size(), hipHostMallocDefault) == hipSuccess)
            c->h_tab_n = H.size();
        else
            hipGetLastError();
    }
    if (c->h_tab) {
        std::memcpy(c->h_tab, H.data(), sizeof(int) * H.size());
        tab_src = c->h_tab;
    }
    HIPCHK(c, hipMemcpyAsync(d_tab, tab_src, sizeof(int) * H.size(), hipMemcpyHostToDevice, s0));
    const char* ife = getenv("SCC_INGEST_FULL");
    hist_rng = !ds->dense && ds->validated && ds->d_nodg && fast && (glo > 0 || ghi < G) && !(ife && atoi(ife));
    // a validated dataset without explicit zeros, FAST, all genes: the counting
    // pass reads the row indices only (the scatter reads the CSC in full)
    const bool hist_ro = !hist_rng && !ds->dense && ds->validated && ds->no_zeros && ds->d_nodg && fast &&
                         !(ife && atoi(ife));
    hist_full = !hist_rng && !hist_ro;
    {
        Scope sc(c, "ingest", s0);
        // error words, counters, rank accumulators and first-occurrence keys in one launch
        HIPCHK(c, scc_launch_de_clear(d_err, d_counts, ttest ? nullptr : d_acc, (long long)acc_n, d_first, (int)G, glo,
                                      ghi, s0));
        de_cleared = true;
        if ((hist_rng || hist_ro) && !ds->d_tbnd) {  // once per dataset: every cell's gene-tile starts
            // (8 B per (cell, tile): ~0.6 GB at config E, held until the dataset
            // is destroyed, outside the workspace; taken only while it leaves
            // three quarters of the free memory to the runs' workspaces, else
            // the counting pass keeps its per-run binary searches: INTEGRATION.md)
            const size_t tb_bytes = sizeof(long long) * (size_t)N * (ntile + 1);
            size_t mfree = 0, mtot = 0;
            const bool room = hipMemGetInfo(&mfree, &mtot) == hipSuccess && tb_bytes <= mfree / 4;
            (void)hipGetLastError();
            if (!room || hipMalloc((void**)&ds->d_tbnd, tb_bytes) != hipSuccess) {
                (void)hipGetLastError();
                ds->d_tbnd = nullptr;
            } else {
                HIPCHK(c, scc_launch_tile_bounds(ds->d_indptr, ds->d_rows, N, gt, ntile, ds->d_tbnd, s0));
            }
        }
        // (the tile-start cache: the scatter reads it instead of the run's bnd)
        const long long* tbnd = (hist_rng || hist_ro) ? ds->d_tbnd : nullptr;
        if ((hist_ro || (hist_rng && ds->no_zeros)) && tbnd && env_int("SCC_COUNT_RO", 1) != 0)
            HIPCHK(c, scc_launch_ingest_count_ro(ds->d_indptr, ds->d_rows, G, d_perm, d_ccp0, d_cccode, nc,
                                                 hist_rng ? glo : 0, hist_rng ? ghi : G, tbnd, d_cnt, s0));
        else
            HIPCHK(c, scc_launch_ingest_hist(ds->d_indptr, ds->d_rows, ds->d_vals, ds->d_dense, G, d_perm, d_ccp0,
                                             d_cccode, nc, ntile, d_cnt, d_bnd, d_nodg, d_wexp, fast ? 0 : 1, glo, ghi,
                                             hist_rng ? 1 : (hist_ro ? 2 : 0), tbnd, d_err, s0));
        if (hist_rng || hist_ro)
            HIPCHK(c, hipMemcpyAsync(d_nodg, ds->d_nodg, sizeof(int) * N, hipMemcpyDeviceToDevice, s0));
        uint32_t* d_cscr;
        WS("colscan", scc_ingest_colscan_scratch(nc, G), d_cscr);
        // range mode: count rows and their column scan over the shard's gene
        // tiles only; the totals row is zero elsewhere (gstart: empty genes)
        int cg0 = 0, cg1 = G;
        if (hist_rng) {
            scc_ingest_count_range(G, glo, ghi, &cg0, &cg1);
            HIPCHK(c, hipMemsetAsync(d_cnt + (size_t)nc * G, 0, sizeof(uint32_t) * G, s0));
        }
        HIPCHK(c, scc_launch_ingest_colscan(d_cnt, nc, nc_kept, G, cg0, cg1, d_cscr, s0));
        const uint32_t* d_total = d_cnt + (size_t)nc * G;
        HIPCHK(c, scc_launch_scan(d_total, G, d_gstart, d_scan, d_gstart + G, s0));
        HIPCHK(c, scc_launch_ingest_scatter(ds->d_indptr, ds->d_rows, ds->d_vals, ds->d_dense, G, d_perm, d_ccp0,
                                            d_sccc0, ns, d_cnt, d_gstart, d_bnd, tbnd, ntile, glo, ghi, d_keys, s0));
        if (!fast) HIPCHK(c, scc_launch_reduce_dd(d_wexp, nwaves, d_gexp, s0));
    }
    {
        Scope sc(c, "gene_stats", s0);
        ScStatsLaunch S{};
        S.gstart = d_gstart;
        S.keys = d_keys;
        S.G = G;
        S.K = K;
        S.n_clu = d_nclu;
        S.coff = d_cnt;
        S.cl_cc = d_clcc;
        S.mean_x = d_mx;
        S.mean_e = d_me;
        S.cnt_pos = d_cntpos;
        S.cnt_neg = d_cntneg;
        S.mode = prm->mode;
        S.test = ttest ? SCC_TEST_T : SCC_TEST_WILCOX;
        S.var_x = d_vx;
        S.glo = glo;
        S.gn = ghi - glo;
        HIPCHK(c, scc_launch_gene_stats(&S, s0));
    }
    // SLOW: log(meanScalingFactor * mean(expm1(X))) (slow:36) gates the pair
    // filter; a scalar read back here.
    if (!fast) {
        double gx[2];
        HIPCHK(c, hipMemcpyAsync(gx, d_gexp, sizeof(double) * 2, hipMemcpyDeviceToHost, s0));
        HIPCHK(c, hipStreamSynchronize(s0));
        // R: LDOUBLE two-pass mean over G*N entries (zeros included) -> double
        const double tot = (double)G * (double)N;
        double q = gx[0] / tot;
        double r = std::fma(-q, tot, gx[0]) + gx[1];
        const double mean = q + r / tot;
        log_thr = std::log(prm->mean_scaling_factor * mean);
    }
    unsigned long long* accS = d_acc;
    unsigned long long* accE = d_acc + PG;
    unsigned long long* accX = d_acc + 2 * PG;
    unsigned long long* accF = d_acc + 3 * PG;
    ScTestLaunch T{};
    T.K = K;
    T.G = G;
    T.glo = glo;
    T.ghi = ghi;
    T.P = P;
    T.mode = prm->mode;
    T.min_pct = prm->min_per_cent;
    T.lfc_thr = prm->log_fc_thrs;
    T.log_thr = log_thr;
    T.n_clu = d_nclu;
    T.mean_x = d_mx;
    T.mean_e = d_me;
    T.cnt_pos = d_cntpos;
    T.cnt_neg = d_cntneg;
    T.accS = accS;
    T.accE = accE;
    T.accX = accX;
    T.accF = accF;
    T.all_pairs = all_pairs ? 1 : 0;
    T.test = ttest ? SCC_TEST_T : SCC_TEST_WILCOX;
    T.var_x = d_vx;
    T.err = d_err;
    T.wtab = c->d_wtab;
    T.woff = c->d_woff;
    T.out_p = d_p;
    T.out_lfc = d_lfc;
    T.out_pct1 = d_pct1;
    T.out_pct2 = d_pct2;
    T.out_u2 = d_u2;
    T.out_t = d_t;
    T.out_flags = d_flags;
    {
        Scope sc(c, "pair_filter", s0);
        HIPCHK(c, scc_launch_pair_filter(&T, s0));
    }
    if (!ttest) {
        Scope sc(c, "gene_rank", s0);
        if (!de_cleared) HIPCHK(c, hipMemsetAsync(d_acc, 0, sizeof(unsigned long long) * acc_n, s0));
        ScRankLaunch L{};
        L.gstart = d_gstart;
        L.keys = d_keys;
        L.G = G;
        L.K = K;
        L.P = P;
        L.all_pairs = all_pairs ? 1 : 0;
        L.coff = d_cnt;
        L.cl_cc = d_clcc;
        L.flags = d_flags;
        L.cap_s = cap_s;
        L.cap_m = cap_m;
        L.bucket_target = bucket_target;
        L.wave_target = wave_target;
        L.rw_slots = P <= 128 ? 2 : P <= 256 ? 4 : P <= 512 ? 8 : 16;
        L.dbg = env_int("SCC_RW_DEBUG", 0);
        L.rw_mfma = env_int("SCC_RANK_MFMA", 1);
        L.rw_mfma16 = env_int("SCC_RANK_MFMA16", -1);
        L.cross_wave = env_int("SCC_CROSS_WAVE", 0);
        L.bucket_cap = bucket_cap;
        L.sbuckets = d_sbk;
        L.hbg = d_hbg;
        L.gene_bk = d_genebk;
        L.gkmin = d_gkmin;
        L.ntp_max = ntp_max;
        L.item_cap = item_cap;
        L.items = d_items;
        L.counts = d_counts;
        L.split_genes = d_splitg;
        L.keys2 = d_keys2;
        L.codes2 = d_codes2;
        L.gix = d_gix;
        L.gwin = d_gwin;
        L.gcode = d_gcode;
        L.gsc = d_gsc;
        L.nnz = nnz1;
        L.accS = accS;
        L.accE = accE;
        L.accX = accX;
        L.accF = accF;
        WS("gene_tp", (size_t)G * P, L.gene_tp);
        WS("gene_nt", (size_t)G, L.gene_nt);
        if (scc_rank_tables_global(ntp_max, K)) {  // items' tested-pair tables in HBM, one slice per workgroup
            L.tp_global = 1;
            L.tp_scr_stride = scc_rank_tables_stride(ntp_max, K);
            const int ncu_items = c->n_cu > 0 ? c->n_cu : 256;
            WS("tp_scr", (size_t)4 * ncu_items * L.tp_scr_stride, L.tp_scr);
        }
        if (env_int("SCC_RESPLIT", 1)) {
            L.fat_cap = (int)std::min<int64_t>(nnz1 / 64 + 64, 1 << 28);
            WS("fatbk", (size_t)L.fat_cap, L.fatbk);
            WS("rsseg", (size_t)L.fat_cap, L.rsseg);
            WS("fatg", (size_t)G, L.fatg);
            L.fat2_cap = L.fat_cap;
            WS("fat2", (size_t)L.fat2_cap, L.fat2);
        }
        unsigned long long* st_buf = nullptr;
        const bool stamps = env_int("SCC_STAMPS", 0) != 0;
        if (stamps) {
            WS("d_rstamps", (size_t)3 * item_cap * 8, st_buf);
            HIPCHK(c, hipMemsetAsync(st_buf, 0, sizeof(unsigned long long) * 3 * item_cap * 8, s0));
            L.stamps = st_buf;
            L.stamp_base[0] = 0;
            L.stamp_base[1] = item_cap;
            L.stamp_base[2] = 2 * item_cap;
        }
        HIPCHK(c, scc_launch_rank_classify(&L, s0));
        const int ncu = c->n_cu > 0 ? c->n_cu : 256;
        HIPCHK(c, scc_launch_rank_split(&L, 2 * ncu, s0));
        if (L.dbg >= 9) {  // per-gene split clocks (diagnostic; 10: without the unstaged stores)
            int hc[SCC_NCOUNTS];
            HIPCHK(c, read_counts(hc));
            scc_rank_split_diag(s0, hc[3] + hc[13]);  // (small split genes + large ones)
        }
        if (stamps) {  // re-split phase clocks (summed over parents): 8 u64 after the item stamps
            ScRankLaunch R = L;
            R.stamps = st_buf + (size_t)3 * item_cap * 8 - 8;
            HIPCHK(c, hipMemsetAsync(R.stamps, 0, 64, s0));
            HIPCHK(c, scc_launch_rank_resplit(&R, 4 * ncu, s0));
            unsigned long long h[8];
            HIPCHK(c, hipMemcpyAsync(h, R.stamps, 64, hipMemcpyDeviceToHost, s0));
            HIPCHK(c, hipStreamSynchronize(s0));
            fprintf(stderr, "[scc stamps] resplit parents %llu, mean cycles: load %.0f bins %.0f scatter %.0f list %.0f cross %.0f\n",
                    h[7], h[0] / (double)std::max(1ull, h[7]), h[1] / (double)std::max(1ull, h[7]),
                    h[2] / (double)std::max(1ull, h[7]), h[3] / (double)std::max(1ull, h[7]),
                    h[4] / (double)std::max(1ull, h[7]));
            HIPCHK(c, hipMemsetAsync(R.stamps, 0, 64, s0));
        } else {
            // (not on small jobs: at config B the fork and join cost more than
            // the overlap of two ~10-us launches)
            // (SCC_RW_STREAMS=2 forces them at any size: the streams test)
            const int rw_mode = env_int("SCC_RW_STREAMS", 1);
            const int rs_side = (rw_mode >= 2 || (rw_mode != 0 && ds->nnz > (64ll << 20))) ? 2 : 0;
            HIPCHK(c, scc_launch_rank_resplit(&L, 4 * ncu, s0, c->sw, rs_side, c->ev_wfork, c->ev_wj));
        }
        // buckets of <= 64 elements (one wave each) beside the fat buckets (LDS
        // items; SCC_ITEMS_SERIAL=1 runs them after the waves on one stream)
        const bool items_serial = env_int("SCC_ITEMS_SERIAL", 0) != 0;
        hipStream_t si = items_serial ? s0 : s1;
        if (!items_serial) {
            HIPCHK(c, hipEventRecord(c->ev_fork, s0));
            HIPCHK(c, hipStreamWaitEvent(s1, c->ev_fork, 0));
        }
        if (L.dbg == 7) scc_rank_mfma_stamps(s0, 0);
        // the slot classes on s0 and two side streams (SCC_RW_STREAMS=0: all on s0)
        // (forked only when a second class launch exists: config B has one)
        // (sides: one side stream and the items' stream s1 -- a second side
        // stream shared the first one's hardware queue, GPU_MAX_HW_QUEUES = 4)
        const int rw_side = (env_int("SCC_RW_STREAMS", 1) != 0 && L.dbg != 7) ? 2 : 0;
        const hipStream_t wsides[2] = {c->sw[0], si};
        HIPCHK(c, scc_launch_rank_waves(&L, 8 * ncu, s0, si != s0 ? wsides : c->sw, rw_side, c->ev_wfork, c->ev_wj));
        if (L.dbg == 7) scc_rank_mfma_stamps(s0, 1);
        HIPCHK(c, scc_launch_rank_items(&L, 1, 2 * ncu, si));
        HIPCHK(c, scc_launch_rank_items(&L, 0, 4 * ncu, si));
        HIPCHK(c, scc_launch_rank_items(&L, 2, ncu, si));
        if (!items_serial) {
            HIPCHK(c, hipEventRecord(c->ev_join, s1));
            HIPCHK(c, hipStreamWaitEvent(s0, c->ev_join, 0));
        }
        HIPCHK(c, scc_launch_rank_cross(&L, 4 * ncu, s0));
        HIPCHK(c, scc_launch_rank_cross_seg(&L, 4 * ncu, s0));
        if (env_int("SCC_RANK_LOG", 0)) {  // diagnostic: the rank stage's work lists
            int h[SCC_NCOUNTS];
            HIPCHK(c, read_counts(h));
            fprintf(stderr, "[scc rank] items %d/%d/%d split genes %d wave buckets %d bucket ids %d parents %d "
                    "segments %d second-level %d\n", h[0], h[1], h[2], h[3] + h[13], h[4], h[5], h[8], h[10], h[12]);
        }
        if (stamps) {
            std::vector<unsigned long long> h((size_t)3 * item_cap * 8);
            int cnts[SCC_NCOUNTS];
            HIPCHK(c, hipMemcpyAsync(h.data(), st_buf, h.size() * 8, hipMemcpyDeviceToHost, s0));
            HIPCHK(c, read_counts(cnts));
            const char* ph[] = {"setup", "sort", "fixup+codes", "partition", "pairs", "ties"};
            fprintf(stderr, "[scc stamps] split genes %d\n", cnts[3]);
            for (int cls = 0; cls < 3; ++cls) {
                double acc[6] = {0, 0, 0, 0, 0, 0};
                int nb = 0;
                for (int b = 0; b < cnts[cls]; ++b) {
                    const unsigned long long* t = &h[((size_t)cls * item_cap + b) * 8];
                    if (!t[0] || !t[6]) continue;
                    for (int q = 0; q < 6; ++q) acc[q] += (double)(t[q + 1] - t[q]);
                    ++nb;
                }
                fprintf(stderr, "[scc stamps] rank class %d: %d items (%d full), mean cycles:", cls, cnts[cls], nb);
                for (int q = 0; q < 6; ++q) fprintf(stderr, " %s %.0f", ph[q], nb ? acc[q] / nb : 0.0);
                fprintf(stderr, "\n");
            }
        }
    }
    {
        Scope sc(c, "pair_test", s0);
        HIPCHK(c, scc_launch_pair_test(&T, s0));
    }
    }  // compute stages
    // the (pair, gene) fields a shard carries, in scc_de_shard_bytes order
    struct Field {
        void* p;
        size_t es;
    };
    const Field fields[7] = {{d_p, 8}, {d_lfc, 8}, {fast ? (void*)d_pct1 : nullptr, 8}, {fast ? (void*)d_pct2 : nullptr, 8},
                             {d_u2, 8}, {d_t, 8}, {d_flags, 1}};
    if (shard_stage) {
        if (stage == DE_SHARD) {
            char* dst = (char*)shard;
            HIPCHK(c, hipMemsetAsync(dst, 0, scc_de_shard_bytes(K, G), s0));
            for (const Field& f : fields) {
                if (f.p && ghi > glo)
                    HIPCHK(c, hipMemcpy2DAsync(dst + glo * f.es, G * f.es, (const char*)f.p + glo * f.es, G * f.es,
                                               (size_t)(ghi - glo) * f.es, P, hipMemcpyDeviceToDevice, s0));
                dst += PG * f.es;
            }
        } else {  // compact records of the tested cells of this shard, (pair, gene) order
            const long long cells = (long long)P * (ghi - glo);
            const int nb = std::max(1, scc_rec_blocks(cells));
            uint32_t* d_rc;
            long long *d_roff, *d_rscr;
            WS("rec_cnt", nb, d_rc);
            WS("rec_off", nb + 1, d_roff);
            WS("rec_scr", scc_scan_scratch_blocks(nb) + 1, d_rscr);
            const int all = fast ? 0 : 1;
            HIPCHK(c, hipMemsetAsync(d_rc, 0, sizeof(uint32_t) * nb, s0));
            HIPCHK(c, scc_launch_rec_count(d_flags, G, P, glo, ghi, all, d_rc, s0));
            HIPCHK(c, scc_launch_scan(d_rc, nb, d_roff, d_rscr, d_roff + nb, s0));
            long long nrec = 0;
            HIPCHK(c, hipMemcpyAsync(&nrec, d_roff + nb, sizeof(long long), hipMemcpyDeviceToHost, s0));
            HIPCHK(c, hipStreamSynchronize(s0));
            *rio->n_out = nrec;
            if (nrec > rio->cap)
                return fail(c, SCC_ERR_INVALID, "scc_de_run_shard_records: record buffer too small (cap < n_records)");
            HIPCHK(c, scc_launch_rec_pack(d_flags, G, P, glo, ghi, all, d_roff, d_p, d_lfc, fast ? d_pct1 : nullptr,
                                          fast ? d_pct2 : nullptr, d_u2, d_t, (scc_de_record*)rio->out, s0));
        }
        std::copy(sig, sig + 6, c->shard_sig);
        c->shard_log_thr = log_thr;
        HIPCHK(c, hipStreamSynchronize(s0));
        int e = 0;
        HIPCHK(c, hipMemcpy(&e, d_err, sizeof(int), hipMemcpyDeviceToHost));
        if (e & 1) return fail(c, SCC_ERR_NONFINITE, "input holds non-finite values");
        if (e & 2) return fail(c, SCC_ERR_INVALID, "row index out of range");
        if (e & 4) return fail(c, SCC_ERR_INVALID, "row indices not strictly increasing within a column (dgCMatrix)");
        if (e & 8) return fail(c, SCC_ERR_RSTOP, "t.test: data are essentially constant (R stop())");
        return note_validated(e);
    }
    if (stage == DE_FINISH) {
        const char* src = (const char*)shard;
        for (const Field& f : fields) {
            if (f.p) HIPCHK(c, hipMemcpyAsync(f.p, src, PG * f.es, hipMemcpyDeviceToDevice, s0));
            src += PG * f.es;
        }
    } else if (stage == DE_FINISH_REC) {
        // pair-split selection (first_out): only this rank's pair rows are
        // read, so only they are cleared and scattered.  FAST reads a cell's
        // statistics only where its flag is set (k_pair_select), so of the
        // range only the flags are cleared; SLOW clears every field of the
        // range.  Outside the range the flags keep older contents: they only
        // size the other pairs' row offsets (at most one row per cell, so the
        // range's rows stay inside the row buffers) and no row there is read.
        const bool pb = rio->first_out != nullptr;
        const int plo = pb ? rio->pair_lo : 0, phi = pb ? rio->pair_hi : P;
        for (const Field& f : fields) {
            if (!f.p) continue;
            if (!pb)
                HIPCHK(c, hipMemsetAsync(f.p, 0, PG * f.es, s0));
            else if (phi > plo && (f.p == (void*)d_flags || !fast))
                HIPCHK(c, hipMemsetAsync((char*)f.p + (size_t)plo * G * f.es, 0, (size_t)(phi - plo) * G * f.es, s0));
        }
        HIPCHK(c, hipMemsetAsync(d_err, 0, sizeof(int) * 4, s0));
        const scc_de_record* rec = (const scc_de_record*)rio->in;
        for (int b = 0; b < rio->nblocks; ++b)
            HIPCHK(c, scc_launch_rec_scatter(rec + (size_t)b * rio->stride, rio->counts[b], G, P, d_p, d_lfc,
                                             fast ? d_pct1 : nullptr, fast ? d_pct2 : nullptr, d_u2, d_t, d_flags,
                                             d_err, plo, phi, s0));
    }
    // rows (FAST) / per-pair vectors (SLOW)
    int* d_row_gene = nullptr;
    double *d_row_p = nullptr, *d_row_q = nullptr, *d_row_lfc = nullptr, *d_row_pct1 = nullptr, *d_row_pct2 = nullptr;
    long long *d_row_u2 = nullptr, *d_row_t = nullptr;
    uint8_t* d_row_flags = nullptr;
    double* d_slow_q = nullptr;
    uint8_t* d_slow_de = nullptr;
    void *d_rec = nullptr, *d_key = nullptr;
    // FAST rows: one per (pair, gene) flag at most, so PG rows hold every row
    // offset count_tested can produce from any flag contents -- including the
    // stale flags a pair-range finish leaves outside its range
    const size_t rowcap = fast ? PG : 1;
    if (fast && rowcap < PG) return fail(c, SCC_ERR_INVALID, "internal: FAST row buffers smaller than P x G");
    WS("row_gene", rowcap, d_row_gene);
    WS("row_p", rowcap, d_row_p);
    WS("row_q", rowcap, d_row_q);
    WS("row_lfc", rowcap, d_row_lfc);
    WS("row_pct1", rowcap, d_row_pct1);
    WS("row_pct2", rowcap, d_row_pct2);
    WS("row_u2", rowcap, d_row_u2);
    WS("row_t", rowcap, d_row_t);
    WS("row_flags", rowcap, d_row_flags);
    WS("slow_q", fast ? 1 : PG, d_slow_q);
    WS("slow_de", fast ? 1 : PG, d_slow_de);
    if ((rc = ws_get(c, "rec_scratch", PG * scc_select_rec_bytes(), &d_rec))) return rc;
    if ((rc = ws_get(c, "key_scratch", std::max<size_t>(PG, G) * scc_select_key_bytes(), &d_key))) return rc;
    {
        Scope sc(c, "pair_select", s0);
        if (!de_cleared) HIPCHK(c, hipMemsetAsync(d_first, 0xFF, sizeof(unsigned long long) * G, s0));
        if (fast) HIPCHK(c, scc_launch_count_tested(d_flags, G, P, d_tested, d_rowoff, s0));
        ScSelectLaunch S{};
        S.K = K;
        S.G = G;
        S.P = P;
        S.mode = prm->mode;
        S.top_n = fast ? prm->top_n : 30;
        S.cap = env_int("SCC_SELECT_CAP", kSelectCap);
        S.q_thr = prm->q_val_thrs;
        S.lfc_cut = fast ? 0.0 : std::log(prm->fc_thrs);
        S.p = d_p;
        S.lfc = d_lfc;
        S.pct1 = d_pct1;
        S.pct2 = d_pct2;
        S.u2 = d_u2;
        S.t = d_t;
        S.flags = d_flags;
        S.row_off = d_rowoff;
        S.rec_scratch = d_rec;
        S.key_scratch = d_key;
        S.row_gene = d_row_gene;
        S.row_p = d_row_p;
        S.row_q = d_row_q;
        S.row_lfc = d_row_lfc;
        S.row_pct1 = d_row_pct1;
        S.row_pct2 = d_row_pct2;
        S.row_u2 = d_row_u2;
        S.row_t = d_row_t;
        S.row_flags = d_row_flags;
        S.slow_q = d_slow_q;
        S.slow_de = d_slow_de;
        S.first_occ = d_first;
        S.err = d_err;
        const bool pairs_only = rio && rio->first_out;
        S.plo = pairs_only ? rio->pair_lo : 0;
        S.phi = pairs_only ? rio->pair_hi : P;
        HIPCHK(c, scc_launch_pair_select(&S, s0));
        if (pairs_only) {
            HIPCHK(c, hipMemcpyAsync(rio->first_out, d_first, sizeof(unsigned long long) * G, hipMemcpyDeviceToDevice,
                                     s0));
            int e = 0;
            HIPCHK(c, hipMemcpyAsync(&e, d_err, sizeof(int), hipMemcpyDeviceToHost, s0));
            HIPCHK(c, hipStreamSynchronize(s0));
            if (e & 16) return fail(c, SCC_ERR_INVALID, "scc_de_finish_records_pairs: record out of range");
            if (e & 0x200) return fail(c, SCC_ERR_RSTOP, "NA in the DE logical vector: R stops at if(sum(...) <= 1)");
            return SCC_OK;
        }
        HIPCHK(c, scc_launch_union(d_first, G, d_key, env_int("SCC_UNION_CAP", kUnionCap), d_union, d_nu, s0));
    }
    // one pinned staging buffer, one synchronisation: [0] |U|, [1] error bits,
    // [2..3] FAST row count (i64), [4, 4 + P) tested rows per pair, then the
    // union (up to G entries)
    const size_t stage_n = 4 + (size_t)P + (size_t)G;
    if (c->h_stage_n < stage_n) {
        if (c->h_stage) hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_n = 0;
        if (hipHostMalloc((void**)&c->h_stage, sizeof(int) * stage_n, hipHostMallocMapped) != hipSuccess) {
            hipGetLastError();
            c->h_stage = nullptr;
            return fail(c, SCC_ERR_OOM, "pinned staging allocation failed");
        }
        c->h_stage_n = stage_n;
    }
    int* hs = c->h_stage;
    int* hs_dev = nullptr;  // the same pinned buffer as the device sees it
    HIPCHK(c, hipHostGetDevicePointer((void**)&hs_dev, hs, 0));
    HIPCHK(c, scc_launch_stage_pack(d_nu, d_err, fast ? d_rowoff + P : nullptr, fast ? d_tested : nullptr, P, d_union,
                                    G, hs_dev, s0));
    HIPCHK(c, hipStreamSynchronize(s0));
    if ((rc = check_pending_eig(c))) return rc;  // an earlier device-output scc_distance
    const int hdr[2] = {hs[0], hs[1]};
    if (hdr[1] & 1) return fail(c, SCC_ERR_NONFINITE, "input holds non-finite values");
    if (hdr[1] & 2) return fail(c, SCC_ERR_INVALID, "row index out of range");
    if (hdr[1] & 4) return fail(c, SCC_ERR_INVALID, "row indices not strictly increasing within a column (dgCMatrix)");
    if (hdr[1] & 8) return fail(c, SCC_ERR_RSTOP, "t.test: data are essentially constant (R stop())");
    if (hdr[1] & 16) return fail(c, SCC_ERR_INVALID, "scc_de_finish_records: record out of range");
    if ((rc = note_validated(hdr[1]))) return rc;
    scc_de_result* r = new scc_de_result();
    r->ctx = c;
    r->generation = c->generation;
    r->mode = prm->mode;
    r->K = K;
    r->P = P;
    r->G = G;
    r->N = N;
    r->d_union = d_union;
    r->log_thr = log_thr;
    if (hdr[0] < 0 || hdr[0] > G) return fail(c, SCC_ERR_HIP, "union size out of range");
    r->union_genes.assign(hs + 4 + P, hs + 4 + P + hdr[0]);
    if (fast) {
        long long nrows = 0;
        std::memcpy(&nrows, &hs[2], sizeof(long long));
        r->pair_tested.assign(hs + 4, hs + 4 + P);
        r->n_rows = nrows;
    }
    r->d_nodg = d_nodg;
    r->d_row_gene = d_row_gene;
    r->d_row_p = d_row_p;
    r->d_row_q = d_row_q;
    r->d_row_lfc = d_row_lfc;
    r->d_row_pct1 = d_row_pct1;
    r->d_row_pct2 = d_row_pct2;
    r->d_row_u2 = d_row_u2;
    r->d_row_t = d_row_t;
    r->d_row_flags = d_row_flags;
    r->d_p = d_p;
    r->d_q = d_slow_q;
    r->d_lfc = d_lfc;
    r->d_u2 = d_u2;
    r->d_de = d_slow_de;
    *out = r;
    // selection-stage conditions (k_pair_select), reported after the result is
    // built: SLOW NA in the DE logical vector (slow:165-186: R stops at
    // if(sum(...) <= 1)); bit 0x100 (FAST NA q in a kept pair: R builds NA rows
    // and does not stop) is informational only
    if (hdr[1] & 0x200) return fail(c, SCC_ERR_RSTOP, "NA in the DE logical vector: R stops at if(sum(...) <= 1)");
    return SCC_OK;
#undef WS
}

// ---------------------------------------------------------------- device list
// ONE DE job over the context's devices (scc_opts.n_devices > 1; SURVEY 8e:
// gene row-blocks, then a gather of compact per-(pair, tested gene) records):
// each device runs the per-(pair, gene) stage of its gene block and packs its
// tested cells (scc_de_record, 64 B) -- one host thread per device --, the
// records are copied to devices[0] (xGMI peer copies) and the per-pair BH,
// filters, top-N and union run there: the scc_de_finish_records result, equal
// to the one-device run bit for bit.  Blocks are balanced by the genes'
// stored values (a CSC row histogram, computed once per dataset).
static int gene_blocks(scc_ctx* c, const scc_dataset* ds, int D, std::vector<int64_t>& cut)
{
    const int64_t G = ds->G;
    cut.assign(D + 1, 0);
    cut[D] = G;
    if (!ds->dense && ds->gene_w.empty() && ds->nnz > 0) {
        unsigned int* d_h = nullptr;
        int rc = ws(c, "row_hist", (size_t)G, &d_h);
        if (rc) return rc;
        HIPCHK(c, scc_launch_row_hist(ds->d_rows, ds->nnz, (int)G, d_h, c->s0));
        std::vector<unsigned int> h(G);
        HIPCHK(c, hipMemcpyAsync(h.data(), d_h, sizeof(unsigned int) * G, hipMemcpyDeviceToHost, c->s0));
        HIPCHK(c, hipStreamSynchronize(c->s0));
        ds->gene_w.assign(h.begin(), h.end());
    }
    std::vector<double> cw(G + 1, 0.0);
    for (int64_t g = 0; g < G; ++g) cw[g + 1] = cw[g] + (ds->gene_w.empty() ? 1.0 : 1.0 + (double)ds->gene_w[g]);
    for (int d = 1; d < D; ++d) {
        const double share = cw[G] * d / D;
        int64_t g = std::lower_bound(cw.begin(), cw.end(), share) - cw.begin();
        // non-empty blocks while genes last
        g = std::max<int64_t>(g, std::min<int64_t>(G, cut[d - 1] + 1));
        cut[d] = std::min<int64_t>(g, G);
    }
    return SCC_OK;
}

static int de_run_multi(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K, const scc_de_params* prm,
                        scc_de_result** out)
{
    *out = nullptr;
    if (ds->reps.size() != c->peers.size()) return fail(c, SCC_ERR_INVALID, "dataset has no replica on every device");
    const int D = 1 + (int)c->peers.size();
    std::vector<scc_ctx*> eng{c};
    std::vector<const scc_dataset*> dsr{ds};
    for (size_t i = 0; i < c->peers.size(); ++i) {
        eng.push_back(c->peers[i]);
        dsr.push_back(ds->reps[i]);
    }
    scc_enter(c);
    std::vector<int64_t> cut;
    int rc = gene_blocks(c, ds, D, cut);
    if (rc) return rc;
    const int64_t P = (int64_t)K * (K - 1) / 2;
    std::vector<int> rcs(D, SCC_OK);
    std::vector<int64_t> nrec(D, 0);
    std::vector<void*> rbuf(D, nullptr);
    {
        std::vector<std::thread> th;
        for (int d = 0; d < D; ++d)
            th.emplace_back([&, d] {
                scc_ctx* x = eng[d];
                hipSetDevice(x->device);
                const int64_t cap = std::max<int64_t>(1, P * (cut[d + 1] - cut[d]));
                if ((rcs[d] = ws_get(x, "mrec", (size_t)cap * sizeof(scc_de_record), &rbuf[d]))) return;
                RecIO io;
                io.out = rbuf[d];
                io.cap = cap;
                io.n_out = &nrec[d];
                rcs[d] = de_run_impl(x, dsr[d], code, K, prm, DE_SHARD_REC, cut[d], cut[d + 1], nullptr, nullptr, &io);
            });
        for (auto& t : th) t.join();
    }
    scc_enter(c);
    for (int d = 0; d < D; ++d)
        if (rcs[d]) return d ? fail(c, rcs[d], eng[d]->err) : rcs[d];
    const int64_t stride = std::max<int64_t>(1, *std::max_element(nrec.begin(), nrec.end()));
    void* all = nullptr;
    if ((rc = ws_get(c, "mrec_all", (size_t)D * stride * sizeof(scc_de_record), &all))) return rc;
    for (int d = 0; d < D; ++d) {
        if (!nrec[d]) continue;
        char* dst = (char*)all + (size_t)d * stride * sizeof(scc_de_record);
        const size_t bytes = (size_t)nrec[d] * sizeof(scc_de_record);
        if (eng[d]->device == c->device)
            HIPCHK(c, hipMemcpyAsync(dst, rbuf[d], bytes, hipMemcpyDeviceToDevice, c->s0));
        else
            HIPCHK(c, hipMemcpyPeerAsync(dst, c->device, rbuf[d], eng[d]->device, bytes, c->s0));
    }
    RecIO io;
    io.in = all;
    io.counts = nrec.data();
    io.nblocks = D;
    io.stride = stride;
    return de_run_impl(c, ds, code, K, prm, DE_FINISH_REC, 0, ds->G, nullptr, out, &io);
}

// one engine run of <= 128 clusters: on the context's device, or sharded over its device list
static int de_run_one(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K, const scc_de_params* prm,
                      scc_de_result** out)
{
    if (!c->peers.empty() && K <= kMaxK) return de_run_multi(c, ds, code, K, prm, out);
    return de_run_impl(c, ds, code, K, prm, DE_FULL, 0, ds->G, nullptr, out);
}

// ---------------------------------------------------------------- any K
// More clusters than one engine run ranks (7-bit codes, 128): the K clusters
// are cut into ng = ceil(K / gmax) groups of balanced size (gmax = 64, or
// SCC_GROUP_SIZE), and the engine runs once per group pair (u < v) on the cells
// of those <= 128 clusters (the others get code -1).  Every per-pair quantity
// of both DE paths depends on the pair's two clusters alone (FAST: pct,
// log-mean logFC, filters, test, BH over the pair's own rows, top_n,
// Fast:229-392; SLOW: test, mean difference, gate with the GLOBAL threshold of
// every entry -- the same in every run, since the ingest sums expm1 over all
// cells whatever their code --, BH with n = G, first 30, slow:36,90-227), so a
// global pair (i, j) is taken from exactly one run: the run of its two groups,
// or for a pair inside one group the first run holding that group.  A run's
// clusters keep the global order, so Cluster1 / Cluster2 orientation and the
// within-run pair order are the global ones.  Rows (FAST) and per-pair vectors
// are moved into the global (i, j) order on the device (k_seg_copy); the
// union is unique() over the pairs' top lists in (i, j) order, i.e. genes by
// their smallest (pair, rank) key: each run's keys are renumbered to global
// pairs and MIN-folded (k_first_remap), then ordered once (k_union).
static int de_run_grouped(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K, const scc_de_params* prm,
                          int gmax, scc_de_result** out)
{
    *out = nullptr;
    const bool fast = prm->mode == SCC_DE_FAST;
    if (prm->mode != SCC_DE_FAST && prm->mode != SCC_DE_SLOW) return fail(c, SCC_ERR_INVALID, "bad mode");
    const int64_t G = ds->G, N = ds->N;
    const int64_t P = (int64_t)K * (K - 1) / 2;
    if (P >= ((int64_t)1 << 31)) return fail(c, SCC_ERR_UNSUPPORTED, "more than 2^31 cluster pairs");
    {
        std::vector<int64_t> n(K, 0);
        for (int64_t i = 0; i < N; ++i) {
            const int a = code[i];
            if (a < -1 || a >= K) return fail(c, SCC_ERR_INVALID, "code out of range");
            if (a >= 0) n[a]++;
        }
        for (int a = 0; a < K; ++a) {
            if (n[a] == 0) return fail(c, SCC_ERR_INVALID, "empty cluster");
            if (fast && n[a] < 3) return fail(c, SCC_ERR_RSTOP, "cluster has fewer than 3 cells (R stop())");
        }
    }
    scc_enter(c);
    hipStream_t s0 = c->s0;
    const int ng = (K + gmax - 1) / gmax;
    std::vector<int> gid(K);
    std::vector<std::vector<int>> grp(ng);
    for (int u = 0; u < ng; ++u)
        for (int a = (int)((int64_t)u * K / ng); a < (int)((int64_t)(u + 1) * K / ng); ++a) {
            grp[u].push_back(a);
            gid[a] = u;
        }
    const bool vectors = !fast || prm->test_all;  // the dense [P][G] per-pair vectors
    const size_t PG = (size_t)P * (size_t)G;
    int rc;
    double *g_p = nullptr, *g_lfc = nullptr, *g_q = nullptr;
    long long* g_u2 = nullptr;
    uint8_t* g_de = nullptr;
    unsigned long long* g_first = nullptr;
#define WSG(name, n, ptr)                                       \
    do {                                                        \
        if ((rc = ws(c, name, (size_t)(n), &(ptr)))) return rc; \
    } while (0)
    WSG("grp_first", G, g_first);
    if (vectors) {
        WSG("grp_p", PG, g_p);
        WSG("grp_lfc", PG, g_lfc);
        WSG("grp_u2", PG, g_u2);
        if (!fast) {
            WSG("grp_q", PG, g_q);
            WSG("grp_de", PG, g_de);
        }
    }
    HIPCHK(c, hipMemsetAsync(g_first, 0xFF, sizeof(unsigned long long) * G, s0));
    // FAST rows: staged in run order (grow-preserving buffers), then gathered
    // into the global pair order at the end
    struct RowField {
        const char* stage;
        const char* fin;
        int es;
    };
    static const RowField rf[9] = {{"grp_s_gene", "grp_row_gene", 4}, {"grp_s_p", "grp_row_p", 8},
                                   {"grp_s_q", "grp_row_q", 8},       {"grp_s_lfc", "grp_row_lfc", 8},
                                   {"grp_s_pct1", "grp_row_pct1", 8}, {"grp_s_pct2", "grp_row_pct2", 8},
                                   {"grp_s_u2", "grp_row_u2", 8},     {"grp_s_t", "grp_row_t", 8},
                                   {"grp_s_flags", "grp_row_flags", 1}};
    int64_t staged = 0;
    std::vector<int64_t> st_off(fast ? P : 0, 0), st_cnt(fast ? P : 0, 0);
    std::vector<char> covered(ng, 0);
    std::vector<int32_t> sub(N);
    std::vector<long long> lp2gp, seg;
    bool rstop = false;
    std::string rstop_msg;
    double log_thr = 0.0;
    for (int u = 0; u < ng; ++u)
        for (int v = u + 1; v < ng; ++v) {
            std::vector<int> cl(grp[u]);
            cl.insert(cl.end(), grp[v].begin(), grp[v].end());
            const int Kl = (int)cl.size();
            std::vector<int> lut(K, -1);
            for (int l = 0; l < Kl; ++l) lut[cl[l]] = l;
            for (int64_t i = 0; i < N; ++i) sub[i] = code[i] >= 0 ? lut[code[i]] : -1;
            scc_de_result* r = nullptr;
            rc = de_run_one(c, ds, sub.data(), Kl, prm, &r);
            if (rc) {
                if (rc != SCC_ERR_RSTOP || !r) {
                    scc_de_result_destroy(r);
                    return rc;
                }
                rstop = true;
                rstop_msg = c->err;
            }
            log_thr = r->log_thr;
            const int Pl = Kl * (Kl - 1) / 2;
            lp2gp.assign(Pl, 0);
            std::vector<char> take(Pl, 0);
            {
                int lp = 0;
                for (int li = 0; li < Kl; ++li)
                    for (int lj = li + 1; lj < Kl; ++lj, ++lp) {
                        const int64_t gi = cl[li], gj = cl[lj];
                        lp2gp[lp] = gi * K - gi * (gi + 1) / 2 + (gj - gi - 1);
                        take[lp] = gid[gi] != gid[gj] || !covered[gid[gi]];
                    }
            }
            covered[u] = covered[v] = 1;
            long long *d_lp2gp = nullptr, *d_seg = nullptr;
            unsigned long long* d_first = nullptr;
            WSG("grp_lp2gp", Pl, d_lp2gp);
            WSG("first", G, d_first);  // the run's per-gene first-occurrence keys
            HIPCHK(c, hipMemcpyAsync(d_lp2gp, lp2gp.data(), sizeof(long long) * Pl, hipMemcpyHostToDevice, s0));
            HIPCHK(c, scc_launch_first_remap(d_first, (int)G, d_lp2gp, g_first, s0));
            if (vectors) {  // per-pair [G] vectors: one segment per taken pair
                seg.clear();
                for (int lp = 0; lp < Pl; ++lp)
                    if (take[lp]) {
                        seg.push_back((long long)lp * G);
                        seg.push_back(lp2gp[lp] * G);
                        seg.push_back(G);
                    }
                const long long ns = (long long)seg.size() / 3;
                WSG("grp_seg", seg.size(), d_seg);
                HIPCHK(c, hipMemcpyAsync(d_seg, seg.data(), sizeof(long long) * seg.size(), hipMemcpyHostToDevice, s0));
                HIPCHK(c, scc_launch_seg_copy(r->d_p, g_p, 8, d_seg, ns, s0));
                HIPCHK(c, scc_launch_seg_copy(r->d_lfc, g_lfc, 8, d_seg, ns, s0));
                HIPCHK(c, scc_launch_seg_copy(r->d_u2, g_u2, 8, d_seg, ns, s0));
                if (!fast) {
                    HIPCHK(c, scc_launch_seg_copy(r->d_q, g_q, 8, d_seg, ns, s0));
                    HIPCHK(c, scc_launch_seg_copy(r->d_de, g_de, 1, d_seg, ns, s0));
                }
                HIPCHK(c, hipStreamSynchronize(s0));  // d_seg is rewritten by the next segment table
            }
            if (fast) {  // the taken pairs' rows, appended to the staging buffers
                seg.clear();
                int64_t lo = 0, add = 0;
                for (int lp = 0; lp < Pl; ++lp) {
                    const int64_t n = r->pair_tested[lp];
                    if (take[lp] && n > 0) {
                        seg.push_back(lo);
                        seg.push_back(staged + add);
                        seg.push_back(n);
                    }
                    if (take[lp]) {
                        st_off[lp2gp[lp]] = staged + add;
                        st_cnt[lp2gp[lp]] = n;
                        add += n;
                    }
                    lo += n;
                }
                const long long ns = (long long)seg.size() / 3;
                if (ns > 0) {
                    WSG("grp_seg", seg.size(), d_seg);
                    HIPCHK(c, hipMemcpyAsync(d_seg, seg.data(), sizeof(long long) * seg.size(), hipMemcpyHostToDevice,
                                             s0));
                    const void* src[9] = {r->d_row_gene, r->d_row_p,  r->d_row_q,  r->d_row_lfc, r->d_row_pct1,
                                          r->d_row_pct2, r->d_row_u2, r->d_row_t, r->d_row_flags};
                    for (int f = 0; f < 9; ++f) {
                        void* dst = nullptr;
                        if ((rc = ws_keep(c, rf[f].stage, (size_t)(staged + add) * rf[f].es, (size_t)staged * rf[f].es,
                                          &dst)))
                            return rc;
                        HIPCHK(c, scc_launch_seg_copy(src[f], dst, rf[f].es, d_seg, ns, s0));
                    }
                    HIPCHK(c, hipStreamSynchronize(s0));
                }
                staged += add;
            }
            scc_de_result_destroy(r);
        }
    scc_de_result* r = new scc_de_result();
    r->ctx = c;
    r->mode = prm->mode;
    r->K = K;
    r->P = (int)P;
    r->G = G;
    r->N = N;
    r->log_thr = log_thr;
    std::unique_ptr<scc_de_result> hold(r);
    if (fast) {  // staged rows -> the global (i, j) order
        r->pair_tested.resize(P);
        seg.clear();
        int64_t row = 0;
        for (int64_t p = 0; p < P; ++p) {
            r->pair_tested[p] = (int32_t)st_cnt[p];
            if (st_cnt[p] > 0) {
                seg.push_back(st_off[p]);
                seg.push_back(row);
                seg.push_back(st_cnt[p]);
            }
            row += st_cnt[p];
        }
        r->n_rows = row;
        const long long ns = (long long)seg.size() / 3;
        long long* d_seg = nullptr;
        WSG("grp_seg", std::max<size_t>(seg.size(), 3), d_seg);
        if (ns > 0)
            HIPCHK(c, hipMemcpyAsync(d_seg, seg.data(), sizeof(long long) * seg.size(), hipMemcpyHostToDevice, s0));
        void* fin[9];
        for (int f = 0; f < 9; ++f) {
            if ((rc = ws_get(c, rf[f].fin, (size_t)std::max<int64_t>(row, 1) * rf[f].es, &fin[f]))) return rc;
            void* stg = nullptr;
            if ((rc = ws_keep(c, rf[f].stage, (size_t)std::max<int64_t>(staged, 1) * rf[f].es, (size_t)staged * rf[f].es,
                              &stg)))
                return rc;
            HIPCHK(c, scc_launch_seg_copy(stg, fin[f], rf[f].es, d_seg, ns, s0));
        }
        r->d_row_gene = (const int*)fin[0];
        r->d_row_p = (const double*)fin[1];
        r->d_row_q = (const double*)fin[2];
        r->d_row_lfc = (const double*)fin[3];
        r->d_row_pct1 = (const double*)fin[4];
        r->d_row_pct2 = (const double*)fin[5];
        r->d_row_u2 = (const long long*)fin[6];
        r->d_row_t = (const long long*)fin[7];
        r->d_row_flags = (const uint8_t*)fin[8];
    }
    r->d_p = g_p;
    r->d_lfc = g_lfc;
    r->d_u2 = g_u2;
    r->d_q = g_q;
    r->d_de = g_de;
    r->vectors = vectors;
    {  // the union: genes ordered by their smallest global (pair, rank) key
        void* d_key = nullptr;
        int *d_union = nullptr, *d_nu = nullptr, *d_nodg = nullptr;
        if ((rc = ws_get(c, "key_scratch", (size_t)G * scc_select_key_bytes(), &d_key))) return rc;
        WSG("union", G, d_union);
        WSG("nu", 4, d_nu);
        WSG("nodg", N, d_nodg);  // every run wrote the same nodg (clustering-independent)
        HIPCHK(c, scc_launch_union(g_first, (int)G, d_key, env_int("SCC_UNION_CAP", kUnionCap), d_union, d_nu, s0));
        int nu = 0;
        HIPCHK(c, hipMemcpyAsync(&nu, d_nu, sizeof(int), hipMemcpyDeviceToHost, s0));
        HIPCHK(c, hipStreamSynchronize(s0));
        if (nu < 0 || nu > G) return fail(c, SCC_ERR_HIP, "union size out of range");
        r->union_genes.resize(nu);
        if (nu) HIPCHK(c, hipMemcpy(r->union_genes.data(), d_union, sizeof(int) * nu, hipMemcpyDeviceToHost));
        r->d_nodg = d_nodg;
    }
    r->generation = c->generation;
    *out = hold.release();
    if (rstop) return fail(c, SCC_ERR_RSTOP, rstop_msg);
    return SCC_OK;
#undef WSG
}

extern "C" int scc_de_run(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K,
                          const scc_de_params* prm, scc_de_result** out)
{
    if (!c || !ds || !code || !prm || !out) return fail(c, SCC_ERR_INVALID, "scc_de_run: null argument");
    *out = nullptr;
    if (ds->ctx != c) return fail(c, SCC_ERR_INVALID, "dataset belongs to another context");
    // SCC_GROUP_SIZE (test knob): group-pair runs of groups <= this size as
    // soon as K exceeds two groups (default 64: K > 128)
    const int gmax = std::min(std::max(env_int("SCC_GROUP_SIZE", kGroupMax), 1), kGroupMax);
    if (K > 2 * gmax) return de_run_grouped(c, ds, code, K, prm, gmax, out);
    return de_run_one(c, ds, code, K, prm, out);
}

extern "C" int64_t scc_de_shard_bytes(int32_t K, int64_t n_genes)
{
    const int64_t PG = (int64_t)K * (K - 1) / 2 * n_genes;
    return (PG * 49 + 7) / 8 * 8;  // p, lfc, pct1, pct2 (f64), u2, ties (i64), flags (u8); 8-byte multiple
}

extern "C" int scc_de_run_shard(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K,
                                const scc_de_params* prm, int64_t gene_lo, int64_t gene_hi, void* shard)
{
    return de_run_impl(c, ds, code, K, prm, DE_SHARD, gene_lo, gene_hi, shard, nullptr);
}

extern "C" int scc_de_finish(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K,
                             const scc_de_params* prm, const void* shards_sum, scc_de_result** out)
{
    return de_run_impl(c, ds, code, K, prm, DE_FINISH, 0, ds ? ds->G : 0, const_cast<void*>(shards_sum), out);
}

extern "C" int scc_de_run_shard_records(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K,
                                        const scc_de_params* prm, int64_t gene_lo, int64_t gene_hi, void* records,
                                        int64_t cap, int64_t* n_records)
{
    if (!records || !n_records || cap < 0) return fail(c, SCC_ERR_INVALID, "scc_de_run_shard_records: null argument");
    RecIO io;
    io.out = records;
    io.cap = cap;
    io.n_out = n_records;
    *n_records = 0;
    return de_run_impl(c, ds, code, K, prm, DE_SHARD_REC, gene_lo, gene_hi, nullptr, nullptr, &io);
}

extern "C" int scc_de_finish_records(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K,
                                     const scc_de_params* prm, const void* records, const int64_t* counts,
                                     int32_t n_blocks, int64_t stride, scc_de_result** out)
{
    if (!counts || n_blocks < 1 || stride < 0 || (!records && stride > 0))
        return fail(c, SCC_ERR_INVALID, "scc_de_finish_records: bad record blocks");
    for (int b = 0; b < n_blocks; ++b)
        if (counts[b] < 0 || counts[b] > stride) return fail(c, SCC_ERR_INVALID, "scc_de_finish_records: count > stride");
    RecIO io;
    io.in = records;
    io.counts = counts;
    io.nblocks = n_blocks;
    io.stride = stride;
    return de_run_impl(c, ds, code, K, prm, DE_FINISH_REC, 0, ds ? ds->G : 0, nullptr, out, &io);
}

extern "C" int scc_de_finish_records_pairs(scc_ctx* c, const scc_dataset* ds, const int32_t* code, int32_t K,
                                           const scc_de_params* prm, const void* records, const int64_t* counts,
                                           int32_t n_blocks, int64_t stride, int32_t pair_lo, int32_t pair_hi,
                                           void* first_occ)
{
    if (!counts || n_blocks < 1 || stride < 0 || (!records && stride > 0) || !first_occ)
        return fail(c, SCC_ERR_INVALID, "scc_de_finish_records_pairs: bad arguments");
    const int P = K * (K - 1) / 2;
    if (pair_lo < 0 || pair_hi > P || pair_lo > pair_hi)
        return fail(c, SCC_ERR_INVALID, "scc_de_finish_records_pairs: pair range out of bounds");
    if (!prm || prm->mode != SCC_DE_FAST)
        return fail(c, SCC_ERR_UNSUPPORTED, "scc_de_finish_records_pairs: FAST mode only");
    for (int b = 0; b < n_blocks; ++b)
        if (counts[b] < 0 || counts[b] > stride)
            return fail(c, SCC_ERR_INVALID, "scc_de_finish_records_pairs: count > stride");
    RecIO io;
    io.in = records;
    io.counts = counts;
    io.nblocks = n_blocks;
    io.stride = stride;
    io.pair_lo = pair_lo;
    io.pair_hi = pair_hi;
    io.first_out = first_occ;
    return de_run_impl(c, ds, code, K, prm, DE_FINISH_REC, 0, ds ? ds->G : 0, nullptr, nullptr, &io);
}

extern "C" int scc_de_union_first_occ(scc_ctx* c, const void* first_occ, int64_t G64, int32_t* genes,
                                      int32_t* n_union)
{
    if (!c || !first_occ || !genes || !n_union || G64 < 1 || G64 > INT32_MAX)
        return fail(c, SCC_ERR_INVALID, "scc_de_union_first_occ: bad arguments");
    const int G = (int)G64;
    scc_enter(c);
    hipStream_t s0 = c->s0;
    int rc;
    void* d_key = nullptr;
    int *d_union = nullptr, *d_nu = nullptr;
    if ((rc = ws_get(c, "key_scratch", (size_t)G * scc_select_key_bytes(), &d_key))) return rc;
    if ((rc = ws(c, "union", G, &d_union))) return rc;
    if ((rc = ws(c, "nu", 4, &d_nu))) return rc;
    HIPCHK(c, scc_launch_union((const unsigned long long*)first_occ, G, d_key, env_int("SCC_UNION_CAP", kUnionCap),
                               d_union, d_nu, s0));
    int nu = 0;
    HIPCHK(c, hipMemcpyAsync(&nu, d_nu, sizeof(int), hipMemcpyDeviceToHost, s0));
    HIPCHK(c, hipStreamSynchronize(s0));
    if (nu < 0 || nu > G) return fail(c, SCC_ERR_HIP, "scc_de_union_first_occ: bad union size");
    if (nu) HIPCHK(c, hipMemcpy(genes, d_union, sizeof(int) * nu, hipMemcpyDeviceToHost));
    *n_union = nu;
    return SCC_OK;
}

static int check_live(const scc_de_result* r)
{
    if (!r) return SCC_ERR_INVALID;
    if (r->generation != r->ctx->generation)
        return fail(r->ctx, SCC_ERR_INVALID, "result is stale: copy it out before the next scc_de_run");
    hipSetDevice(r->ctx->device);
    return SCC_OK;
}

extern "C" int scc_de_result_counts(const scc_de_result* r, int32_t* n_pairs, int64_t* n_rows, int32_t* n_union)
{
    if (!r) return SCC_ERR_INVALID;
    if (n_pairs) *n_pairs = r->P;
    if (n_rows) *n_rows = r->n_rows;
    if (n_union) *n_union = (int32_t)r->union_genes.size();
    return SCC_OK;
}

extern "C" int scc_de_result_union(const scc_de_result* r, int32_t* genes)
{
    if (!r || !genes) return SCC_ERR_INVALID;
    std::copy(r->union_genes.begin(), r->union_genes.end(), genes);
    return SCC_OK;
}

template <class T>
static int d2h(scc_ctx* c, T* dst, const T* src, size_t n)
{
    if (!dst || n == 0) return SCC_OK;
    HIPCHK(c, hipMemcpy(dst, src, sizeof(T) * n, hipMemcpyDeviceToHost));
    return SCC_OK;
}

extern "C" int scc_de_result_rows(const scc_de_result* r, int32_t* pair_rows, int32_t* gene, double* p, double* q,
                                  double* lfc, double* pct1, double* pct2, int64_t* u2, int64_t* ties,
                                  uint8_t* flags)
{
    int rc = check_live(r);
    if (rc) return rc;
    if (r->mode != SCC_DE_FAST) return fail(r->ctx, SCC_ERR_INVALID, "rows exist for SCC_DE_FAST only");
    scc_ctx* c = r->ctx;
    const size_t n = (size_t)r->n_rows;
    if (pair_rows) std::copy(r->pair_tested.begin(), r->pair_tested.end(), pair_rows);
    if ((rc = d2h(c, gene, r->d_row_gene, n))) return rc;
    if ((rc = d2h(c, p, r->d_row_p, n))) return rc;
    if ((rc = d2h(c, q, r->d_row_q, n))) return rc;
    if ((rc = d2h(c, lfc, r->d_row_lfc, n))) return rc;
    if ((rc = d2h(c, pct1, r->d_row_pct1, n))) return rc;
    if ((rc = d2h(c, pct2, r->d_row_pct2, n))) return rc;
    if ((rc = d2h(c, (long long*)u2, r->d_row_u2, n))) return rc;
    if ((rc = d2h(c, (long long*)ties, r->d_row_t, n))) return rc;
    if ((rc = d2h(c, flags, r->d_row_flags, n))) return rc;
    return SCC_OK;
}

extern "C" int scc_de_result_pair_vectors(const scc_de_result* r, double* p, double* q, double* lfc, int64_t* u2,
                                          uint8_t* de)
{
    int rc = check_live(r);
    if (rc) return rc;
    scc_ctx* c = r->ctx;
    const size_t n = (size_t)r->P * (size_t)r->G;
    if (!r->vectors && (p || lfc || u2))
        return fail(c, SCC_ERR_INVALID, "per-pair vectors of a FAST group-pair run exist with test_all = 1 only");
    if ((rc = d2h(c, p, r->d_p, n))) return rc;
    if ((rc = d2h(c, lfc, r->d_lfc, n))) return rc;
    if ((rc = d2h(c, (long long*)u2, r->d_u2, n))) return rc;
    if (r->mode == SCC_DE_SLOW) {
        if ((rc = d2h(c, q, r->d_q, n))) return rc;
        if ((rc = d2h(c, de, r->d_de, n))) return rc;
    } else if (q || de) {
        return fail(c, SCC_ERR_INVALID, "q/de vectors exist for SCC_DE_SLOW only");
    }
    return SCC_OK;
}

extern "C" int scc_de_result_log_threshold(const scc_de_result* r, double* log_thr)
{
    if (!r || !log_thr) return SCC_ERR_INVALID;
    *log_thr = r->log_thr;
    return SCC_OK;
}

extern "C" int scc_de_result_nodg(const scc_de_result* r, int32_t* nodg)
{
    int rc = check_live(r);
    if (rc) return rc;
    return d2h(r->ctx, nodg, r->d_nodg, (size_t)r->N);
}

extern "C" void scc_de_result_destroy(scc_de_result* r) { delete r; }

// distance entry points live in scc_distance.cpp
