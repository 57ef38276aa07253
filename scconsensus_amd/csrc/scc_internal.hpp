// scc_internal.hpp — runtime-internal state shared by the C ABI translation
// units (scc_runtime.cpp: context/dataset/DE; scc_distance.cpp: stage 3).
#pragma once
#include "scc.h"
#include "scc_kernels.hpp"

#ifndef SCC_MAX_K
#define SCC_MAX_K 128  // (same value as scc_common.hpp)
#endif

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace scc_rt {

constexpr int kCapSmall = 2048;    // rank work item in LDS, 256 threads
constexpr int kCapMedium = 16384;  // rank work item in LDS, 1024 threads (capped by the LDS budget);
                                   // larger genes are split into value buckets
constexpr int kCountChunk = 32;    // cells per ingest count chunk (one cluster each)
constexpr int kScatterCC = 8;      // count chunks per ingest scatter chunk (at most)
constexpr int kSelectCap = 2048;   // per-pair records sorted in LDS
constexpr int kUnionCap = 4096;
constexpr int kMaxK = SCC_MAX_K;  // 7-bit cluster codes in the rank kernels: clusters per engine run
constexpr int kGroupMax = 64;     // K > 2 * kGroupMax: group-pair runs of <= 2 * kGroupMax clusters

struct Timer {
    double ms = 0.0;
    int64_t n = 0;
};

struct PendingEv {
    std::string name;
    hipEvent_t a, b;
};

}  // namespace scc_rt

struct scc_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t s0 = nullptr, s1 = nullptr;
    hipStream_t own_s0 = nullptr;  // the context's own stream (s0 unless scc_ctx_set_stream)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipStream_t sw[2] = {nullptr, nullptr};        // side streams of the wave kernels' slot classes
    hipEvent_t ev_wj[2] = {nullptr, nullptr};      // their joins
    hipEvent_t ev_wfork = nullptr;                 // and fork
    std::string err;
    // workspace slots (grow-only)
    std::map<std::string, std::pair<void*, size_t>> ws;
    // exact-test table
    double* d_wtab = nullptr;
    int* d_woff = nullptr;
    int wtab_m = 0;  // cluster sizes up to wtab_m are in the table (0: none yet)
    // profiling
    bool profile = false;
    std::vector<scc_rt::PendingEv> pending;
    std::vector<hipEvent_t> ev_pool;
    std::map<std::string, scc_rt::Timer> timers;
    uint64_t generation = 0;
    uint64_t serial = 0;  // unique per context in this process (never reused, unlike its address)
    uint64_t ws_gen = 0;  // bumped by every workspace (re)allocation
    std::vector<int> host_tables;  // cell permutation + chunk tables of the last scc_de_run
    int* h_stage = nullptr;        // pinned: the DE result header, tested counts and union, one D2H
    size_t h_stage_n = 0;
    int* h_tab = nullptr;          // pinned: a DE call's host tables (asynchronous H2D)
    size_t h_tab_n = 0;
    int* h_genes = nullptr;        // pinned: a distance call's gene list (asynchronous H2D)
    size_t h_genes_n = 0;
    hipEvent_t ev_genes = nullptr;  // recorded after the last copy out of h_genes
    // last PCA
    const double* d_last_scores = nullptr;  // N x 16 in the workspace
    int last_n = 0;
    int last_ncomp = 0;
    unsigned int eig_err = 0;  // hand-off timeout flag of the last eigensolve (host copy)
    unsigned int* h_flag = nullptr;  // pinned, device-mapped: where a kernel ORs that flag in
    bool eig_flag_pending = false;   // an unsynchronised scc_distance left its flag in h_flag
    const void* d_last_dist = nullptr;  // device copy of the last full scc_distance output
    int64_t last_dist_n = 0;
    int last_dist_f32 = 0;
    int64_t shard_sig[6] = {-1, -1, -1, -1, -1, -1};  // inputs of the last scc_de_run_shard
    double shard_log_thr = 0.0;
    // pinned staging ring of the streamed distance output (scc_distance to a
    // pageable host buffer): 2 slots of dstage_bytes each
    char* h_dstage = nullptr;
    size_t dstage_bytes = 0;
    // sharded PCA (scc_pca_shard_*): this rank's cells and the union width
    int pca_nu = 0, pca_ld = 0;
    int64_t pca_N = 0, pca_clo = 0, pca_chi = 0;
    int pca_stage = 0;  // 1 after colsum, 2 after gram
    // device list (scc_opts.n_devices > 1): the engines of devices[1..], each
    // with its own streams and workspace; this context is devices[0]'s
    std::vector<scc_ctx*> peers;
    // the last full distance kept on this device when its columns were
    // written by several devices: peer slices not yet copied in (entries
    // [off, off + n) of d_last_dist live at ptr on device dev)
    struct Slice {
        int dev;
        const void* ptr;
        size_t off, n;
    };
    std::vector<Slice> last_dist_pending;
};

struct scc_dataset {
    scc_ctx* ctx = nullptr;  // borrowed; the dataset must be destroyed before its context
    int device = 0;
    int64_t G = 0, N = 0, nnz = 0;
    bool dense = false;
    long long* d_indptr = nullptr;
    int* d_rows = nullptr;
    double* d_vals = nullptr;
    double* d_dense = nullptr;
    bool owned = false;
    // set by the first DE run that read every entry without an input error
    // (rows in range and sorted): a gene shard of a later FAST run then reads
    // only its tiles (k_ing_hist rng) and takes nodg (clustering-independent)
    // from this device cache.  The data must not change while the dataset lives.
    mutable bool validated = false;
    mutable bool no_zeros = false;  // the validating read saw no explicit (stored) zero
    mutable int* d_nodg = nullptr;  // [N], always owned
    // [N][ntile + 1] entry offsets where each cell's gene tiles start
    // (clustering-independent), built by the first range-mode run: later
    // gene-shard runs read a cell's shard entries without binary searches
    mutable long long* d_tbnd = nullptr;
    // device list: the replica on each peer engine of the context (same order
    // as scc_ctx::peers), and the stored values per gene that balance the
    // gene row-blocks (computed on the first sharded run)
    std::vector<scc_dataset*> reps;
    mutable std::vector<int64_t> gene_w;
};

struct scc_de_result {
    scc_ctx* ctx = nullptr;
    uint64_t generation = 0;
    int mode = 0, K = 0, P = 0;
    int64_t G = 0, N = 0;
    int64_t n_rows = 0;
    std::vector<int32_t> union_genes;
    std::vector<int32_t> pair_tested;
    double log_thr = 0.0;
    // device views into the context workspace (valid while generation matches)
    const int* d_nodg = nullptr;
    const int* d_union = nullptr;  // the union in device memory (the single-device engine run; else nullptr)
    const int* d_row_gene = nullptr;
    const double *d_row_p = nullptr, *d_row_q = nullptr, *d_row_lfc = nullptr, *d_row_pct1 = nullptr,
                 *d_row_pct2 = nullptr;
    const long long *d_row_u2 = nullptr, *d_row_t = nullptr;
    const uint8_t* d_row_flags = nullptr;
    const double *d_p = nullptr, *d_q = nullptr, *d_lfc = nullptr;
    const long long* d_u2 = nullptr;
    const uint8_t* d_de = nullptr;
    bool vectors = true;  // d_p / d_lfc / d_u2 hold the [P][G] vectors (a FAST group-pair run: test_all only)
};

namespace scc_rt {

inline int fail(scc_ctx* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                              \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess)                                                                          \
            return fail((ctx), SCC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));         \
    } while (0)

extern "C" void scc_fsi_forget(const void* p, size_t bytes);  // scc_subspace.hip: cached graphs over p

// grow-only named workspace buffer
inline int ws_get(scc_ctx* c, const char* name, size_t bytes, void** out)
{
    bytes = std::max<size_t>(bytes, 256);
    auto it = c->ws.find(name);
    if (it != c->ws.end() && it->second.second >= bytes) {
        *out = it->second.first;
        return SCC_OK;
    }
    if (it != c->ws.end()) {
        hipStreamSynchronize(c->s0);
        hipStreamSynchronize(c->s1);
        scc_fsi_forget(it->second.first, it->second.second);
        hipFree(it->second.first);
        c->ws.erase(it);
    }
    void* p = nullptr;
    size_t grow = bytes + bytes / 8;
    if (hipMalloc(&p, grow) != hipSuccess) {
        hipGetLastError();
        return fail(c, SCC_ERR_OOM, std::string("hipMalloc failed for workspace ") + name);
    }
    c->ws[name] = {p, grow};
    c->ws_gen++;
    *out = p;
    return SCC_OK;
}

// grow-only named workspace buffer whose first `used` bytes survive a growth
inline int ws_keep(scc_ctx* c, const char* name, size_t bytes, size_t used, void** out)
{
    auto it = c->ws.find(name);
    if (it != c->ws.end() && it->second.second >= bytes) {
        *out = it->second.first;
        return SCC_OK;
    }
    const size_t grow = std::max<size_t>(256, bytes + bytes / 2);
    void* p = nullptr;
    if (hipMalloc(&p, grow) != hipSuccess) {
        hipGetLastError();
        return fail(c, SCC_ERR_OOM, std::string("hipMalloc failed for workspace ") + name);
    }
    if (it != c->ws.end()) {
        if (used && hipMemcpyAsync(p, it->second.first, used, hipMemcpyDeviceToDevice, c->s0) != hipSuccess) {
            hipGetLastError();
            hipFree(p);
            return fail(c, SCC_ERR_HIP, std::string("workspace growth copy failed for ") + name);
        }
        hipStreamSynchronize(c->s0);
        hipStreamSynchronize(c->s1);
        scc_fsi_forget(it->second.first, it->second.second);
        hipFree(it->second.first);
        c->ws.erase(it);
    }
    c->ws[name] = {p, grow};
    c->ws_gen++;
    *out = p;
    return SCC_OK;
}

// The filtered eigensolver's graph-cache key: this context and the state of
// its workspace (a graph bakes in workspace pointers; any reallocation makes
// every earlier graph of the context unreachable)
inline unsigned long long eig_graph_key(const scc_ctx* c)
{
    return ((unsigned long long)c->serial << 32) ^ (unsigned long long)(c->ws_gen & 0xffffffffu);
}

template <class T>
inline int ws(scc_ctx* c, const char* name, size_t count, T** out)
{
    void* p = nullptr;
    int rc = ws_get(c, name, count * sizeof(T), &p);
    *out = (T*)p;
    return rc;
}

inline hipEvent_t ev_take(scc_ctx* c)
{
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

// Entry of every C-ABI call: the context's device, and the thread's HIP
// "last error" cleared (each of our runtime calls is checked where it is made;
// a residue left by a call outside the engine or a deliberate probe must not
// be reported by the next kernel launch's hipGetLastError()).
void scc_enter(const scc_ctx* c);

// after a synchronisation: the eigensolver flag an earlier device-output
// scc_distance (which returns without synchronising) left in h_flag
int check_pending_eig(scc_ctx* c);

inline int env_int(const char* name, int dflt)
{
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// SCC_DEBUG_SYNC=1: synchronise after every stage and report it on stderr
// (locates a faulting kernel; never set in timed runs).
inline bool debug_sync()
{
    static int v = env_int("SCC_DEBUG_SYNC", 0);
    return v != 0;
}

// Whether a profiled context times the stage `name`: every stage, unless
// SCC_PROFILE_STAGES holds a comma-separated list (read at each stage: a
// caller may switch it between calls).  A timing event between two kernels
// leaves the GPU idle ~12 us, ~0.14 ms per config-B step with every stage
// timed, so a timed benchmark region brackets only the stage it reports.
inline bool stage_timed(const scc_ctx* c, const char* name)
{
    if (!c->profile) return false;
    const char* f = getenv("SCC_PROFILE_STAGES");
    if (!f || !*f) return true;
    const size_t n = strlen(name);
    for (const char* q = f; (q = strstr(q, name)) != nullptr; q += n)
        if ((q == f || q[-1] == ',') && (q[n] == ',' || q[n] == 0)) return true;
    return false;
}

struct Scope {
    scc_ctx* c;
    const char* name;
    hipStream_t st;
    hipEvent_t a = nullptr;
    bool on = false;
    Scope(scc_ctx* c_, const char* n, hipStream_t s) : c(c_), name(n), st(s)
    {
        on = stage_timed(c, name);
        if (on) {
            a = ev_take(c);
            hipEventRecord(a, st);
        }
        if (debug_sync()) fprintf(stderr, "[scc] %s: start\n", name);
    }
    ~Scope()
    {
        if (on) {
            hipEvent_t b = ev_take(c);
            hipEventRecord(b, st);
            c->pending.push_back({name, a, b});
        }
        if (debug_sync()) {
            hipError_t e0 = hipStreamSynchronize(c->s0), e1 = hipStreamSynchronize(c->s1);
            fprintf(stderr, "[scc] %s: done (%s / %s)\n", name, hipGetErrorString(e0), hipGetErrorString(e1));
            fflush(stderr);
        }
    }
};

inline void resolve_timers(scc_ctx* c)
{
    if (c->pending.empty()) return;
    hipStreamSynchronize(c->s0);
    hipStreamSynchronize(c->s1);
    for (auto& pe : c->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
            auto& t = c->timers[pe.name];
            t.ms += ms;
            t.n += 1;
        }
        c->ev_pool.push_back(pe.a);
        c->ev_pool.push_back(pe.b);
    }
    c->pending.clear();
}

// R's exact Wilcoxon distribution (cwilcox counts) for cluster sizes up to
// mmax: built the first time a run has two clusters of fewer than 50 cells
// (the only pairs wilcox.test.default tests exactly), and grown when a later
// run has larger ones.  Runs without such a pair build nothing.
inline int ensure_wtab(scc_ctx* c, int mmax)
{
    mmax = std::min(mmax, 49);
    if (!c->d_woff) {
        std::vector<int> woff(50 * 50);
        const int total = scc_wilcox_table_layout(woff.data());
        int rc = ws(c, "wtab", (size_t)total, &c->d_wtab);
        if (rc) return rc;
        rc = ws(c, "woff", woff.size(), &c->d_woff);
        if (rc) return rc;
        HIPCHK(c, hipMemcpyAsync(c->d_woff, woff.data(), woff.size() * sizeof(int), hipMemcpyHostToDevice, c->s0));
    }
    if (mmax <= c->wtab_m) return SCC_OK;
    HIPCHK(c, scc_launch_wilcox_table(c->d_wtab, c->d_woff, mmax, c->s0));
    c->wtab_m = mmax;
    return SCC_OK;
}

// the largest cluster size a pair of clusters that both hold < 50 cells can
// have (0: no such pair, no exact test in this run)
inline int exact_test_max_size(const std::vector<int>& nclu)
{
    int n_small = 0, m = 0;
    for (int v : nclu)
        if (v < 50) {
            ++n_small;
            m = std::max(m, v);
        }
    return n_small >= 2 ? m : 0;
}

}  // namespace scc_rt
