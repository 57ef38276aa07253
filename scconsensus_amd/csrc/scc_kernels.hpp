// scc_kernels.hpp — internal launcher interface between the runtime
// (scc_runtime.cpp) and the HIP kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#ifndef SCC_DE_FAST  // (same values as include/scc.h)
#define SCC_DE_FAST 0
#define SCC_DE_SLOW 1
#endif
#ifndef SCC_TEST_T
#define SCC_TEST_WILCOX 0
#define SCC_TEST_T 1
#endif

#define SCC_ING_HIST_WAVES 16  // waves per ingest histogram workgroup (one partial expm1 sum each)

struct dd;

// The rank stage's work counters (ScRankLaunch::counts, 16 of them) sit
// SCC_CNT_STRIDE ints apart, one 128-B line each: every split workgroup adds
// to several of them per gene, and on one shared line the atomics (and any
// load of a neighbour) queued behind each other in L2.
#define SCC_NCOUNTS 16
#define SCC_CNT_STRIDE 32

struct ScStatsLaunch {
    const long long* gstart;
    const unsigned long long* keys;
    int G, K;
    const int* n_clu;
    const uint32_t* coff;
    const int* cl_cc;
    double* mean_x;     // [K][G] (slow mode only)
    double* mean_e;     // [K][G] (fast mode only)
    double* var_x;      // [K][G] (fast t test only)
    int mode;           // SCC_DE_FAST: mean of expm1(x); SCC_DE_SLOW: mean of x
    int test;           // SCC_TEST_WILCOX | SCC_TEST_T (FAST)
    uint32_t* cnt_pos;  // [K][G]
    uint32_t* cnt_neg;  // [K][G]
    int glo, gn;        // the genes [glo, glo + gn) (a gene shard; nothing else is read downstream)
};

// one unit of rank work: a whole gene (src 0: the ingest's cluster-grouped
// segment) or one value bucket of a split gene (src 1: keys2 / codes2)
struct ScRankItem {
    long long base;
    int n, gene, src, bucket;  // bucket: global bucket id (its cluster histogram row), -1 none
};

struct ScRankLaunch {
    const long long* gstart;
    const unsigned long long* keys;
    int G, K, P, all_pairs;
    const uint32_t* coff;
    const int* cl_cc;
    const uint8_t* flags;  // [P][G] bit0: the pair tests the gene
    int cap_s, cap_m, cap_lds, bucket_target, ntp_max, item_cap;
    int wave_target;       // split: bins are packed into buckets of < 2 * wave_target elements
    int rw_slots;          // wave kernel: tested pairs per gene held in registers, 64 * rw_slots (2, 4, 8 or 16)
    int dbg;               // SCC_RW_DEBUG timing experiments (1: no pair counts, 2: no sort); results invalid
    int bucket_cap;        // capacity of sbuckets / hbg rows
    ScRankItem* sbuckets;  // [bucket_cap] buckets of <= 64 elements (one wave each)
    unsigned int* hbg;     // [bucket_cap][K] per-bucket cluster counts
    int* gene_bk;          // [2 G] first bucket id and bucket count of each split gene
    unsigned long long* gkmin;  // [G] key minimum of a split gene when its range fits 58 bits, else ~0
    ScRankItem* items;     // [3][item_cap]
    int* counts;           // [0..2] items per class, [3] split genes, [4] wave buckets, [5] bucket ids,
                           // [8] fat buckets, [9] re-split queue, [10] re-split segments, [11] re-split genes,
                           // [12] second-level re-split parents
    uint32_t* gene_tp;     // [G][P] tested pairs of each split gene, p | a << 16 | b << 24 (pair order)
    int* gene_nt;          // [G] their number
    int wv_lo, wv_hi;      // wave kernel launch: genes with wv_lo < tested pairs <= wv_hi
    int wv_base;           // ... and their tested pairs [wv_base, wv_base + 64 * slots)
    int wv_filter;         // 0: one launch holds every gene (no per-bucket class test)
    int rw_mfma;           // K <= 64: the wave buckets' pair counts on the int8 matrix cores (k_rank_mfma16)
    int rw_mfma16;         // the 16 x 16 x 64 form for the genes the slot kernels take (k_rank_mfma16): -1 at K <= 16, 1 at K <= 32, 0 off
    ScRankItem* fatbk;     // [fat_cap] buckets of > 64 distinct values (re-split into sub-buckets)
    int4* fatg;            // [G] {gene, first fatbk entry, parents}: the re-split work units
    int4* rsseg;           // [fat_cap] {gene, first sub-bucket id, sub-buckets}: in-parent cross terms
    int fat_cap;
    int rsw_chunk;         // wave re-split: bucket ids / list slots taken per global atomic
    ScRankItem* fat2;      // [fat2_cap] second re-split level (counts[12])
    int fat2_cap;
    int rs_level;          // wave re-split launch: 0 reads fatbk, 1 reads fat2
    int rsw_all;           // wave re-split: one launch takes every gene (no split by tested pairs)
    int cross_wave;        // 1: gene-level cross terms by the per-(gene, pair) wave kernel
    int* split_genes;      // [G]
    unsigned long long* keys2;  // [nnz] bucket-ordered keys of split genes
    uint8_t* codes2;            // [nnz]
    uint32_t* gix;              // [2][nnz] index ping-pong of HBM-resident items
    uint32_t* gwin;             // [nnz] key windows of HBM-resident items
    uint8_t* gcode;             // [nnz]
    uint8_t* gsc;               // [nnz]
    long long nnz;
    unsigned long long* accS;   // [P][G] #{x > y}, nonzeros
    unsigned long long* accE;   // [P][G] cross-cluster equal pairs
    unsigned long long* accX;   // [P][G] sum c_a c_b (c_a + c_b) over tie groups
    unsigned long long* accF;   // [K][G] sum c^3 - c over within-cluster runs
    unsigned long long* stamps; // diagnostic phase clocks [item][8] (nullptr normally)
    int stamp_base[3];
    int tp_global;              // items' tested-pair tables in HBM (scc_rank_tables_global)
    char* tp_scr;               // [item workgroups][tp_scr_stride] when tp_global
    size_t tp_scr_stride;
};


struct ScTestLaunch {
    int K, G, P, mode;
    int glo, ghi;          // genes [glo, ghi): a run's gene shard (all genes: 0, G)
    double min_pct, lfc_thr, log_thr;
    const int* n_clu;
    const double* mean_x;
    const double* mean_e;
    const uint32_t* cnt_pos;
    const uint32_t* cnt_neg;
    const unsigned long long* accS;
    const unsigned long long* accE;
    const unsigned long long* accX;
    const unsigned long long* accF;
    int all_pairs;
    int test;              // SCC_TEST_WILCOX | SCC_TEST_T
    const double* var_x;   // [K][G] (t test)
    int* err;              // bit 8: t.test would stop ("data are essentially constant")
    const double* wtab;
    const int* woff;
    double* out_p;
    double* out_lfc;
    double* out_pct1;
    double* out_pct2;
    long long* out_u2;
    long long* out_t;
    uint8_t* out_flags;
};

struct ScSelectLaunch {
    int K, G, P, mode, top_n, cap;
    int plo, phi;          // pairs [plo, phi) (all: 0, P)
    double q_thr, lfc_cut;
    const double* p;
    const double* lfc;
    const double* pct1;
    const double* pct2;
    const long long* u2;
    const long long* t;
    const uint8_t* flags;
    const long long* row_off;
    void* rec_scratch;
    void* key_scratch;
    int* row_gene;
    double* row_p;
    double* row_q;
    double* row_lfc;
    double* row_pct1;
    double* row_pct2;
    long long* row_u2;
    long long* row_t;
    uint8_t* row_flags;
    double* slow_q;
    uint8_t* slow_de;
    unsigned long long* first_occ;
    int* err;
};

extern "C" {
int scc_ingest_gene_tile(void);
hipError_t scc_launch_de_clear(int* err, int* counts, unsigned long long* acc, long long acc_n,
                               unsigned long long* first, int G, int glo, int ghi, hipStream_t st);
int scc_ingest_hist_window(int G);
hipError_t scc_launch_ingest_hist(const long long* indptr, const int* rows, const double* vals, const double* dense,
                                  int G, const int* perm, const int* cc_p0, const int* cc_code, int nc, int ntile,
                                  uint32_t* cnt, long long* bnd, int* nodg, dd* wave_expm1, int want_expm1, int glo,
                                  int ghi, int rng, const long long* tbnd, int* err, hipStream_t st);
hipError_t scc_launch_tile_bounds(const long long* indptr, const int* rows, int N, int gt, int ntile, long long* tbnd,
                                  hipStream_t st);
int scc_ingest_colscan_scratch(int nc, int G);
hipError_t scc_launch_ingest_colscan(uint32_t* cnt, int nc, int nc_kept, int G, int g0, int g1, uint32_t* scratch,
                                     hipStream_t st);
void scc_ingest_count_range(int G, int glo, int ghi, int* g0, int* g1);
hipError_t scc_launch_ingest_scatter(const long long* indptr, const int* rows, const double* vals,
                                     const double* dense, int G, const int* perm, const int* cc_p0, const int* sc_cc0,
                                     int ns, const uint32_t* cnt, const long long* gstart, const long long* bnd,
                                     const long long* tbnd, int ntile, int glo, int ghi, unsigned long long* keys,
                                     hipStream_t st);
// the counting pass of a validated zero-free dataset over all genes (FAST; the
// tile starts come from the dataset's cache, nodg from its cache)
// (a gene shard [glo, ghi) of a validated dataset too: its tiles' entries from tbnd)
hipError_t scc_launch_ingest_count_ro(const long long* indptr, const int* rows, int G, const int* perm,
                                      const int* cc_p0, const int* cc_code, int nc, int glo, int ghi,
                                      const long long* tbnd, uint32_t* cnt, hipStream_t st);
hipError_t scc_launch_scan(const uint32_t* in, long long n, long long* out, long long* bsum_scratch,
                           long long* total, hipStream_t st);
int scc_scan_scratch_blocks(long long n);
// CSR -> CSC transpose (scc_csr.hip): a plan sized on the host from (G, N,
// nnz), one scratch blob, a validating pass, then the two-pass transpose
struct ScCsrPlan {
    long long G, N, nnz;
    int SB, NS;      // cells per superblock, superblocks
    int T;           // gene tiles of 256
    int CG, NG;      // cells per output group, groups
    size_t off_bnd, off_rs, off_tt, off_ts, off_off, off_gm, off_gb, off_scan, off_meta, off_ival, bytes;
};
int scc_csr_plan(long long G, long long N, long long nnz, ScCsrPlan* P);
// validation (columns in [0, N), strictly ascending per gene) + superblock bounds
hipError_t scc_launch_csr_check(const ScCsrPlan* P, const long long* indptr, const int* cols, void* scratch,
                                int* err, hipStream_t st);
hipError_t scc_launch_csr_to_csc(const ScCsrPlan* P, const long long* indptr, const int* cols, const double* vals,
                                 void* scratch, long long* csc_indptr, int* csc_rows, double* csc_vals,
                                 hipStream_t st);
hipError_t scc_launch_reduce_dd(const dd* parts, int n, dd* out, hipStream_t st);

hipError_t scc_launch_gene_stats(const ScStatsLaunch* L, hipStream_t st);
hipError_t scc_launch_rank_classify(const ScRankLaunch* L, hipStream_t st);
size_t scc_rank_item_lds(int cls, int cap, int ntp_max, int K);
int scc_rank_item_cap(int cls, int want, int ntp_max, int K, int lim);
size_t scc_rank_split_lds(int K);
int scc_rank_tables_global(int ntp_max, int K);
size_t scc_rank_tables_stride(int ntp_max, int K);
hipError_t scc_launch_rank_split(const ScRankLaunch* L, int grid, hipStream_t st);
hipError_t scc_launch_rank_items(const ScRankLaunch* L, int cls, int grid, hipStream_t st);
// the slot classes' launches go round st, side[0], side[1], ... (nside 0: all
// on st); a side stream is forked from st (event fork) when it first gets a
// launch and joined back (its event in join[]) at the end
hipError_t scc_launch_rank_waves(const ScRankLaunch* L, int grid, hipStream_t st, const hipStream_t* side = nullptr,
                                 int nside = 0, hipEvent_t fork = nullptr, const hipEvent_t* join = nullptr);
void scc_rank_mfma_stamps(hipStream_t st, int print);
hipError_t scc_launch_rank_cross(const ScRankLaunch* L, int grid_genes, hipStream_t st);
hipError_t scc_launch_rank_resplit(const ScRankLaunch* L, int grid, hipStream_t st, const hipStream_t* side = nullptr,
                                   int nside = 0, hipEvent_t fork = nullptr, const hipEvent_t* join = nullptr);
hipError_t scc_launch_rank_cross_seg(const ScRankLaunch* L, int grid, hipStream_t st);
hipError_t scc_launch_pair_filter(const ScTestLaunch* L, hipStream_t st);
size_t scc_eigen_scratch_doubles(int n, int lda, int k);
hipError_t scc_launch_eigen_topk(const double* A, int n, int lda, int k, double* scratch, double* Z, double* W,
                                 unsigned int** err_dev, int* nwg_out, hipEvent_t* marks,
                                 unsigned long long* stamps, unsigned long long key, hipStream_t st);

hipError_t scc_launch_wilcox_table(double* W, const int* woff, int mmax, hipStream_t st);
int scc_wilcox_table_layout(int* woff);
hipError_t scc_launch_pair_test(const ScTestLaunch* L, hipStream_t st);
hipError_t scc_launch_count_tested(const uint8_t* flags, int G, int P, int* tested, long long* row_off,
                                   hipStream_t st);
size_t scc_select_lds_bytes(int cap);
size_t scc_select_rec_bytes(void);
size_t scc_select_key_bytes(void);
hipError_t scc_launch_pair_select(const ScSelectLaunch* L, hipStream_t st);
hipError_t scc_launch_union(const unsigned long long* first_occ, int G, void* scratch, int cap, int* out,
                            int* n_out, hipStream_t st);
hipError_t scc_launch_flag_copy(const unsigned int* src, unsigned int* dst_dev, hipStream_t st);
hipError_t scc_launch_stage_pack(const int* nu, const int* err, const long long* nrows, const int* tested, int P,
                                 const int* uni, int G, int* out_dev, hipStream_t st);
hipError_t scc_launch_seg_copy(const void* src, void* dst, int elem_bytes, const long long* seg, long long nseg,
                               hipStream_t st);
hipError_t scc_launch_row_hist(const int* rows, long long nnz, int G, unsigned int* cnt, hipStream_t st);
hipError_t scc_launch_first_remap(const unsigned long long* local, int G, const long long* lp2gp,
                                  unsigned long long* global, hipStream_t st);
}
