/*
 * scc.h — C ABI of the MI355X scConsensus engine (libscc.so).
 *
 * Drop-in boundary for the data-parallel core of the reference R package
 * (bbbranjan/scConsensus).  The reference has no native code and no FFI
 * (NAMESPACE:3-6 has no useDynLib); these entry points are what its R
 * functions bind through `.Call` (see INTEGRATION.md for the R glue):
 *
 *   reclusterDEConsensusFast()  R/reclusterDEConsensusFast.R:22-33
 *       pair loop + ComputePairWiseDE + union      :57-392  -> scc_de_run(SCC_DE_FAST)
 *       prcomp_irlba + dist                         :398-400 -> scc_distance(SCC_DIST_PCA_EUCLID)
 *       `1 - cor(...)` (commented alternative)      :403     -> scc_distance(SCC_DIST_PEARSON)
 *       nodg loop                                   :440-443 -> scc_de_result_nodg
 *   reclusterDEConsensus()      R/reclusterDEConsensus.R:20-29
 *       global threshold + pair loop + union        :32-227  -> scc_de_run(SCC_DE_SLOW)
 *       prcomp_irlba + dist                         :234-236 -> scc_distance(SCC_DIST_PCA_EUCLID)
 *
 * Conventions: plain pointers and sizes, no C++ types, int status returns
 * (SCC_OK == 0), no exceptions or longjmp across the ABI.  Inputs are borrowed
 * read-only; the caller owns every output buffer.  Cluster selection (R's
 * table()/grepl("grey")/locale order, Fast:40-53) stays in the caller, which
 * passes integer codes: code[c] in [0, K) in the reference's cluster order,
 * or -1 for cells whose cluster is not compared.  Pairs are (i<j) in the
 * reference's nested-loop order: p = i*K - i*(i+1)/2 + (j-i-1).
 */
#ifndef SCC_H
#define SCC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#define SCC_API __attribute__((visibility("default")))
#else
#define SCC_API
#endif

#define SCC_OK 0
#define SCC_ERR_INVALID 1     /* bad argument / shape */
#define SCC_ERR_HIP 2         /* HIP runtime error (no device, launch failure) */
#define SCC_ERR_OOM 3         /* device allocation failed */
#define SCC_ERR_NONFINITE 4   /* input holds NaN/Inf or out-of-range row index */
#define SCC_ERR_RSTOP 5       /* the reference R code would stop() on this input */
#define SCC_ERR_UNSUPPORTED 6 /* valid input outside this build's limits (e.g. ncomp > 16) */

#define SCC_DE_FAST 0 /* reclusterDEConsensusFast(method = "wilcox") */
#define SCC_DE_SLOW 1 /* reclusterDEConsensus(method = "Wilcoxon") */
#define SCC_TEST_WILCOX 0 /* FAST test.use = "wilcox" (WilcoxDETest, Fast:78-91) */
#define SCC_TEST_T 1      /* FAST test.use = "t" (DiffTTest: Welch t.test, Fast:185-196) */

#define SCC_DIST_PCA_EUCLID 0 /* dist(prcomp_irlba(t(X[U,]), n=min(|U|,15))$x) */
#define SCC_DIST_PEARSON 1    /* as.dist(1 - cor(X[U,], method = "pearson")) */

#define SCC_PTR_HOST 0   /* pointers are host memory (copied H2D by the engine) */
#define SCC_PTR_DEVICE 1 /* pointers are device memory of the context's device */

typedef struct scc_ctx scc_ctx;
typedef struct scc_dataset scc_dataset;
typedef struct scc_de_result scc_de_result;

typedef struct {
    int32_t device;      /* HIP device ordinal (the context's only device when n_devices <= 1) */
    int32_t profile;     /* 1: time the dominant kernels with HIP events */
    int32_t n_devices;   /* > 1: ONE job over the devices devices[0 .. n_devices) (SURVEY 8b's device
                            list; replaces the reference's nCores PSOCK workers, Fast:61-65,384) */
    int32_t reserved[5];
    const int32_t* devices; /* n_devices HIP ordinals, devices[0] the primary (a repeated ordinal runs
                               several engines on one device: the sharded path on one GPU) */
} scc_opts;

typedef struct {
    int32_t mode;               /* SCC_DE_FAST | SCC_DE_SLOW */
    int32_t top_n;              /* FAST: NumbertopDEGenes (Fast:32); SLOW: 30 (slow:218) */
    double q_val_thrs;          /* qValThrs */
    double log_fc_thrs;         /* FAST: logFCThrs, natural log (Fast:26) */
    double min_per_cent;        /* FAST: minPerCent (Fast:29) */
    double fc_thrs;             /* SLOW: fcThrs, compared as log(fcThrs) (slow:167) */
    double mean_scaling_factor; /* SLOW: meanScalingFactor (slow:23) */
    int32_t test_all;           /* FAST: 1 = also compute U / p for the (pair, gene) cells the
                                   feature filters drop (diagnostics; R never tests them) */
    int32_t test;               /* FAST: SCC_TEST_WILCOX (default) | SCC_TEST_T; u2 / ties are 0 for t */
} scc_de_params;

/* ---- context ---------------------------------------------------------- */
/* With a device list (opts.n_devices > 1) the context drives every device of
 * the list from this one host process (one host thread per device inside
 * each call; peer copies over xGMI between them):
 *   scc_dataset_create_*  uploads to devices[0] and replicates the matrix on
 *                         the others (peer copies; a repeated ordinal shares it)
 *   scc_de_run            gene row-blocks balanced by stored values, one per
 *                         device, their tested-cell records gathered on
 *                         devices[0], which runs the per-pair selection: the
 *                         result equals the one-device run bit for bit
 *                         (K > 128: every group-pair run is sharded this way)
 *   scc_distance(_cols)   the PCA on devices[0], its N x 16 scores copied to
 *                         every device, each device the packed columns of an
 *                         equal share of the entries, streamed straight to
 *                         the caller's host buffer or copied into its device
 *                         buffer (bit for bit the one-device output; the
 *                         Pearson metric runs on devices[0] only)
 * Every other entry point works on devices[0].  Results and outputs live on
 * devices[0]. */
SCC_API int scc_ctx_create(const scc_opts* opts, scc_ctx** out);
/* number of visible HIP devices (0 when none) */
SCC_API int scc_device_count(int32_t* n);
SCC_API void scc_ctx_destroy(scc_ctx* ctx);
SCC_API const char* scc_ctx_last_error(const scc_ctx* ctx);
SCC_API int scc_ctx_synchronize(scc_ctx* ctx);
/* Launch the engine's work on the caller's stream (a hipStream_t of the
 * context's device; external = 1, the legacy default stream NULL included)
 * instead of its own non-blocking one (external = 0: back to its own).  A
 * caller whose buffers come from a framework stream (torch) then needs no host
 * synchronisation between its own work, its collectives and the engine. */
SCC_API int scc_ctx_set_stream(scc_ctx* ctx, void* stream, int32_t external);
/* Kernel timing (opts.profile = 1): total ms and launch count of a named
 * kernel family since the last reset ("gene_rank", "dist", "gram", ...). */
SCC_API int scc_ctx_kernel_time(const scc_ctx* ctx, const char* name, double* total_ms, int64_t* launches);
SCC_API void scc_ctx_reset_timers(scc_ctx* ctx);

/* ---- dataset: the genes x cells matrix as R holds it ------------------- */
/* dgCMatrix (CSC over cells): indptr[N+1] (R @p), rows[nnz] (R @i, 0-based
 * gene rows), vals[nnz] (R @x).  Replaces as.matrix(dataMatrix) (Fast:368).
 * SCC_PTR_HOST copies the arrays; SCC_PTR_DEVICE borrows them, and their
 * contents must not change while the dataset lives: the first error-free DE
 * run that reads every entry marks the dataset validated (rows in range and
 * sorted) and caches nodg, and later gene-shard runs read only their genes. */
SCC_API int scc_dataset_create_csc(scc_ctx* ctx, const int64_t* indptr, const int32_t* rows, const double* vals,
                           int64_t n_genes, int64_t n_cells, int64_t nnz, int32_t ptr_kind,
                           scc_dataset** out);
/* Gene-major CSR (genes x cells; per gene ascending cell columns, e.g. a
 * scipy csr_matrix or an AnnData .X transposed; BASELINE config E's CSR
 * input): indptr[G+1], cols[nnz] (0-based cells), vals[nnz].  Transposed once
 * on the device into the resident CSC over cells above (the dgCMatrix R
 * would hold for the same matrix), so every result equals the CSC path's.
 * Column indices outside [0, N), or not strictly ascending within a gene
 * (unsorted, or a repeated (gene, cell)), fail with SCC_ERR_INVALID here;
 * more than 262,144 genes with SCC_ERR_UNSUPPORTED.  No
 * reference interface: the reference takes dataMatrix as an R matrix
 * (Fast:22, :368); this is the R-free caller's equivalent. */
SCC_API int scc_dataset_create_csr(scc_ctx* ctx, const int64_t* indptr, const int32_t* cols, const double* vals,
                           int64_t n_genes, int64_t n_cells, int64_t nnz, int32_t ptr_kind,
                           scc_dataset** out);
/* base R matrix: G x N column-major doubles (slow:32 as.matrix). */
SCC_API int scc_dataset_create_dense(scc_ctx* ctx, const double* x_colmajor, int64_t n_genes, int64_t n_cells,
                             int32_t ptr_kind, scc_dataset** out);
/* Destroy every dataset before the context it was created on. */
SCC_API void scc_dataset_destroy(scc_dataset* ds);
/* Copy a sparse dataset's resident dgCMatrix (indptr[N+1], rows[nnz],
 * vals[nnz]) to host arrays: what the CSR transpose built, for checks and
 * for callers that want the CSC back (rows = vals = NULL: indptr only).  No
 * reference interface (the R side already holds its matrix). */
SCC_API int scc_dataset_read_csc(scc_dataset* ds, int64_t* indptr, int32_t* rows, double* vals);

/* ---- stage 1+2: per-cluster statistics, all-pairs Wilcoxon, BH, union --- */
SCC_API int scc_de_run(scc_ctx* ctx, const scc_dataset* ds, const int32_t* code /* host, [N] */, int32_t K,
               const scc_de_params* params, scc_de_result** out);

/* ---- the same DE sharded over gene row-blocks (one process per GPU) -------
 * Replaces the reference's per-cluster foreach workers (Fast:61-65,359,384):
 * every rank holds the whole dataset and runs scc_de_run_shard on its genes
 * [gene_lo, gene_hi); `shard` (device, scc_de_shard_bytes) receives the
 * per-(pair, gene) cells p, avg_logFC, pct1, pct2 (f64), 2U, ties (i64) and
 * flags (u8), each [n_pairs][G], zero outside the shard.  The caller sums the
 * shards of all ranks as int64 words (one all-reduce: the shards are
 * disjoint, so the sum is the exact union) and calls scc_de_finish on the
 * same context with the sum: per-pair BH, filters, top-N and the union, the
 * same result scc_de_run gives. */
SCC_API int64_t scc_de_shard_bytes(int32_t K, int64_t n_genes);
SCC_API int scc_de_run_shard(scc_ctx* ctx, const scc_dataset* ds, const int32_t* code /* host, [N] */, int32_t K,
                     const scc_de_params* params, int64_t gene_lo, int64_t gene_hi, void* shard /* device */);
SCC_API int scc_de_finish(scc_ctx* ctx, const scc_dataset* ds, const int32_t* code /* host, [N] */, int32_t K,
                  const scc_de_params* params, const void* shards_sum /* device */, scc_de_result** out);
/* The compact exchange (gather of per-(pair, tested gene)
 * records): scc_de_run_shard_records runs the shard's per-(pair, gene) stage
 * like scc_de_run_shard and packs, in (pair, gene) order, one scc_de_record per
 * cell the pair tests (FAST: the cells that pass the feature filters; SLOW:
 * every cell) into `records` (device, capacity `cap` records; cap >=
 * n_pairs * (gene_hi - gene_lo) always suffices), *n_records = the count.
 * The caller gathers every rank's records (block r = rank r's, stride
 * `stride` records apart, counts[r] valid) and calls scc_de_finish_records on
 * the same context: the result equals scc_de_run's. */
typedef struct {
    int32_t pair, gene;
    double p, avg_logfc, pct1, pct2;
    int64_t u2, ties;
    uint32_t flags, reserved;
} scc_de_record; /* 64 bytes */
SCC_API int scc_de_run_shard_records(scc_ctx* ctx, const scc_dataset* ds, const int32_t* code /* host, [N] */,
                                     int32_t K, const scc_de_params* params, int64_t gene_lo, int64_t gene_hi,
                                     void* records /* device */, int64_t cap, int64_t* n_records);
SCC_API int scc_de_finish_records(scc_ctx* ctx, const scc_dataset* ds, const int32_t* code /* host, [N] */, int32_t K,
                                  const scc_de_params* params, const void* records /* device */,
                                  const int64_t* counts /* host [n_blocks] */, int32_t n_blocks, int64_t stride,
                                  scc_de_result** out);
/* The per-pair selection of a FAST job split over the ranks by PAIRS (each
 * rank the pairs [pair_lo, pair_hi); the pairs are independent until the
 * union, Fast:359-392): scatters the gathered records like
 * scc_de_finish_records, runs BH / filters / top_n for its pairs only and
 * writes the first-occurrence key of every gene (u64 [G], device: pair-major
 * order key, all ones = not selected; ordered by (pair, rank in the pair)).
 * The caller combines the ranks' arrays by an element-wise MIN (all-reduce)
 * and scc_de_union_first_occ turns the combined array into deGeneUnion in
 * the reference's order (unique() over the pairs' top lists, Fast:392): the
 * same union scc_de_finish_records returns.  No result object. */
SCC_API int scc_de_finish_records_pairs(scc_ctx* ctx, const scc_dataset* ds, const int32_t* code /* host, [N] */,
                                        int32_t K, const scc_de_params* params, const void* records /* device */,
                                        const int64_t* counts /* host [n_blocks] */, int32_t n_blocks, int64_t stride,
                                        int32_t pair_lo, int32_t pair_hi, void* first_occ /* device u64 [G] */);
SCC_API int scc_de_union_first_occ(scc_ctx* ctx, const void* first_occ /* device u64 [G] */, int64_t n_genes,
                                   int32_t* genes /* host [G] */, int32_t* n_union);

/* n_pairs = K(K-1)/2; n_rows = FAST tested rows over all pairs (0 for SLOW);
 * n_union = |deGeneUnion|. */
SCC_API int scc_de_result_counts(const scc_de_result* r, int32_t* n_pairs, int64_t* n_rows, int32_t* n_union);
/* deGeneUnion as 0-based gene rows, in the reference's order (Fast:392 / slow:224). */
SCC_API int scc_de_result_union(const scc_de_result* r, int32_t* genes);
/* FAST rows, pair-major, inside a pair in R's order(p, -avg_logFC) (Fast:346):
 * every tested feature of every pair.  flags bit0 = kept DE row
 * (pair has > 1 row and q < qValThrs, Fast:376-377), bit1 = survives
 * top_n (Fast:391).  u2 = 2 * W (W = wilcox STATISTIC); ties = sum(t^3 - t).
 * Any pointer may be NULL. */
SCC_API int scc_de_result_rows(const scc_de_result* r, int32_t* pair_rows /* [n_pairs] */, int32_t* gene,
                       double* p, double* q, double* avg_logfc, double* pct1, double* pct2, int64_t* u2,
                       int64_t* ties, uint8_t* flags);
/* SLOW per-pair full vectors [n_pairs][G] (the qValueList/logFCList RDS dumps,
 * slow:181-184,200-202) plus p, u2 and de (0/1).  Any pointer may be NULL. */
SCC_API int scc_de_result_pair_vectors(const scc_de_result* r, double* p, double* q, double* logfc, int64_t* u2,
                               uint8_t* de);
/* log(meanScalingFactor * mean(expm1(X))) used by SLOW (slow:36,111). */
SCC_API int scc_de_result_log_threshold(const scc_de_result* r, double* log_thr);
/* nodg: number of genes with x > 0 per cell, all cells (Fast:440-443). */
SCC_API int scc_de_result_nodg(const scc_de_result* r, int32_t* nodg /* [N] */);
SCC_API void scc_de_result_destroy(scc_de_result* r);

/* ---- stage 3: cell x cell distance on the DE-gene union ---------------- */
/* Packed lower triangle in R `dist` order (column-major: (1,0),(2,0),...,
 * (N-1,0),(2,1),...), length N(N-1)/2.  out_kind SCC_PTR_HOST copies to the
 * caller's host buffer; SCC_PTR_DEVICE writes a device buffer of the ctx
 * device (dist_out == NULL: the engine keeps it HBM-resident in its own
 * workspace, valid until the next call; that call returns as soon as its work
 * is queued, and a failure of its eigensolver's cross-workgroup hand-off is
 * reported by the next synchronising call: scc_ctx_synchronize, scc_de_run,
 * or an scc_distance into a host or caller buffer).  ncomp <= 0 means min(n_union, 15) (Fast:398).  out_f32 != 0 writes
 * float instead of double. */
SCC_API int scc_distance(scc_ctx* ctx, const scc_dataset* ds, const int32_t* genes /* host */, int32_t n_union,
                 int32_t metric, int32_t ncomp, void* dist_out, int32_t out_kind, int32_t out_f32);
/* reclusterDEConsensusFast's compute path in one call (Fast:57-400): the DE
 * of scc_de_run, then scc_distance over its gene union, without returning to
 * the caller in between (one host round trip fewer per job).  *out receives
 * the DE result as from scc_de_run (the union: scc_de_result_union); the
 * distance goes to dist_out as in scc_distance.  An empty union fails with
 * SCC_ERR_INVALID after *out is set. */
SCC_API int scc_de_distance(scc_ctx* ctx, const scc_dataset* ds, const int32_t* code /* host, [N] */, int32_t K,
                    const scc_de_params* params, int32_t metric, int32_t ncomp, void* dist_out, int32_t out_kind,
                    int32_t out_f32, scc_de_result** out);
/* The same for the columns [col_lo, col_hi) only: entries
 * [col_lo(2N-col_lo-1)/2, col_hi(2N-col_hi-1)/2) of the packed R `dist`
 * vector, a contiguous slice.  Ranks that split [0, N) into column ranges of
 * equal entry counts each compute and keep their slice (the
 * distance tiles stay HBM-resident per GPU); the PCA is recomputed on every
 * rank.  The eigensolver's reductions have a fixed shape (no dependence on how
 * many workgroups joined a hand-off), so every rank gets the same scores bit
 * for bit on the same device type. */
SCC_API int scc_distance_cols(scc_ctx* ctx, const scc_dataset* ds, const int32_t* genes /* host */,
                      int32_t n_union, int32_t metric, int32_t ncomp, int64_t col_lo, int64_t col_hi,
                      void* dist_out, int32_t out_kind, int32_t out_f32);
/* ---- stage 3 sharded over ranks (one process per GPU) --------
 * prcomp_irlba + dist (Fast:398-400) of ONE job over the ranks of a process
 * group: every rank holds the dataset and owns the cells [cell_lo, cell_hi)
 * (ranks in order, covering [0, N)).  Each rank calls, with the same genes:
 *   scc_pca_shard_colsum(.., part)      part: device, 2 * n_union doubles =
 *       this rank's double-double column sums of X[U, cell_lo:cell_hi)
 *   -> the caller all-gathers the parts in rank order: parts [world][2 n_union]
 *   scc_pca_shard_gram(.., parts, world, gram)   gram: device, n_union^2
 *       doubles = this rank's partial Gram of the centred rows
 *   -> the caller all-reduces (sums) gram
 *   scc_pca_shard_scores(.., gram_sum, ncomp, scores)   scores: device
 *       [N][16] doubles; rows [cell_lo, cell_hi) written, others untouched
 *   -> the caller combines the score rows of all ranks (disjoint)
 *   scc_distance_scores(.., scores, ..)  the packed `dist` columns
 *       [col_lo, col_hi) from the full score matrix.
 * The mean is the same double-double sum as the unsharded path's, combined in
 * rank order, so every rank sees identical bits; the eigensolve of the summed
 * Gram runs once (scc_pca_shard_eigen on rank 0, vectors broadcast) or on every
 * rank (scc_pca_shard_scores = eigen + project, single-rank use). */
SCC_API int scc_pca_shard_colsum(scc_ctx* ctx, const scc_dataset* ds, const int32_t* genes /* host */,
                                 int32_t n_union, int64_t cell_lo, int64_t cell_hi, void* part /* device */);
SCC_API int scc_pca_shard_gram(scc_ctx* ctx, const void* parts /* device [world][2 n_union] */, int32_t world,
                               void* gram /* device [n_union][n_union] */);
SCC_API int scc_pca_shard_scores(scc_ctx* ctx, const void* gram_sum /* device */, int32_t ncomp,
                                 void* scores /* device [N][16] */);
/* scc_pca_shard_scores in two halves, so the eigenvectors can come from ONE
 * rank: scc_pca_shard_eigen writes the top-ncomp eigenvectors of gram_sum as
 * vecs [n_union][16] doubles (device; columns >= ncomp zero); the caller
 * broadcasts rank 0's vecs; scc_pca_shard_project scores this rank's cells
 * with them (rows [cell_lo, cell_hi) of scores).  The eigensolver's hand-off
 * kernel sums per-workgroup partials and how many workgroups join depends on
 * arrival order, so separate eigensolves may differ in the last bits; one
 * broadcast set of vectors makes every rank's block a block of one embedding. */
SCC_API int scc_pca_shard_eigen(scc_ctx* ctx, const void* gram_sum /* device */, int32_t ncomp,
                                void* vecs /* device [n_union][16] */);
SCC_API int scc_pca_shard_project(scc_ctx* ctx, const void* vecs /* device [n_union][16] */, int32_t ncomp,
                                  void* scores /* device [N][16] */);
/* Packed `dist` columns [col_lo, col_hi) from a device score matrix [N][16]
 * (components >= ncomp zero); output as in scc_distance_cols. */
SCC_API int scc_distance_scores(scc_ctx* ctx, const void* scores /* device */, int64_t n_cells, int64_t col_lo,
                                int64_t col_hi, void* dist_out, int32_t out_kind, int32_t out_f32);

/* ---- silhouette on the distance vector (Fast:433) ---------
 * cluster::silhouette(groups, dmatrix = as.matrix(d)) without the N x N
 * matrix: widths[i] = s(i) (0 for a singleton cluster), clus_avg[k] = mean
 * width of the k-th cluster in increasing group-id order (summary(.)$
 * clus.avg.widths; the reference averages them into "SI").  dist: device
 * pointer to the full packed vector (f64, or f32 if dist_f32), or NULL for
 * the engine-kept output of the last full scc_distance call.  Needs
 * 2 <= n_groups < n_cells (R returns NA otherwise).  Any output may be NULL. */
SCC_API int scc_silhouette(scc_ctx* ctx, int64_t n_cells, const int32_t* groups /* host [N] */, const void* dist,
                   int32_t dist_f32, double* widths /* host [N] */, double* clus_avg /* host [n_groups] */,
                   int32_t* n_groups);
/* PCA scores (N x ncomp, row-major) of the last PCA distance call. */
SCC_API int scc_last_pca_scores(const scc_ctx* ctx, double* scores, int32_t* ncomp);

/* ---- host clustering on the packed distance --------------
 * Host code (no device needed), restating the packages the reference calls:
 *   fastcluster::hclust(d, method = "ward.D2")            Fast:406-411
 *     merge: [2 (n-1)] int32, R's column-major (n-1) x 2 merge matrix
 *     (-i = observation i, +k = merge k, 1-based); height [n-1]; order [n]
 *     (1-based leaf order, may be NULL).  dist: host packed R `dist` vector.
 *   dynamicTreeCut::cutreeDynamic(dendro, distM = as.matrix(d), deepSplit,
 *     pamStage = FALSE, minClusterSize) (method "hybrid", default cut height)
 *                                                         Fast:421-427
 *     labels [n]: 0 = unassigned, 1.. by decreasing cluster size; cut_height
 *     (may be NULL) receives the default cut height used. */
SCC_API int scc_hclust_ward_d2(const double* dist, int64_t n, int32_t* merge, double* height, int32_t* order);
SCC_API int scc_cutree_hybrid(const int32_t* merge, const double* height, int64_t n, const double* dist,
                              int32_t deep_split, int32_t min_cluster_size, int32_t* labels, double* cut_height);

/* ---- diagnostics (tests): the PCA eigensolver's parts on device pointers --
 * Not on the R path.  Each synchronises the device and returns 0 on success.
 *   scc_diag_eigen_topk   top-k eigenpairs of a device n x n symmetric A (lda)
 *                         through the engine's eigensolver (Z [n][16], W [k]);
 *                         *path: which solver answered (0 direct, 1 subspace
 *                         iteration, 2 Chebyshev-filtered subspace iteration)
 *   scc_diag_small_syev   the one-workgroup solver for n <= 64 (Rayleigh-Ritz)
 *   scc_diag_cholinv      T = R^-1 of G + shift_rel tr(G) I = R^T R, P = 48 or 64
 *   scc_diag_eig_last_path  the calling thread's last answer path */
SCC_API int scc_diag_eigen_topk(const double* A, int n, int lda, int k, double* Z, double* W, int* path);
SCC_API int scc_diag_small_syev(const double* H, int n, int ldh, int k, double* Y, double* theta, unsigned* flag);
SCC_API int scc_diag_cholinv(const double* G, int P, double shift_rel, double* T, unsigned* flag);
SCC_API int scc_diag_eig_last_path(void);
/* s_memtime stamps of the last scc_diag_small_syev's phases [8] */
SCC_API int scc_diag_small_syev_stamps(unsigned long long* out);

#ifdef __cplusplus
}
#endif
#endif /* SCC_H */
