# scConsensusAMD.R — drop-in R wrappers that route the data-parallel core of
# scConsensus to the MI355X engine (libscc via .Call; see INTEGRATION.md).
#
# Signatures and return objects are those of the reference:
#   reclusterDEConsensusFast  R/reclusterDEConsensusFast.R:22-33, returns :446-450
#   reclusterDEConsensus      R/reclusterDEConsensus.R:20-29,      returns :278-282
# Kept in R (host), exactly as the reference does them: cluster selection
# (table / grepl("grey") / locale order), hclust(ward.D2), cutreeDynamic,
# labels2colors, silhouette, saveRDS, printing and cellTypeDEPlot.

# Cluster selection exactly as Fast:39-47 / slow:38-48: table() over ALL of
# consensusClusterLabels (locale collation), "> minClusterSize", no "grey";
# then each matrix column's code (0-based index into the kept clusters, -1
# for cells of other clusters or without a label).
.scc_codes <- function(consensusClusterLabels, dataMatrix, minClusterSize) {
  colorCounts <- table(consensusClusterLabels)
  keep <- names(colorCounts[colorCounts > minClusterSize])
  keep <- keep[!grepl("grey", keep)]
  if (is.null(names(consensusClusterLabels))) names(consensusClusterLabels) <- colnames(dataMatrix)
  colLabels <- consensusClusterLabels[colnames(dataMatrix)]
  code <- match(as.character(colLabels), keep) - 1L
  code[is.na(code)] <- -1L
  list(clusters = keep, code = as.integer(code))
}

.scc_slots <- function(m) {
  if (inherits(m, "dgCMatrix")) {
    list(x = m@x, p = m@p, i = m@i, dim = dim(m))
  } else if (inherits(m, "dgRMatrix")) {
    # gene-major CSR: a third dim entry 1L selects scc_dataset_create_csr
    list(x = m@x, p = m@p, i = m@j, dim = c(dim(m), 1L))
  } else {
    m <- as.matrix(m)
    storage.mode(m) <- "double"
    list(x = m, p = NULL, i = NULL, dim = dim(m))
  }
}

# the matrix uploaded ONCE per call of the R function; DE and distance share
# the device copy through this handle (freed by C_scc_release or the GC)
.scc_dataset <- function(m) {
  s <- .scc_slots(m)
  .Call("C_scc_dataset", s$x, s$p, s$i, s$dim)
}

.scc_dist <- function(h, genes, n_cells, metric = 0L) {
  d <- .Call("C_scc_distance", h, as.integer(genes), as.integer(metric), 0L)
  structure(d, Size = n_cells, Diag = FALSE, Upper = FALSE,
            method = if (metric == 0L) "euclidean" else "pearson", class = "dist")
}

# hclust(ward.D2) as Fast:406-411; with options(scConsensus.engineTree = TRUE)
# the engine's C++ restatement (no fastcluster needed; same merge rule)
.scc_hclust <- function(d) {
  if (isTRUE(getOption("scConsensus.engineTree", FALSE))) {
    t <- .Call("C_scc_hclust", d)
    return(structure(list(merge = t[[1]], height = t[[2]], order = t[[3]], labels = attr(d, "Labels"),
                          method = "ward.D2", call = match.call(), dist.method = attr(d, "method")),
                     class = "hclust"))
  }
  if (requireNamespace("fastcluster", quietly = TRUE)) fastcluster::hclust(d, method = "ward.D2")
  else stats::hclust(d, method = "ward.D2")
}

.scc_tree_and_colors <- function(d, deepSplitValues, minClusterSize, with_si) {
  tree <- .scc_hclust(d)
  # cutreeDynamic needs distM = as.matrix(d): N^2 doubles on the host (5.4 GB
  # at 26k cells, 80 GB at 100k, 320 GB at 200k).  options(scConsensus.engineCut
  # = TRUE) runs the engine's restatement of the hybrid cut on the packed d
  # instead (parity against dynamicTreeCut itself unpinned: INTEGRATION.md)
  engine_cut <- isTRUE(getOption("scConsensus.engineCut", FALSE))
  dm <- if (engine_cut) NULL else as.matrix(d)
  colors <- list()
  for (dsv in deepSplitValues) {
    grp <- if (engine_cut) {
      .Call("C_scc_cutree", tree$merge, as.double(tree$height), d, as.integer(dsv), as.integer(minClusterSize))
    } else {
      dynamicTreeCut::cutreeDynamic(dendro = tree, distM = dm, deepSplit = dsv,
                                    pamStage = FALSE, minClusterSize = minClusterSize)
    }
    colors[[paste("deepsplit:", dsv)]] <- WGCNA::labels2colors(grp)
    # deepSplitInfo's SI (Fast:433, computed and discarded by the reference):
    # the engine's silhouette on its HBM-resident copy of d (no N x N matrix)
    if (with_si) invisible(.Call("C_scc_si", as.integer(grp)))
  }
  names(colors) <- paste("deepsplit:", deepSplitValues)
  list(tree = tree, colors = colors)
}

reclusterDEConsensusFast <- function(dataMatrix, consensusClusterLabels, method = "wilcox",
                                     qValThrs = 0.1, logFCThrs = 0.5, deepSplitValues = 1:4,
                                     minClusterSize = 10, minPerCent = 20,
                                     filename = "de_gene_object.rds", plotName = "DE_Heatmap",
                                     NumbertopDEGenes = 30, nCores = 1) {
  # test.use = method (Fast:372): "wilcox" and "t" run on the engine; "bimod" /
  # "roc" need Seurat helpers the reference never loads
  if (!(method %in% c("wilcox", "t"))) stop("Unknown test: ", method)
  sel <- .scc_codes(consensusClusterLabels, dataMatrix, minClusterSize)
  # nCores PSOCK workers (Fast:61-65) -> min(nCores, GPUs) devices of ONE sharded job
  .Call("C_scc_devices", as.integer(nCores))
  h <- .scc_dataset(dataMatrix)
  on.exit(.Call("C_scc_release", h), add = TRUE)
  res <- .Call("C_scc_de_fast", h, sel$code, length(sel$clusters),
               as.double(qValThrs), as.double(logFCThrs), as.double(minPerCent),
               as.integer(NumbertopDEGenes), as.integer(method == "t"))
  deGeneUnion <- rownames(dataMatrix)[res[[1]]]
  print(str(deGeneUnion))
  d <- .scc_dist(h, res[[1]], ncol(dataMatrix))
  tc <- .scc_tree_and_colors(d, deepSplitValues, minClusterSize, with_si = TRUE)
  out <- list("deGeneUnion" = deGeneUnion, "cellTree" = tc$tree, "dynamicColors" = tc$colors)
  saveRDS(object = out, file = filename)
  cellTypeDEPlot(dataMatrix = dataMatrix[deGeneUnion, ], nodg = res[[2]], cellTree = tc$tree,
                 clusterLabels = consensusClusterLabels, dynamicColorsList = tc$colors,
                 colScheme = "violet", filename = plotName)
  out
}

reclusterDEConsensus <- function(dataMatrix, consensusClusterLabels, method = "Wilcoxon",
                                 meanScalingFactor = 5, qValThrs, fcThrs, deepSplitValues = 1:4,
                                 minClusterSize = 10, filename = "de_gene_object.rds",
                                 plotName = "DE_Heatmap") {
  if (method != "Wilcoxon") {
    print("Incorrect method chosen.")
    return(NULL)
  }
  sel <- .scc_codes(consensusClusterLabels, dataMatrix, minClusterSize)
  h <- .scc_dataset(dataMatrix)
  on.exit(.Call("C_scc_release", h), add = TRUE)
  res <- .Call("C_scc_de_slow", h, sel$code, length(sel$clusters),
               as.double(qValThrs), as.double(fcThrs), as.double(meanScalingFactor))
  K <- length(sel$clusters)
  qValueList <- rep(list(list()), K); logFCList <- rep(list(list()), K); deGeneList <- rep(list(list()), K)
  pcol <- 0L
  for (a in seq_len(K - 1)) for (b in (a + 1):K) {
    pcol <- pcol + 1L
    de <- as.integer(res[[4]][, pcol]) == 1L
    print(paste0(sel$clusters[a], ", ", sel$clusters[b], " DE genes: ", sum(de)))
    qValueList[[a]][[b]] <- res[[2]][, pcol]
    logFCList[[a]][[b]] <- res[[3]][, pcol]
    deGeneList[[a]][[b]] <- rownames(dataMatrix)[de]
  }
  names(qValueList) <- names(logFCList) <- names(deGeneList) <- sel$clusters
  saveRDS(object = qValueList, file = "qValueList.rds")
  saveRDS(object = logFCList, file = "logFCList.rds")
  saveRDS(object = deGeneList, file = "deGeneList.rds")
  deGeneUnion <- rownames(dataMatrix)[res[[1]]]
  print(str(deGeneUnion))
  saveRDS(deGeneUnion, file = "deGeneUnion.rds")
  d <- .scc_dist(h, res[[1]], ncol(dataMatrix))
  tc <- .scc_tree_and_colors(d, deepSplitValues, minClusterSize, with_si = FALSE)
  out <- list("deGeneUnion" = deGeneUnion, "cellTree" = tc$tree, "dynamicColors" = tc$colors)
  saveRDS(object = out, file = filename)
  cellTypeDEPlot(dataMatrix = as.matrix(dataMatrix)[deGeneUnion, ], nodg = res[[5]], cellTree = tc$tree,
                 clusterLabels = consensusClusterLabels, dynamicColorsList = tc$colors,
                 colScheme = "violet", filename = plotName)
  out
}
