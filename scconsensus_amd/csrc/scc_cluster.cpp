// scc_cluster.cpp — host-side tree building and dynamic tree cut on the packed
// distance vector (include/scc.h: scc_hclust_ward_d2,
// scc_cutree_hybrid, scc_labels2colors).
//
// The reference keeps these on the host (north_star: "flashClust/
// dynamicTreeCut ... stay on the host CPU as in the reference"):
//   cellTree = fastcluster::hclust(d, method = "ward.D2")     Fast:406-411
//   cutreeDynamic(dendro = cellTree, distM = as.matrix(d), deepSplit = dsv,
//                 pamStage = FALSE, minClusterSize = minClusterSize)  Fast:421-427
//   WGCNA::labels2colors(dynamicGroups)                       Fast:428
// R and those packages are absent from the image, so these are
// restatements of the packages' published algorithms (versions unpinned by the
// reference's DESCRIPTION:8):
//   fastcluster (Müllner): ward.D2 = squared input, NN-chain with the
//     Lance-Williams Ward update, sqrt of the heights, stable sort by height,
//     union-find relabelling to R's merge convention, R's left-to-right order.
//   dynamicTreeCut::cutreeHybrid (Langfelder et al.), pamStage = FALSE: the
//     branch-building pass over the merges below the cut height, the
//     core-scatter / gap / size merge criteria, cluster assignment and the
//     size-ranked relabelling.
// Nothing here needs the N x N matrix: entries are read from the packed R
// `dist` vector (or a full symmetric working copy when it fits) directly.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "scc.h"

namespace {

// packed R `dist` index of (i, j), i != j: column-major lower triangle ==
// row-major upper triangle of (min, max)
inline int64_t pidx(int64_t n, int64_t i, int64_t j)
{
    if (i > j) std::swap(i, j);
    return (2 * n - 3 - i) * i / 2 + j - 1;
}

// ---- hclust(ward.D2) -------------------------------------------------------

struct Step {
    int64_t a, b;
    double h;
};

// Working distance matrix of squared distances.  FULL keeps both triangles
// (every scan is a contiguous row); otherwise the packed triangle (half the
// memory, column reads strided) — fastcluster's own layout.
template <bool FULL>
struct WorkD {
    int64_t n;
    std::vector<double> d;
    double& at(int64_t i, int64_t j) { return FULL ? d[(size_t)(i * n + j)] : d[(size_t)pidx(n, i, j)]; }
    void set(int64_t i, int64_t j, double v)
    {
        if (FULL) {
            d[(size_t)(i * n + j)] = v;
            d[(size_t)(j * n + i)] = v;
        } else {
            d[(size_t)pidx(n, i, j)] = v;
        }
    }
};

// NN-chain core (fastcluster NN_chain_core<METHOD_METR_WARD>): the chain tip
// handling, scan order (active nodes ascending, strict <, starting from the
// previous chain element's distance) and the update arithmetic
//   d(k, i∪j) = ((s_k+s_i) d(k,i) + (s_k+s_j) d(k,j) - s_k d(i,j)) / (s_i+s_j+s_k)
// (f_ward, operands in that order) follow the package, so ties resolve as it
// resolves them.  The surviving node is the larger index.
template <bool FULL>
static void nn_chain_ward(WorkD<FULL>& D, std::vector<Step>& out)
{
    const int64_t N = D.n;
    std::vector<int64_t> chain(N), succ(N + 1), pred(N + 1);
    std::vector<double> size(N, 1.0);
    for (int64_t i = 0; i <= N; ++i) {
        succ[i] = i + 1;
        pred[i] = i - 1;
    }
    int64_t start = 0;
    auto remove = [&](int64_t idx) {
        if (idx == start) {
            start = succ[idx];
        } else {
            succ[pred[idx]] = succ[idx];
            pred[succ[idx]] = pred[idx];
        }
        succ[idx] = 0;
    };
    int64_t tip = 0, i1 = 0, i2 = 0;
    double mn = 0.0;
    for (int64_t step = 0; step < N - 1; ++step) {
        if (tip <= 3) {
            chain[0] = i1 = start;
            tip = 1;
            i2 = succ[i1];
            mn = D.at(i1, i2);
            for (int64_t i = succ[i2]; i < N; i = succ[i]) {
                const double v = D.at(i1, i);
                if (v < mn) {
                    mn = v;
                    i2 = i;
                }
            }
        } else {
            tip -= 3;
            i1 = chain[tip - 1];
            i2 = chain[tip];
            mn = D.at(i1, i2);
        }
        do {
            chain[tip] = i2;
            if (FULL) {
                const double* row = &D.d[(size_t)(i2 * N)];
                for (int64_t i = start; i < N; i = succ[i]) {
                    if (i == i2) continue;
                    if (row[i] < mn) {
                        mn = row[i];
                        i1 = i;
                    }
                }
            } else {
                int64_t i = start;
                for (; i < i2; i = succ[i]) {
                    const double v = D.at(i, i2);
                    if (v < mn) {
                        mn = v;
                        i1 = i;
                    }
                }
                for (i = succ[i2]; i < N; i = succ[i]) {
                    const double v = D.at(i2, i);
                    if (v < mn) {
                        mn = v;
                        i1 = i;
                    }
                }
            }
            i2 = i1;
            i1 = chain[tip++];
        } while (i2 != chain[tip - 2]);

        out.push_back({i1, i2, mn});
        if (i1 > i2) std::swap(i1, i2);
        const double s = size[i1], t = size[i2];
        size[i2] += size[i1];
        remove(i1);
        for (int64_t i = start; i < N; i = succ[i]) {
            if (i == i2) continue;
            const double v = size[i];
            const double b = D.at(i, i2), a = D.at(i, i1);
            D.set(i, i2, ((v + s) * a - v * mn + (v + t) * b) / (s + t + v));
        }
    }
}

static void ward_d2(const double* dist, int64_t N, int32_t* merge, double* height, int32_t* order, bool full)
{
    std::vector<Step> st;
    st.reserve((size_t)N);
    if (full) {
        WorkD<true> D{N, std::vector<double>((size_t)(N * N), 0.0)};
        for (int64_t j = 0; j < N; ++j)
            for (int64_t i = j + 1; i < N; ++i) {
                const double x = dist[pidx(N, i, j)];
                D.set(i, j, x * x);
            }
        nn_chain_ward(D, st);
    } else {
        const int64_t M = N * (N - 1) / 2;
        WorkD<false> D{N, std::vector<double>((size_t)M)};
        for (int64_t k = 0; k < M; ++k) D.d[(size_t)k] = dist[k] * dist[k];
        nn_chain_ward(D, st);
    }
    for (auto& s : st) s.h = std::sqrt(s.h);
    std::stable_sort(st.begin(), st.end(), [](const Step& x, const Step& y) { return x.h < y.h; });
    // union-find: the k-th merge in height order becomes node N + k
    std::vector<int64_t> parent(2 * N - 1, 0);
    auto find = [&](int64_t x) {
        int64_t r = x;
        while (parent[r]) r = parent[r];
        while (parent[x] && parent[x] != r) {
            const int64_t nx = parent[x];
            parent[x] = r;
            x = nx;
        }
        return r;
    };
    std::vector<int64_t> nsize(N - 1);
    auto sz = [&](int64_t node) { return node < N ? (int64_t)1 : nsize[node - N]; };
    for (int64_t k = 0; k < N - 1; ++k) {
        int64_t a = find(st[k].a), b = find(st[k].b);
        parent[a] = parent[b] = N + k;
        if (a > b) std::swap(a, b);
        merge[k] = a < N ? -(int32_t)a - 1 : (int32_t)(a - N + 1);
        merge[k + N - 1] = b < N ? -(int32_t)b - 1 : (int32_t)(b - N + 1);
        height[k] = st[k].h;
        nsize[k] = sz(a) + sz(b);
    }
    // left-to-right leaf order (fastcluster order_nodes)
    if (order) {
        struct PN {
            int64_t pos, node;
        };
        std::vector<PN> q;
        q.push_back({0, N - 2});
        while (!q.empty()) {
            PN cur = q.back();
            q.pop_back();
            int64_t pos = cur.pos;
            const int32_t c1 = merge[cur.node], c2 = merge[cur.node + N - 1];
            if (c1 < 0) {
                order[pos++] = -c1;
            } else {
                q.push_back({pos, c1 - 1});
                pos += nsize[c1 - 1];
            }
            if (c2 < 0) order[pos] = -c2;
            else q.push_back({pos, c2 - 1});
        }
    }
}

// ---- cutreeDynamic(method = "hybrid", pamStage = FALSE) ---------------------

// R's mean(): long-double sum / n, then one correction pass (summary.c)
static double r_mean(const std::vector<double>& x)
{
    const size_t n = x.size();
    long double s = 0.0L;
    for (double v : x) s += v;
    s /= (long double)n;
    long double t = 0.0L;
    for (double v : x) t += (long double)v - s;
    s += t / (long double)n;
    return (double)s;
}

// mean(colSums(distM[Core, Core]) / (coresize - 1)); colSums accumulates in
// long double (R's do_colsum); core holds 1-based object ids
static double core_scatter(const double* dist, int64_t N, const int32_t* core, int cs)
{
    std::vector<double> col((size_t)cs);
    for (int j = 0; j < cs; ++j) {
        long double s = 0.0L;
        const int64_t cj = core[j] - 1;
        for (int i = 0; i < cs; ++i) {
            const int64_t ci = core[i] - 1;
            s += ci == cj ? 0.0 : dist[pidx(N, ci, cj)];
        }
        col[(size_t)j] = (double)s / (double)(cs - 1);
    }
    return r_mean(col);
}

// .CoreSize(BranchSize, minClusterSize)
static int core_size(int branch_size, int min_cluster_size)
{
    const double base = min_cluster_size / 2.0 + 1.0;
    if (base < branch_size) return (int)(base + std::sqrt((double)branch_size - base));
    return branch_size;
}

// .interpolate(data, index)
static double interpolate(const double* data, int n, double index)
{
    const double i = std::nearbyint(index);  // R round(): half to even
    if (i < 1) return data[0];
    if (i >= n) return data[n - 1];
    const double r = index - i;
    return data[(int)i - 1] * (1 - r) + data[(int)i] * r;
}

struct Branch {
    bool is_basic = true, is_top_basic = true, fail_size = false;
    double attach_height = NAN;
    int size = 2, n_merge = 1, n_basic = 0;
    int merged_into = 0;
    std::vector<int32_t> singletons, basic, merging_h_dummy;
};

static int cutree_hybrid(const int32_t* merge, const double* height, int64_t N, const double* dist, int deep_split,
                         int min_cluster_size, int32_t* labels, double* cut_out, std::string& err)
{
    const int64_t n_merge = N - 1;
    double hmax = -INFINITY;
    for (int64_t m = 0; m < n_merge; ++m) hmax = std::max(hmax, height[m]);
    // reference height: the merge at the 5 % quantile of the merge list
    int64_t ref_merge = (int64_t)std::nearbyint((double)n_merge * 0.05);
    if (ref_merge < 1) ref_merge = 1;
    const double ref_height = height[ref_merge - 1];
    const double cut_height = 0.99 * (hmax - ref_height) + ref_height;
    if (cut_out) *cut_out = cut_height;
    int64_t n_below = 0;
    for (int64_t m = 0; m < n_merge; ++m) n_below += height[m] <= cut_height;
    std::fill(labels, labels + N, 0);
    if (n_below < min_cluster_size) return SCC_OK;  // "all data will be unlabeled"

    static const double defMCS[5] = {0.64, 0.73, 0.82, 0.91, 0.95};
    double defMG[5];
    for (int i = 0; i < 5; ++i) defMG[i] = (1 - defMCS[i]) * 3 / 4;
    const double ds = deep_split + 1;
    if (ds < 1 || ds > 5) {
        err = "Parameter deepSplit out of range: allowable range is 0 through 4";
        return SCC_ERR_INVALID;
    }
    const double max_core_scatter = interpolate(defMCS, 5, ds);
    const double min_gap = interpolate(defMG, 5, ds);
    const double max_abs_core_scatter = ref_height + max_core_scatter * (cut_height - ref_height);
    const double min_abs_gap = min_gap * (cut_height - ref_height);
    const double min_abs_split_height = ref_height + 0.0 * (cut_height - ref_height);

    std::vector<Branch> br(1);  // 1-based like R
    br.reserve((size_t)n_below + 2);
    std::vector<int32_t> merge_to_branch((size_t)n_merge, 0);
    auto scatter_of = [&](const Branch& b) {
        const int cs = core_size((int)b.singletons.size(), min_cluster_size);
        return core_scatter(dist, N, b.singletons.data(), cs);
    };
    for (int64_t m = 0; m < n_merge; ++m) {
        if (!(height[m] <= cut_height)) continue;
        const int32_t m1 = merge[m], m2 = merge[m + n_merge];
        const double h = height[m];
        if (m1 < 0 && m2 < 0) {
            Branch b;
            b.singletons = {-m1, -m2};
            br.push_back(std::move(b));
            merge_to_branch[(size_t)m] = (int32_t)(br.size() - 1);
        } else if ((m1 < 0) != (m2 < 0)) {
            const int32_t clust = merge_to_branch[(size_t)std::max(m1, m2) - 1];
            if (clust == 0) {
                err = "Internal error: a previous merge has no associated cluster";
                return SCC_ERR_INVALID;
            }
            const int32_t gene = -std::min(m1, m2);
            Branch& b = br[(size_t)clust];
            if (b.is_basic) b.singletons.push_back(gene);
            b.size += 1;
            b.n_merge += 1;
            merge_to_branch[(size_t)m] = clust;
        } else {
            int32_t c1 = merge_to_branch[(size_t)m1 - 1], c2 = merge_to_branch[(size_t)m2 - 1];
            // rank(sizes, ties.method = "first"): the first is small unless strictly larger
            int32_t small = c1, large = c2;
            if (br[(size_t)c1].size > br[(size_t)c2].size) std::swap(small, large);
            const double sm_ave = br[(size_t)small].is_basic ? scatter_of(br[(size_t)small]) : 0.0;
            const double lg_ave = br[(size_t)large].is_basic ? scatter_of(br[(size_t)large]) : 0.0;
            bool do_merge = false, smaller_fail_size = false;
            {
                const Branch& s = br[(size_t)small];
                const bool c2s = s.size < min_cluster_size, c3 = sm_ave > max_abs_core_scatter,
                           c4 = h - sm_ave < min_abs_gap, c5 = h < min_abs_split_height;
                if (s.is_basic && (c2s || c3 || c4 || c5)) {
                    do_merge = true;
                    smaller_fail_size = !(c3 || c4);
                } else {
                    const Branch& l = br[(size_t)large];
                    const bool d2 = l.size < min_cluster_size, d3 = lg_ave > max_abs_core_scatter,
                               d4 = h - lg_ave < min_abs_gap, d5 = h < min_abs_split_height;
                    if (l.is_basic && (d2 || d3 || d4 || d5)) {
                        do_merge = true;
                        smaller_fail_size = !(d3 || d4);
                        std::swap(small, large);
                    }
                }
            }
            if (do_merge) {
                Branch& s = br[(size_t)small];
                Branch& l = br[(size_t)large];
                s.fail_size = smaller_fail_size;
                s.merged_into = large;
                s.attach_height = h;
                s.is_top_basic = false;
                if (l.is_basic) {
                    l.singletons.insert(l.singletons.end(), s.singletons.begin(), s.singletons.end());
                } else if (!s.is_basic) {
                    err = "Internal error: merging two composite clusters";
                    return SCC_ERR_INVALID;
                }
                l.n_merge += 1;
                l.size += s.size;
                merge_to_branch[(size_t)m] = large;
            } else {
                if (br[(size_t)large].is_basic && !br[(size_t)small].is_basic) std::swap(small, large);
                if (br[(size_t)large].is_basic) {  // (pamStage & pamRespectsDendro) is FALSE here
                    Branch nb;
                    nb.is_basic = false;
                    nb.is_top_basic = false;
                    {
                        Branch& s = br[(size_t)small];
                        Branch& l = br[(size_t)large];
                        s.attach_height = l.attach_height = h;
                        s.merged_into = l.merged_into = (int)br.size();
                        if (s.is_basic) nb.basic.push_back(small);
                        else nb.basic = s.basic;
                        if (l.is_basic) nb.basic.push_back(large);
                        else nb.basic.insert(nb.basic.end(), l.basic.begin(), l.basic.end());
                        nb.n_merge = 2;
                        nb.size = s.size + l.size;
                        nb.n_basic = (int)nb.basic.size();
                    }
                    br.push_back(std::move(nb));
                    merge_to_branch[(size_t)m] = (int32_t)(br.size() - 1);
                } else {
                    Branch& s = br[(size_t)small];
                    Branch& l = br[(size_t)large];
                    if (s.is_basic) l.basic.push_back(small);
                    else l.basic.insert(l.basic.end(), s.basic.begin(), s.basic.end());
                    l.n_basic = (int)l.basic.size();
                    l.size += s.size;
                    l.n_merge += 1;
                    s.attach_height = h;
                    s.merged_into = large;
                    merge_to_branch[(size_t)m] = large;
                }
            }
        }
    }
    // clusters: top basic branches that pass size, core scatter and gap
    const int nb = (int)br.size() - 1;
    std::vector<int32_t> colors((size_t)N, 0);
    int color = 0;
    for (int c = 1; c <= nb; ++c) {
        Branch& b = br[(size_t)c];
        if (std::isnan(b.attach_height)) b.attach_height = cut_height;
        if (!b.is_top_basic) continue;
        const double cs = scatter_of(b);
        if (b.size >= min_cluster_size && cs < max_abs_core_scatter && b.attach_height - cs > min_abs_gap) {
            ++color;
            for (int32_t g : b.singletons) colors[(size_t)g - 1] = color;
        }
    }
    // relabel: 0 stays unlabeled, clusters by decreasing size (ties: lower
    // color first — rank(-Sizes, ties.method = "first"))
    std::vector<int64_t> cnt((size_t)color + 1, 0);
    for (int32_t v : colors) cnt[(size_t)v] += 1;
    std::vector<int> ord((size_t)color);
    for (int k = 0; k < color; ++k) ord[(size_t)k] = k + 1;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return cnt[(size_t)a] > cnt[(size_t)b]; });
    std::vector<int32_t> rel((size_t)color + 1, 0);
    for (int k = 0; k < color; ++k) rel[(size_t)ord[(size_t)k]] = k + 1;
    for (int64_t i = 0; i < N; ++i) labels[i] = rel[(size_t)colors[(size_t)i]];
    return SCC_OK;
}

}  // namespace

extern "C" {

SCC_API int scc_hclust_ward_d2(const double* dist, int64_t n, int32_t* merge, double* height, int32_t* order)
{
    if (!dist || !merge || !height || n < 2 || n > (int64_t)INT32_MAX) return SCC_ERR_INVALID;
    const int64_t M = n * (n - 1) / 2;
    for (int64_t k = 0; k < M; ++k)
        if (!std::isfinite(dist[k])) return SCC_ERR_NONFINITE;  // fastcluster: nan_error
    // the symmetric working copy when it is at most 16 GB, else the packed one
    const bool full = (double)n * (double)n * 8.0 <= 16e9;
    try {
        ward_d2(dist, n, merge, height, order, full);
    } catch (const std::bad_alloc&) {
        return SCC_ERR_OOM;
    }
    return SCC_OK;
}

SCC_API int scc_cutree_hybrid(const int32_t* merge, const double* height, int64_t n, const double* dist,
                              int32_t deep_split, int32_t min_cluster_size, int32_t* labels, double* cut_height)
{
    if (!merge || !height || !dist || !labels || n < 2) return SCC_ERR_INVALID;
    std::string err;
    try {
        return cutree_hybrid(merge, height, n, dist, deep_split, min_cluster_size, labels, cut_height, err);
    } catch (const std::bad_alloc&) {
        return SCC_ERR_OOM;
    }
}

}  // extern "C"
