"""Test infrastructure: every (gene, cluster pair)'s Wilcoxon 2U and tie term
at full size, computed independently of the engine in plain torch on the GPU
(a global sort and prefix counts -- no buckets, no splits, no wave kernels),
so the large configurations' rank sums are checked on EVERY tested row, not
only on the oracle's gene sample (R/reclusterDEConsensusFast.R:78-91: the
rank sums wilcox.test computes for each tested feature).

For a gene g and clusters a < b over all cells of a and b (zeros included):
  2U_ab = 2 #(x_a > x_b) + #(x_a = x_b)
        = 2 S_ab + 2 pos_a z_b + z_a z_b + E_ab
  S_ab  = sum over stored a-values of the stored b-values strictly below
  E_ab  = sum over tie groups of stored values of t_a t_b
  T_ab  = sum over the tie groups of the pair's sample of t^3 - t
        = F_a + F_b + 3 (Y_ab + Y_ba) + (z_a + z_b)^3 - (z_a + z_b)
  F_a   = sum over groups (t_a^3 - t_a),  Y_ab = sum over groups t_a^2 t_b
(pos: stored values, all > 0 here; z = cluster size - pos).  Every sum is an
exact integer (int64).

Also `packed_max_err`: the max error over EVERY entry of a packed `dist`
vector against fp64 values formed block by block on the GPU (the large
configurations' distances, checked in full rather than sampled)."""
import time

import torch


def pair_stats(indptr, cols, vals, code, K, max_chunk=16 << 20):
    """indptr [G+1] (int64), cols [nnz] (cells), vals [nnz] (> 0): a gene-major
    CSR on the GPU; code [N] cluster of each cell (-1: none).  Returns int64
    tensors u2 [G, P] and ties [G, P] (P = K (K-1) / 2, pairs in (i, j) order)
    on the GPU."""
    dev = vals.device
    G = indptr.numel() - 1
    code = torch.as_tensor(code, device=dev, dtype=torch.int64)
    n = torch.bincount(code[code >= 0], minlength=K).to(torch.int64)
    ia, ib = torch.triu_indices(K, K, offset=1, device=dev)
    P = ia.numel()
    u2 = torch.empty((G, P), dtype=torch.int64, device=dev)
    ties = torch.empty((G, P), dtype=torch.int64, device=dev)
    ip = indptr.to(torch.int64)
    ip_h = ip.cpu()
    g0, tick = 0, time.perf_counter()
    while g0 < G:
        if time.perf_counter() - tick > 30:  # progress for long GPU runs
            print(f"[torch_ranksum] gene {g0} / {G}", flush=True)
            tick = time.perf_counter()
        g1 = g0 + 1  # genes [g0, g1): at most max_chunk stored values (at least one gene)
        while g1 < G and int(ip_h[g1 + 1] - ip_h[g0]) <= max_chunk:
            g1 += 1
        e0, e1 = int(ip_h[g0]), int(ip_h[g1])
        ng = g1 - g0
        cnt = (ip[g0 + 1:g1 + 1] - ip[g0:g1])
        gene = torch.repeat_interleave(torch.arange(ng, device=dev), cnt)
        cl = code[cols[e0:e1].to(torch.int64)]
        v = vals[e0:e1]
        keep = cl >= 0
        gene, cl, v = gene[keep], cl[keep], v[keep]
        assert bool((v > 0).all()), "the checker assumes stored values > 0 (log-normalised data)"
        # order by (gene, value): stable sorts, value first
        o = torch.sort(v, stable=True).indices
        gene, cl, v = gene[o], cl[o], v[o]
        o = torch.sort(gene, stable=True).indices
        gene, cl, v = gene[o], cl[o], v[o]
        m = v.numel()
        # cluster-major [K, *] layouts: every scan runs along the contiguous axis
        Sg = torch.zeros((K, ng * K), dtype=torch.int64, device=dev)   # [b, g K + a]
        Eg = torch.zeros((K, ng * K), dtype=torch.int64, device=dev)
        Yg = torch.zeros((K, ng * K), dtype=torch.int64, device=dev)
        Fg = torch.zeros((K, ng), dtype=torch.int64, device=dev)
        pos = torch.zeros((ng, K), dtype=torch.int64, device=dev)
        if m:
            newgene = torch.ones(m, dtype=torch.bool, device=dev)
            newgene[1:] = gene[1:] != gene[:-1]
            newgrp = newgene.clone()
            newgrp[1:] |= v[1:] != v[:-1]
            grp = torch.cumsum(newgrp.to(torch.int64), 0) - 1
            gstart = torch.nonzero(newgrp).flatten()          # first entry of each tie group
            gbeg = torch.nonzero(newgene).flatten()           # first entry of each gene
            gene_first = gbeg[torch.cumsum(newgene.to(torch.int64), 0) - 1]
            onehot = (cl.view(1, -1) == torch.arange(K, device=dev).view(-1, 1)).to(torch.int64)  # [K, m]
            excl = torch.cumsum(onehot, 1) - onehot            # values before each entry (all genes)
            below = excl[:, gstart[grp]] - excl[:, gene_first]  # of its gene, strictly below its group
            del excl
            key = gene * K + cl
            Sg.index_add_(1, key, below)
            del below
            pos.view(-1).index_add_(0, key, torch.ones_like(key))
            # tie groups (counts per cluster), only where a group holds >= 2 values
            ng_grp = gstart.numel()
            gsize = torch.bincount(grp, minlength=ng_grp)
            tied = gsize[grp] >= 2
            if bool(tied.any()):
                Cg = torch.zeros((K, ng_grp), dtype=torch.int64, device=dev)
                Cg.index_add_(1, grp[tied], onehot[:, tied])
                rows = Cg[:, grp[tied]]                         # the group's counts, at each of its values
                Eg.index_add_(1, key[tied], rows)               # sum_groups t_a t_b
                ta = rows.gather(0, cl[tied].view(1, -1))       # t_a of the value's own cluster
                Yg.index_add_(1, key[tied], ta * rows)          # sum_groups t_a^2 t_b
                ggrp = gene[gstart]                             # gene of each group
                Fg.index_add_(1, ggrp, Cg * Cg * Cg - Cg)
        Sg = Sg.view(K, ng, K).permute(1, 2, 0)                 # [g, a, b]
        Eg = Eg.view(K, ng, K).permute(1, 2, 0)
        Y = Yg.view(K, ng, K).permute(1, 2, 0)
        Fg = Fg.T
        S = Sg[:, ia, ib]
        E = Eg[:, ia, ib]
        X = Y[:, ia, ib] + Y[:, ib, ia]
        za = n[ia].view(1, -1) - pos[:, ia]
        zb = n[ib].view(1, -1) - pos[:, ib]
        u2[g0:g1] = 2 * S + 2 * pos[:, ia] * zb + za * zb + E
        zs = za + zb
        ties[g0:g1] = Fg[:, ia] + Fg[:, ib] + 3 * X + zs * zs * zs - zs
        g0 = g1
    return u2, ties


def packed_max_err(out, block_fn, N, cols=256):
    """Max |out - want| over EVERY entry of a packed `dist` vector on the GPU
    (R's column-major lower triangle: column j holds rows j+1 .. N-1).
    block_fn(j0, j1) returns the [j1 - j0, N] fp64 block of wanted values
    (row r = column j0 + r against every cell); only its entries below the
    diagonal are compared, in packed order."""
    dev = out.device
    ar = torch.arange(N, device=dev)
    worst = 0.0
    for j0 in range(0, N - 1, cols):
        j1 = min(N - 1, j0 + cols)
        lo = j0 * (2 * N - j0 - 1) // 2
        hi = j1 * (2 * N - j1 - 1) // 2
        want = block_fn(j0, j1)
        mask = ar.view(1, -1) > (j0 + torch.arange(j1 - j0, device=dev)).view(-1, 1)
        got = out[lo:hi].to(torch.float64)
        e = (got - want[mask]).abs()
        m = float(e.max())
        if m > worst and m > 1e-5 and worst <= 1e-5:  # the first bad block: where (diagnostics)
            k = int(e.argmax())
            print(f"[packed_max_err] columns {j0}..{j1}: entry {lo + k} off by {m:.3g} "
                  f"(got {float(got[k]):.6g}, want {float(want[mask][k]):.6g})", flush=True)
        worst = max(worst, m)
    return worst


def euclid_block(St):
    """block_fn for packed_max_err: Euclidean distances of the score rows
    j0 .. j1-1 to every row, summed component by component in fp64 (no
    matrix-product shortcut)."""
    def fn(j0, j1):
        acc = None
        for q in range(St.shape[1]):
            d = St[j0:j1, q].view(-1, 1) - St[:, q].view(1, -1)
            acc = d * d if acc is None else acc + d * d
        return torch.sqrt(acc)
    return fn
