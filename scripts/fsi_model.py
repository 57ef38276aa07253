"""numpy model of the engine's Chebyshev-filtered subspace iteration
(csrc/scc_subspace.hip, scc_eigen_fsi) on a PCA Gram: the same schedule
(64-column block, segments of degree m restarted from the orthonormalised
block, the damped interval [0, b] with b the largest seen minimum Rayleigh
quotient of the block's columns, shifted CholQR between segments, Rayleigh-Ritz
at the end) in fp64, reporting per segment the worst Ritz residual / theta_1
and the largest distance error against the exact top-15 subspace on a sample
of cells.

    python scripts/fsi_model.py B            # builds config B's union Gram on the CPU (~2 min)
    python scripts/fsi_model.py path/to/Xu.npy   # cells x |U| matrix of a union
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def union_matrix(cfg):
    import oracle as O
    from scconsensus_amd import api, synth
    d = synth.generate(cfg)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    uni = np.asarray(O.de_fast(X, code, len(names)).union)
    return X[uni, :].T.copy()


def cholqr(Y, passes, shift_rel):
    for p in range(passes):
        G = Y.T @ Y
        if p == 0:
            G = G + shift_rel * np.trace(G) * np.eye(G.shape[0])
        Y = Y @ np.linalg.inv(np.linalg.cholesky(G).T)
    return Y


def main():
    arg = sys.argv[1] if len(sys.argv) > 1 else "B"
    if arg.endswith(".npy"):
        Xu = np.load(arg)
    else:
        Xu = union_matrix(arg)
        if os.environ.get("SAVE"):
            np.save(os.environ["SAVE"], Xu)
    Xc = Xu - Xu.mean(0)
    C = Xc.T @ Xc
    n, p, k = C.shape[0], int(os.environ.get("P", 64)), 15
    S = int(os.environ.get("SEG", 5))
    m = int(os.environ.get("DEG", 8))
    passes = int(os.environ.get("PASSES", 2))
    w, V = np.linalg.eigh(C)
    w, V = w[::-1], V[:, ::-1]
    rng = np.random.default_rng(1)
    idx = rng.choice(Xc.shape[0], min(800, Xc.shape[0]), replace=False)
    Xs = Xc[idx]

    def dist(Sc):
        return np.sqrt(np.maximum(((Sc[:, None, :] - Sc[None, :, :]) ** 2).sum(-1), 0))

    Dref = dist(Xs @ V[:, :k])
    npad = (n + 15) // 16 * 16
    shift_rel = 11.0 * (npad * p + p * (p + 1)) * 1.11e-16
    Q = cholqr(rng.standard_normal((n, p)), 1, shift_rel)
    b = 0.0
    for s in range(S):
        W = C @ Q
        rq = np.sum(Q * W, 0) / np.sum(Q * Q, 0)
        b = max(b, rq.min())
        Y0, Y1 = Q, (2.0 / b) * W - Q
        for _ in range(2, m + 1):
            Y0, Y1 = Y1, (4.0 / b) * (C @ Y1) - 2.0 * Y1 - Y0
        Q = cholqr(Y1, passes if s + 1 < S else 3, shift_rel)
        W = C @ Q
        H = Q.T @ W
        h, Yr = np.linalg.eigh((H + H.T) / 2)
        h, Yr = h[::-1], Yr[:, ::-1]
        Z = Q @ Yr[:, :k]
        res = np.linalg.norm(W @ Yr[:, :k] - Z * h[:k], axis=0).max() / h[0]
        err = np.abs(dist(Xs @ Z) - Dref).max()
        print(f"segment {s + 1}: products {(s + 1) * m}, b/lambda_15 {b / w[k - 1]:.3f}, "
              f"max residual / theta_1 {res:.2e}, max |dist error| {err:.2e}")


if __name__ == "__main__":
    main()
