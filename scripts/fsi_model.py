"""numpy model of the eigen stage's filtered subspace iteration (the schedule
k_fsi_engine runs, scconsensus_amd/csrc/scc_subspace.hip:466-485) on the PCA
Gram of a bench configuration, to ask how the block WIDTH changes the work:
for each width w the smallest (segments x degree) schedule whose Rayleigh-Ritz
result passes the engine's residual bar (every |C u - theta u| <= 1e-11
theta_1), and the spectrum ratio that sets the filter's rate.

Per segment: W = C Q, b = max(b_prev, min_j q_j.w_j / q_j.q_j), then the
degree-m Chebyshev recurrence on [0, b] (Y1 = (2/b) W - Q, Y_{t+1} =
(4/b) C Y_t - 2 Y_t - Y_{t-1}), Q = orth(Y_m); m products a segment.  Start
block: k_si_init's hash (scc_subspace.hip:203-216), the first w of its 64
columns.  Usage: python scripts/fsi_model.py [config=B]"""
import sys

import numpy as np

sys.path.insert(0, "oracle")
sys.path.insert(1, ".")
import oracle as O  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402


def start_block(n, w):
    e = np.arange(n * 64, dtype=np.uint64)
    h = (e * np.uint64(2654435761) & np.uint64(0xffffffff)) ^ np.uint64(0x9e3779b9)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0x5bd1e995)) & np.uint64(0xffffffff)
    h ^= h >> np.uint64(15)
    V = ((h & np.uint64(0xffffff)).astype(np.float64) / 16777216.0 - 0.5).reshape(n, 64)
    return V[:, :w]


def orth(Y):
    return np.linalg.qr(Y)[0]


def fsi(C, w, S, m, k=15):
    Q = orth(start_block(C.shape[0], w))
    b_prev = 0.0
    for _ in range(S):
        W = C @ Q
        b = max(b_prev, float(np.min(np.einsum("ij,ij->j", Q, W) / np.einsum("ij,ij->j", Q, Q))))
        b_prev = b
        y0, y1 = Q, (2.0 / b) * W - Q
        for _ in range(m - 1):
            y0, y1 = y1, (4.0 / b) * (C @ y1) - 2.0 * y1 - y0
        Q = orth(y1)
    th, Y = np.linalg.eigh(Q.T @ C @ Q)
    th, Y = th[::-1][:k], Y[:, ::-1][:, :k]
    U = Q @ Y
    res = np.linalg.norm(C @ U - U * th, axis=0).max() / abs(th[0])
    return res, b_prev


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
    d = synth.generate(cfg)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    o = O.de_fast(X, code, len(names))
    Xu = X[o.union].T
    Xc = Xu - Xu.mean(axis=0, keepdims=True)
    C = Xc.T @ Xc
    lam = np.linalg.eigvalsh(C)[::-1]
    print(f"config {cfg}: |U| = {C.shape[0]}; lambda_16/lambda_15 = {lam[15] / lam[14]:.3f}")
    for w in (24, 32, 48, 64):
        print(f"width {w}: lambda_{w + 1}/lambda_15 = {lam[w] / lam[14]:.3f}")
        for total in range(16, 161, 8):
            best = None
            for m in range(4, 17):
                if total % m:
                    continue
                S = total // m
                res, b = fsi(C, w, S, m)
                if res <= 1e-11:
                    best = (S, m, res)
                    break
            if best:
                print(f"  passes at {total} products: {best[0]} x {best[1]}, residual {best[2]:.2e}")
                break
        else:
            print("  no schedule <= 160 products passes")
    for S, m in ((5, 8), (5, 7), (4, 9)):  # the engine's measured sweep at width 64 (r05_eigen_b.md)
        print(f"width 64, {S} x {m}: residual {fsi(C, 64, S, m)[0]:.2e}")


if __name__ == "__main__":
    main()
