"""numpy model of the engine's two-stage symmetric eigen-reduction
(scconsensus_amd/csrc/scc_sbr.hip), step for step, for the CPU tests.

Stage 1 (dense -> band of width b): panel k (columns [c0, c0 + b), c0 = k b)
is QR-factored below the band, P = A[c0+b:, c0:c0+b] = Q R with
Q = I - V T V^T (Householder, LAPACK dgeqrf/dlarft order), and the trailing
matrix is updated two-sidedly, A22 <- Q^T A22 Q = A22 - V W^T - W V^T with
Y = A22 V T, M = T^T V^T Y, W = Y - V M / 2.
Stage 2 (band -> tridiagonal, bulge chasing): sweep j annihilates column j
below the subdiagonal with a reflector on rows [j+1, j+b]; the right
application to the rows below creates a bulge whose first column is
annihilated by the next reflector, and so on down the band.
Eigenvectors: x = Q1 (Q2 z) for an eigenvector z of the tridiagonal.
"""
import numpy as np


def house(x):
    """LAPACK dlarfg: H = I - tau v v^T with v[0] = 1, H x = beta e_1."""
    alpha = x[0]
    xn2 = float(np.dot(x[1:], x[1:]))
    v = np.zeros_like(x)
    v[0] = 1.0
    if xn2 == 0.0:
        return v, 0.0, alpha
    beta = -np.copysign(np.sqrt(alpha * alpha + xn2), alpha)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def stage1(A, b):
    """Dense symmetric A (n x n) -> band of width b.  Returns (band matrix,
    list of panels (row0, V, T))."""
    A = np.array(A, dtype=np.float64, copy=True)
    n = A.shape[0]
    panels = []
    c0 = 0
    while c0 + b < n - 1 or (c0 + b < n and n - c0 - b > 1):
        r0 = c0 + b
        m = n - r0
        nr = min(m, b)
        P = A[r0:, c0:c0 + b].copy()
        V = np.zeros((m, nr))
        taus = np.zeros(nr)
        for t in range(nr):
            v, tau, beta = house(P[t:, t])
            V[t:, t] = v
            taus[t] = tau
            # apply H from the left to the panel's remaining columns
            w = v @ P[t:, t:]
            P[t:, t:] -= tau * np.outer(v, w)
        # T (dlarft forward, columnwise)
        T = np.zeros((nr, nr))
        for t in range(nr):
            T[t, t] = taus[t]
            if t:
                T[:t, t] = -taus[t] * (T[:t, :t] @ (V[:, :t].T @ V[:, t]))
        A[r0:, c0:c0 + b] = P
        A[c0:c0 + b, r0:] = P.T
        A22 = A[r0:, r0:]
        Y = A22 @ V @ T
        M = T.T @ (V.T @ Y)
        W = Y - 0.5 * V @ M
        A[r0:, r0:] = A22 - V @ W.T - W @ V.T
        panels.append((r0, V, T))
        c0 += b
    return A, panels


def stage2(A, b):
    """Band (width b) symmetric -> tridiagonal by bulge chasing.  Returns
    (d, e, reflectors [(row0, v, tau)] in application order)."""
    A = np.array(A, dtype=np.float64, copy=True)
    n = A.shape[0]
    refl = []

    def apply_two_sided(r0, r1, v, tau):
        # rows / cols [r0, r1] of the whole matrix: A <- H A H
        H = np.eye(r1 - r0 + 1) - tau * np.outer(v, v)
        A[r0:r1 + 1, :] = H @ A[r0:r1 + 1, :]
        A[:, r0:r1 + 1] = A[:, r0:r1 + 1] @ H

    for j in range(n - 2):
        p0, p1 = j + 1, min(j + b, n - 1)
        if p1 <= p0:
            continue
        v, tau, beta = house(A[p0:p1 + 1, j].copy())
        apply_two_sided(p0, p1, v, tau)
        refl.append((p0, v, tau))
        while True:
            q0, q1 = p1 + 1, min(p1 + b, n - 1)
            if q1 <= q0:
                break
            v, tau, beta = house(A[q0:q1 + 1, p0].copy())
            apply_two_sided(q0, q1, v, tau)
            refl.append((q0, v, tau))
            p0, p1 = q0, q1
    d = np.diag(A).copy()
    e = np.diag(A, -1).copy()
    return d, e, refl, A


def back_transform(z, panels, refl):
    """x = Q1 Q2 z for the columns of z."""
    x = np.array(z, dtype=np.float64, copy=True)
    for r0, v, tau in reversed(refl):
        x[r0:r0 + len(v)] -= tau * np.outer(v, v @ x[r0:r0 + len(v)])
    for r0, V, T in reversed(panels):
        x[r0:] -= V @ (T @ (V.T @ x[r0:]))
    return x
