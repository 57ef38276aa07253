"""CPU checks of tests/sbr_model.py, the numpy model of the opt-in two-stage
eigen-reduction (scconsensus_amd/csrc/scc_sbr.hip): the band after stage 1,
the tridiagonal after stage 2 and the back-transformed eigenvectors against
numpy's eigh, including a rank-deficient matrix (zero-norm reflectors)."""
import numpy as np
import pytest

import sbr_model as S


def _sym(n, seed, rank=None):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, rank or n))
    return X @ X.T


@pytest.mark.parametrize("n,b", [(20, 4), (37, 8), (64, 16), (50, 8)])
def test_band_tridiagonal_and_vectors(n, b):
    A = _sym(n, n + b)
    band, panels = S.stage1(A, b)
    # stage 1 is an orthogonal similarity to a band of width b
    assert np.max(np.abs(np.tril(band, -b - 1))) < 1e-12 * np.abs(A).max()
    np.testing.assert_allclose(np.linalg.eigvalsh(band), np.linalg.eigvalsh(A), rtol=0, atol=1e-10 * np.abs(A).max())
    d, e, refl, T = S.stage2(band, b)
    assert np.max(np.abs(np.tril(T, -2))) < 1e-12 * np.abs(A).max()
    Tm = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    w, z = np.linalg.eigh(Tm)
    np.testing.assert_allclose(w, np.linalg.eigvalsh(A), rtol=0, atol=1e-10 * np.abs(A).max())
    x = S.back_transform(z[:, -15:], panels, refl)
    # A x = lambda x for the top eigenvectors
    res = A @ x - x * w[-15:]
    assert np.max(np.abs(res)) < 1e-9 * np.abs(A).max()


def test_rank_deficient_panels():
    A = np.zeros((40, 40))
    A[:12, :12] = _sym(12, 3, rank=6)  # genes 12.. identically zero: zero-norm panel columns
    band, panels = S.stage1(A, 8)
    assert any(np.any(np.diag(T) == 0.0) for _, _, T in panels)  # identity reflectors (tau = 0)
    d, e, refl, _ = S.stage2(band, 8)
    Tm = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    np.testing.assert_allclose(np.linalg.eigvalsh(Tm), np.linalg.eigvalsh(A), rtol=0, atol=1e-9 * np.abs(A).max())
