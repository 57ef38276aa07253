"""Launch the FSI's one-workgroup kernels alone (for rocprofv3 --kernel-trace
--stats): k_small_syev on a 64 x 64 SPD matrix and k_fsi_cholinv64 on a
condition-1e6 Gram, 20 times each."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scconsensus_amd import _native as nat  # noqa: E402

L = nat.load()
rng = np.random.default_rng(0)
A = rng.standard_normal((64, 64))
H = torch.tensor(A @ A.T, dtype=torch.float64, device="cuda:0")
U, _ = np.linalg.qr(rng.standard_normal((64, 64)))
G = torch.tensor((U * np.logspace(0, 6, 64)) @ U.T, dtype=torch.float64, device="cuda:0")
Y = torch.zeros(64 * 16, dtype=torch.float64, device="cuda:0")
th = torch.zeros(16, dtype=torch.float64, device="cuda:0")
T = torch.zeros(64 * 64, dtype=torch.float64, device="cuda:0")
fl = torch.zeros(4, dtype=torch.int32, device="cuda:0")
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
for _ in range(20):
    assert L.scc_diag_small_syev(p(H), 64, 64, 15, p(Y), p(th), p(fl)) == 0
for _ in range(20):
    assert L.scc_diag_cholinv(p(G), 64, 3e-11, p(T), p(fl)) == 0
print("flag", int(fl[0]))
st = (ctypes.c_ulonglong * 8)()
assert L.scc_diag_small_syev(p(H), 64, 64, 15, p(Y), p(th), p(fl)) == 0
L.scc_diag_small_syev_stamps(st)
names = ["tridiag", "gershgorin", "bisection", "inverse-iteration", "gram-schmidt+RQ", "back-transform"]
print("k_small_syev phases (s_memtime ticks, 100 MHz):", {nm: st[i + 1] - st[i] for i, nm in enumerate(names)})
