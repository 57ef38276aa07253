"""Config E's CSR -> CSC dataset build, timed alone (wall, synchronised) over
a few repeats; run under `rocprofv3 --kernel-trace --stats` for the per-kernel
split (k_ct_*), or `--pmc FETCH_SIZE` / `WRITE_SIZE` for its traffic."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import synth  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "E"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    d = synth.generate_device(cfg, "cuda:0", seed=synth.CONFIGS[cfg]["seed"], layout="csr")
    torch.cuda.synchronize()
    eng = nat.Engine(0)
    for i in range(reps):
        eng.synchronize()
        t0 = time.perf_counter()
        ds = eng.dataset_csr_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
        eng.synchronize()
        print(f"build {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms (G={d.G} N={d.N} nnz={d.nnz})", flush=True)
        ds.close()
    eng.close()


if __name__ == "__main__":
    main()
