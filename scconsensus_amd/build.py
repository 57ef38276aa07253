"""Build ``scconsensus_amd/lib/libscc.so`` in-tree for gfx950 with hipcc.

Every translation unit under ``csrc/`` is compiled separately (in parallel,
only when its sources changed) and linked into one C-ABI shared library whose
exported symbols are exactly those declared in ``include/scc.h``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(HERE, "lib", "libscc.so")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("SCC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
    "-fvisibility=hidden", "-Wno-unused-result", "-Wno-unused-value", f"-I{INCLUDE}", f"-I{CSRC}",
]
LDFLAGS = ["-shared", f"--offload-arch={ARCH}"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def _needs(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if _needs(obj, [src] + _headers()):
        cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
        if src.endswith(".cpp"):
            cmd = [HIPCC] + CFLAGS + ["-x", "hip", "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if _needs(LIB, objs):
        cmd = [HIPCC] + objs + LDFLAGS + ["-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
