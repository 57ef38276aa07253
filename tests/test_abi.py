"""CPU: the C-ABI library builds for gfx950, loads, and exports exactly the
symbols include/scc.h declares (no compute call — there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib_path():
    from scconsensus_amd import build
    return build.build()


def _declared():
    hdr = open(os.path.join(ROOT, "include", "scc.h")).read()
    return sorted(set(re.findall(r"^SCC_API [^(]*?\b(scc_\w+)\(", hdr, re.M)))


def test_header_lists_all_entry_points():
    from scconsensus_amd import _native
    assert _declared() == sorted(_native.EXPORTS)


def test_library_exports_every_declared_symbol():
    path = _lib_path()
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (scc_\w+)$", out, re.M))
    assert set(_declared()) == exported


def test_library_loads_and_binds():
    _lib_path()
    from scconsensus_amd import _native
    L = _native.load()
    for name in _native.EXPORTS:
        assert isinstance(getattr(L, name), ctypes._CFuncPtr)


def test_code_object_targets_gfx950():
    path = _lib_path()
    data = open(path, "rb").read()
    assert b".hip_fatbin" in data
    assert b"amdgcn-amd-amdhsa--gfx950" in data
