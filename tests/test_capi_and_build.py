"""The drop-in boundary: libmivs.so loads on CPU and exports every entry point include/mivs.h declares.

No compute calls here (no GPU in the build container); -m gpu tests exercise them.
"""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mivs.h")
LIB = os.path.join(ROOT, "cuvs-rag_amd", "mivs", "libmivs.so")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mivs_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_hot_path_entry_points():
    fns = header_functions()
    for required in ("mivs_ivf_flat_build", "mivs_ivf_flat_search", "mivs_brute_force_build",
                     "mivs_brute_force_search", "mivs_kmeans_fit", "mivs_kmeans_steps", "mivs_merge_topk", "mivs_index_free",
                     "mivs_last_error"):
        assert required in fns


def test_library_exports_every_declared_symbol(mivs_lib):
    lib = ctypes.CDLL(LIB)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, f"libmivs.so lacks {missing}"


def test_python_binding_covers_the_header():
    from mivs import _native

    assert set(header_functions()) == set(_native.EXPORTED_SYMBOLS)


def test_library_is_built_for_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", LIB], capture_output=True,
                         text=True)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_missing_library_fails_loudly(tmp_path):
    code = ("import sys; sys.path.insert(0, %r); import mivs._native as n; "
            "n.LIB_PATH = %r\ntry:\n    n.load()\nexcept n.NativeLibraryMissing as e:\n    print('LOUD', e)\n")
    r = subprocess.run([sys.executable, "-c", code % (os.path.join(ROOT, "cuvs-rag_amd"),
                                                      str(tmp_path / "nope.so"))], capture_output=True, text=True)
    assert "LOUD" in r.stdout


def test_version_and_error_channel(mivs_lib):
    from mivs import _native

    lib = _native.lib()
    assert lib.mivs_version() >= 100
    h = ctypes.c_void_p()
    rc = lib.mivs_brute_force_build(0, None, None, 10, 0, 0, 0, ctypes.byref(h))  # invalid dim -> no GPU work
    assert rc != 0 and lib.mivs_last_error()
