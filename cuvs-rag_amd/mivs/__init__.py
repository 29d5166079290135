"""mivs — MI355X-native IVF-Flat / brute-force k-NN engine (PyTorch-ROCm host, HIP/CDNA4 kernels).

Python mirror of the cuVS modules the reference calls (``cuvs.neighbors.ivf_flat``,
``cuvs.neighbors.brute_force``, ``cuvs.cluster.kmeans``, ``pylibraft.config``); all arithmetic
runs in the in-tree ``libmivs.so`` through the C-ABI of include/mivs.h.
"""
from . import _native, config  # noqa: F401
from ._native import MAX_K, MivsError, MivsOutOfMemoryError, NativeLibraryMissing, available, load  # noqa: F401
from ._native import cached_memory, release_cached_memory, set_block_cache_limit  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing mivs must not require a GPU
    if name in ("neighbors", "cluster", "ops", "distributed", "faiss_io"):
        import importlib

        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
