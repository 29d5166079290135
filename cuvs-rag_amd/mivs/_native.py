"""ctypes binding of libmivs.so (the C-ABI declared in include/mivs.h).

This module is the only place Python touches the native library. It loads the
in-tree ``libmivs.so`` (built by ``__graft_entry__.build()`` /
``make -C cuvs-rag_amd/csrc``) and fails LOUDLY when it is missing: there is no
CPU or PyTorch fallback for any ANN operation.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_double, c_float, c_int32, c_int64, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MIVS_LIB", os.path.join(_HERE, "libmivs.so"))

MIVS_OK = 0
MIVS_ERR_INVALID = 1
MIVS_ERR_OOM = 2
MIVS_ERR_HIP = 3
MIVS_ERR_UNSUPPORTED = 4

METRIC_L2 = 0
METRIC_IP = 1
MAX_K = 4096  # include/mivs.h MIVS_MAX_K


class MivsError(RuntimeError):
    """Error raised by the native engine (carries the MIVS_ERR_* code)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


class MivsOutOfMemoryError(MivsError, MemoryError):
    """hipErrorOutOfMemory inside the engine (the reference's OOM paths catch MemoryError/RuntimeError)."""


class NativeLibraryMissing(ImportError):
    pass


class IvfFlatParams(ctypes.Structure):
    _fields_ = [
        ("n_lists", c_int32),
        ("metric", c_int32),
        ("kmeans_n_iters", c_int32),
        ("kmeans_trainset_fraction", c_double),
        ("kmeans_max_train_per_list", c_int64),
        ("add_data_on_build", c_int32),
        ("chunk_rows", c_int32),
        ("kmeans_balance", c_int32),
        ("prefilter", c_int32),
    ]


class IvfPqParams(ctypes.Structure):
    """include/mivs.h mivs_ivf_pq_params."""
    _fields_ = [
        ("n_lists", c_int32),
        ("metric", c_int32),
        ("kmeans_n_iters", c_int32),
        ("kmeans_trainset_fraction", c_double),
        ("pq_dim", c_int32),
        ("pq_bits", c_int32),
        ("max_train_points_per_pq_code", c_int64),
        ("kmeans_balance", c_int32),
        ("add_data_on_build", c_int32),
    ]


class SearchStats(ctypes.Structure):
    _fields_ = [
        ("n_queries", c_int64),
        ("n_probes", c_int32),
        ("k", c_int32),
        ("scanned_rows", c_int64),
        ("streamed_groups", c_int64),
        ("work_items", c_int64),
        ("query_tile", c_int32),
        ("kcap", c_int32),
        ("prefilter", c_int32),
        ("overflow_queries", c_int64),
        ("window_candidates", c_int64),
        ("unique_groups", c_int64),
        ("scan_kernel", c_int32),
        ("candidates", c_int64),
        ("cand_overflow", c_int64),
        ("spun_out_waves", c_int64),
        ("copies_skipped", c_int32),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class IndexMemory(ctypes.Structure):
    _fields_ = [
        ("n_rows", c_int64),
        ("rows_bytes", c_int64),
        ("side_bytes", c_int64),
        ("centroid_bytes", c_int64),
        ("fp16_bytes", c_int64),
        ("fp8_bytes", c_int64),
        ("pq_bytes", c_int64),
        ("total_bytes", c_int64),
        ("copies_skipped", c_int32),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class Profile(ctypes.Structure):
    _fields_ = [
        ("n_calls", c_int32),
        ("coarse_ms", c_float),
        ("scan_ms", c_float),
        ("scan_ms_min", c_float),
        ("scan_ms_max", c_float),
        ("total_ms", c_float),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class BuildKernel(ctypes.Structure):
    """mivs_build_kernel (include/mivs.h): one hot kernel kind of an ivf_flat build, profiled"""
    _fields_ = [("kind", c_int32), ("calls", c_int32), ("ms", ctypes.c_double), ("work", ctypes.c_double)]


# kinds of mivs_index_build_kernels: (name, unit of `work`)
BUILD_KERNELS = (("kmeans_assign", "flop"), ("final_assign", "flop"), ("kmeans_update", "byte"), ("pack", "byte"),
                 ("fp16_copy", "byte"), ("fp8_copy", "byte"))


_SIGS = {
    "mivs_last_error": (ctypes.c_char_p, []),
    "mivs_version": (c_int32, []),
    "mivs_set_profiling": (None, [c_int32]),
    "mivs_ivf_flat_build": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, POINTER(IvfFlatParams), c_int64,
                                      POINTER(c_void_p)]),
    "mivs_ivf_flat_build_from_centroids": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int32,
                                                     c_int32, c_int64, c_int32, POINTER(c_void_p)]),
    "mivs_ivf_flat_build_from_lists": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                                 c_void_p, c_int32, c_int32, c_int32, c_int32, POINTER(c_void_p)]),
    "mivs_ivf_flat_extend": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64]),
    "mivs_ivf_flat_search": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p,
                                       c_void_p]),
    "mivs_ivf_flat_get_centroids": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "mivs_ivf_flat_get_list_sizes": (c_int32, [c_void_p, c_void_p]),
    "mivs_ivf_flat_get_list_ids": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "mivs_ivf_flat_get_list_rows": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "mivs_ivf_pq_build": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, POINTER(IvfPqParams), c_int64,
                                    POINTER(c_void_p)]),
    "mivs_ivf_pq_search": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p,
                                     c_void_p]),
    "mivs_ivf_pq_search_ex": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p,
                                        c_void_p, c_void_p]),
    "mivs_ivf_pq_info": (c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "mivs_ivf_pq_get_codebooks": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "mivs_ivf_pq_get_codes": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "mivs_brute_force_build": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int64,
                                         POINTER(c_void_p)]),
    "mivs_brute_force_search": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    "mivs_index_info": (c_int32, [c_void_p, POINTER(c_int64), POINTER(c_int32), POINTER(c_int32), POINTER(c_int32),
                                  POINTER(c_int32)]),
    "mivs_index_last_search_stats": (c_int32, [c_void_p, POINTER(SearchStats)]),
    "mivs_index_memory_info": (c_int32, [c_void_p, POINTER(IndexMemory)]),
    "mivs_index_profile_collect": (c_int32, [c_void_p, POINTER(Profile)]),
    "mivs_index_build_phases": (c_int32, [c_void_p, c_void_p, c_int32, POINTER(c_int32)]),
    "mivs_index_build_kernels": (c_int32, [c_void_p, POINTER(BuildKernel), c_int32, POINTER(c_int32)]),
    "mivs_index_set_prefilter": (c_int32, [c_void_p, c_void_p, c_int32]),
    "mivs_index_get_prefilter": (c_int32, [c_void_p, POINTER(c_int32)]),
    "mivs_index_free": (None, [c_void_p]),
    "mivs_set_block_cache_limit": (c_int32, [c_int32, c_int64]),
    "mivs_release_cached_memory": (c_int32, [c_int32, POINTER(c_int64)]),
    "mivs_cached_memory": (c_int32, [c_int32, POINTER(c_int64), POINTER(c_int64)]),
    "mivs_reload_settings": (None, []),
    "mivs_kmeans_fit": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32, c_int32,
                                  c_void_p]),
    "mivs_kmeans_predict": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int32, c_int32,
                                      c_void_p]),
    "mivs_kmeans_steps": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32,
                                    c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "mivs_merge_topk": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                  c_void_p, c_void_p]),
    "mivs_merge_topk_gathered": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_int64, c_int32, c_int32,
                                           c_int32, c_void_p, c_void_p]),
    "mivs_comm_init_all": (c_int32, [c_int32, POINTER(c_int32), POINTER(c_void_p)]),
    "mivs_comm_size": (c_int32, [c_void_p, POINTER(c_int32)]),
    "mivs_merge_topk_allgather": (c_int32, [c_void_p, POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p), c_int64,
                                            c_int32, c_int32, c_int32, POINTER(c_void_p), POINTER(c_void_p)]),
    "mivs_comm_destroy": (None, [c_void_p]),
    "mivs_refine": (c_int32, [c_int32, c_void_p, c_void_p, c_int32, c_int64, c_int32, c_void_p, c_int64, c_void_p,
                              c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "mivs_row_norms": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p]),
    "mivs_normalize_rows": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int32, c_void_p]),
    "mivs_synth_mixture": (c_int32, [c_int32, c_void_p, c_void_p, c_int64, c_int64, c_int32, c_uint64, c_int32,
                                     c_float, c_int32]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None
_lock = threading.Lock()
_load_error: str | None = None


def load(path: str | None = None):
    """Load libmivs.so (idempotent). Raises NativeLibraryMissing if it cannot be loaded."""
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            _load_error = f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            raise NativeLibraryMissing(_load_error)
        try:
            lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the ROCm runtime install
            _load_error = f"cannot load {p}: {e}"
            raise NativeLibraryMissing(_load_error) from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def available() -> bool:
    try:
        load()
        return True
    except NativeLibraryMissing:
        return False


def lib():
    return load()


def check(rc: int) -> None:
    if rc == MIVS_OK:
        return
    msg = load().mivs_last_error().decode(errors="replace")
    if rc == MIVS_ERR_OOM:
        raise MivsOutOfMemoryError(rc, msg)
    if rc in (MIVS_ERR_INVALID, MIVS_ERR_UNSUPPORTED):
        raise ValueError(msg)
    raise MivsError(rc, msg)


_PROFILING = False


def set_profiling(on: bool) -> None:
    global _PROFILING
    _PROFILING = bool(on)
    load().mivs_set_profiling(1 if on else 0)


def profiling() -> bool:
    """Whether set_profiling(True) is in effect (build phase clocks, search hipEvents)."""
    return _PROFILING


BUILD_PHASES = {0: ("prepare", "coarse_kmeans", "assign_pack", "fp16_copy"),
                2: ("prepare", "coarse_kmeans", "assign_sort", "codebooks", "encode")}


def build_kernels(handle) -> dict:
    """{kind: {calls, ms, work, unit}} of an ivf_flat build's hot kernels (device time by hipEvents; recorded only while
    profiling was on during the build)"""
    n_max = len(BUILD_KERNELS)
    buf = (BuildKernel * n_max)()
    n = c_int32(0)
    check(lib().mivs_index_build_kernels(handle, buf, n_max, ctypes.byref(n)))
    return {BUILD_KERNELS[i][0]: {"calls": int(buf[i].calls), "ms": float(buf[i].ms), "work": float(buf[i].work),
                                  "unit": BUILD_KERNELS[i][1]} for i in range(min(n.value, n_max))}


def build_phases(handle, kind: int) -> dict:
    """{phase: seconds} of an index's build (recorded only while profiling was on)."""
    import ctypes

    buf = (ctypes.c_double * 16)()
    n = c_int32(0)
    check(lib().mivs_index_build_phases(handle, buf, 16, ctypes.byref(n)))
    names = BUILD_PHASES.get(kind, ())
    return {(names[i] if i < len(names) else f"phase{i}"): round(buf[i], 4) for i in range(min(n.value, 16))}


def set_block_cache_limit(bytes_: int, device: int = -1) -> None:
    """Let the engine keep up to `bytes_` of released large device blocks per device for reuse (0: off, the default;
    device -1: every device). Lowering it frees the blocks above the new limit."""
    check(lib().mivs_set_block_cache_limit(int(device), int(bytes_)))


def release_cached_memory(device: int = -1) -> int:
    """Return every block the engine's block cache holds on `device` (-1: all devices) to the driver; bytes freed.
    Called by the drop-ins' cleanup and OOM paths before torch.cuda.empty_cache()."""
    if _lib is None:  # nothing loaded: nothing cached
        return 0
    freed = c_int64(0)
    check(_lib.mivs_release_cached_memory(int(device), ctypes.byref(freed)))
    return int(freed.value)


def cached_memory(device: int = -1) -> dict:
    """{"bytes": cached, "limit": per-device limit (-1 for device -1)}"""
    b, lim = c_int64(0), c_int64(0)
    check(lib().mivs_cached_memory(int(device), ctypes.byref(b), ctypes.byref(lim)))
    return {"bytes": int(b.value), "limit": int(lim.value)}


def reload_settings() -> None:
    """Re-read the engine settings the library caches from the environment (MIVS_FALLBACK_SYNC)."""
    if _lib is not None:
        _lib.mivs_reload_settings()
