"""Exact k-NN on MI355X — drop-in for ``cuvs.neighbors.brute_force`` and the search
semantics of FAISS ``IndexFlatL2`` (colab_a100_test.ipynb:433-456; the CPU
``IndexFlat`` of Latest/faiss.ipynb:1051) / sklearn ``NearestNeighbors(brute)``
(VectorSearch_QuestionRetrieval.ipynb:878).

``build`` packs the dataset once into the interleaved 32-row group layout and
precomputes row norms; ``search`` streams it through the same fused MFMA
distance + register top-k scan kernel as IVF-Flat (one list, every query).
"""
from __future__ import annotations

import ctypes

import torch

from .. import _cosine, _native
from .._tensors import as_device_f32, emit, out_tensor, ptr, stream_ptr
from .ivf_flat import _SQRT_METRICS, metric_code


class Index:
    def __init__(self, handle: int, metric: str):
        self._h = ctypes.c_void_p(handle)
        self.metric = metric
        n, d, nl, m, dev = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib().mivs_index_info(self._h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(nl),
                                                    ctypes.byref(m), ctypes.byref(dev)))
        self.size = int(n.value)
        self.dim = int(d.value)
        self.device = int(dev.value)

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("index has been closed")
        return self._h

    def __len__(self):
        return self.size

    @property
    def prefilter(self) -> bool:
        """True when the fp16 copy of the rows is kept: k <= 16 searches then run the fp16 pre-filter
        scan + exact fp32 refine instead of the fp32 scan; results are identical."""
        v = ctypes.c_int32()
        _native.check(_native.lib().mivs_index_get_prefilter(self.handle, ctypes.byref(v)))
        return bool(v.value)

    def set_prefilter(self, enable: bool) -> None:
        """Build (True) or free (False) the fp16 copy of the rows."""
        _native.check(_native.lib().mivs_index_set_prefilter(self.handle, stream_ptr(self.device),
                                                             1 if enable else 0))

    def memory(self) -> dict:
        """Bytes the index holds in HBM by part (mivs_index_memory_info): the fp32 rows, norms / ids / offsets,
        centroids, the fp16 and fp8 copies, PQ codes; copies_skipped = 1 when the fp8 copy was left out (HBM
        budget, MIVS_INDEX_HBM_FRAC)."""
        m = _native.IndexMemory()
        _native.check(_native.lib().mivs_index_memory_info(self.handle, ctypes.byref(m)))
        return m.as_dict()

    def last_search_stats(self) -> dict:
        st = _native.SearchStats()
        _native.check(_native.lib().mivs_index_last_search_stats(self.handle, ctypes.byref(st)))
        return st.as_dict()

    def profile_collect(self) -> dict:
        """Device time of the searches since the last collect (needs mivs._native.set_profiling(True))."""
        pr = _native.Profile()
        _native.check(_native.lib().mivs_index_profile_collect(self.handle, ctypes.byref(pr)))
        return pr.as_dict()

    def close(self):
        if self._h is not None and self._h.value and _native._lib is not None:
            _native._lib.mivs_index_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self):
        return f"brute_force.Index(size={self.size}, dim={self.dim}, metric={self.metric!r}, device=cuda:{self.device})"


def build(dataset, metric: str = "sqeuclidean", metric_arg: float = 2.0, resources=None, ids_offset: int = 0) -> Index:
    x = as_device_f32(dataset, name="dataset")
    if _cosine.is_cosine(metric):
        x = _cosine.normalize_rows(x)
    dev = x.device.index
    h = ctypes.c_void_p()
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_brute_force_build(dev, stream_ptr(dev), ptr(x), x.shape[0], x.shape[1],
                                                           metric_code(metric), int(ids_offset), ctypes.byref(h)))
    return Index(h.value, metric)


def _search(index, queries, k: int, neighbors=None, distances=None):
    """search() without the output hook: torch tensors on the index's device (mivs.neighbors.streaming)."""
    if not isinstance(index, Index):
        raise TypeError("index must be a brute_force.Index")
    k = int(k)
    if k < 1:
        raise ValueError(f"k must be >= 1, got {k}")
    dev = index.device
    q = as_device_f32(queries, device=dev, name="queries")
    if q.shape[1] != index.dim:
        raise ValueError(f"queries have dim {q.shape[1]}, index has {index.dim}")
    cos = _cosine.is_cosine(index.metric)
    if cos:
        q = _cosine.normalize_rows(q)
    nq = q.shape[0]
    dist = out_tensor(distances, (nq, k), torch.float32, dev, "distances")
    nbrs = out_tensor(neighbors, (nq, k), torch.int64, dev, "neighbors")
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_brute_force_search(index.handle, stream_ptr(dev), ptr(q), nq, k, ptr(dist),
                                                            ptr(nbrs)))
    if index.metric in _SQRT_METRICS:
        dist.sqrt_()  # in place: a caller-provided `distances` holds the final values
    if cos:
        _cosine.to_distance_(dist)
    return dist, nbrs


def _emit2(r):
    return emit(r[0]), emit(r[1])


def search(index: Index, queries, k: int, neighbors=None, distances=None, resources=None):
    return _emit2(_search(index, queries, k, neighbors, distances))


def knn(dataset, queries, k: int, metric: str = "sqeuclidean"):
    """One-shot exact k-NN (builds a temporary index)."""
    idx = build(dataset, metric=metric)
    try:
        return search(idx, queries, k)
    finally:
        idx.close()


__all__ = ["Index", "build", "search", "knn"]
