"""IVF-Flat on MI355X — drop-in for ``cuvs.neighbors.ivf_flat`` (cuVS 25.6.0).

The reference uses exactly these call shapes:
  * ``ivf_flat.IndexParams(n_lists=...)``             index_building_coordinator.py:395
  * ``ivf_flat.build(params, torch_cuda_tensor)``      index_building_coordinator.py:396
  * ``ivf_flat.SearchParams()``                        improved_multi_gpu_rag.py:226
  * ``ivf_flat.search(sp, index, q_2d, k)``            improved_multi_gpu_rag.py:227
    -> ``(distances, neighbors)``

Everything runs in libmivs.so (hand-written HIP for gfx950); this module only
validates arguments and moves pointers. Defaults follow cuVS: 20 k-means
iterations on a 0.5 trainset fraction, 20 probes.
"""
from __future__ import annotations

import ctypes
import math

import torch

from .. import _native
from .. import _cosine
from .._tensors import as_device_f32, emit, out_tensor, ptr, stream_ptr

_METRICS = {
    "sqeuclidean": _native.METRIC_L2,
    "l2": _native.METRIC_L2,
    "L2Expanded": _native.METRIC_L2,
    "euclidean": _native.METRIC_L2,  # same ranking; distances are sqrt'ed on output
    "L2SqrtExpanded": _native.METRIC_L2,
    "inner_product": _native.METRIC_IP,
    "InnerProduct": _native.METRIC_IP,
    "cosine": _native.METRIC_IP,  # over normalised rows, distance 1 - ip (mivs._cosine)
    "CosineExpanded": _native.METRIC_IP,
}
_SQRT_METRICS = ("euclidean", "L2SqrtExpanded")


def metric_code(metric: str) -> int:
    try:
        return _METRICS[metric]
    except KeyError:
        raise ValueError(f"unsupported metric {metric!r}; supported: {sorted(_METRICS)}") from None


class IndexParams:
    """cuvs.neighbors.ivf_flat.IndexParams."""

    def __init__(self, n_lists: int = 1024, metric: str = "sqeuclidean", kmeans_n_iters: int = 20,
                 kmeans_trainset_fraction: float = 0.5, add_data_on_build: bool = True,
                 adaptive_centers: bool = False, conservative_memory_allocation: bool = False,
                 kmeans_max_train_per_list: int = 0, chunk_rows: int = 0, kmeans_balance: bool = True,
                 prefilter: bool = True):
        if int(n_lists) < 1:
            raise ValueError(f"n_lists must be >= 1, got {n_lists}")
        metric_code(metric)
        if adaptive_centers:
            raise NotImplementedError("adaptive_centers is not supported by mivs")
        self.n_lists = int(n_lists)
        self.metric = metric
        self.kmeans_n_iters = int(kmeans_n_iters)
        self.kmeans_trainset_fraction = float(kmeans_trainset_fraction)
        self.add_data_on_build = bool(add_data_on_build)
        self.adaptive_centers = bool(adaptive_centers)
        self.conservative_memory_allocation = bool(conservative_memory_allocation)
        self.kmeans_max_train_per_list = int(kmeans_max_train_per_list)
        self.chunk_rows = int(chunk_rows)
        self.kmeans_balance = bool(kmeans_balance)
        # fp16 copy of the lists for the exact-result fp16 pre-filter search
        self.prefilter = bool(prefilter)

    def _c(self) -> _native.IvfFlatParams:
        return _native.IvfFlatParams(self.n_lists, metric_code(self.metric), self.kmeans_n_iters,
                                     self.kmeans_trainset_fraction, self.kmeans_max_train_per_list,
                                     1 if self.add_data_on_build else 0, self.chunk_rows,
                                     1 if self.kmeans_balance else 0, 1 if self.prefilter else 0)

    def __repr__(self):
        return (f"IndexParams(n_lists={self.n_lists}, metric={self.metric!r}, kmeans_n_iters={self.kmeans_n_iters}, "
                f"kmeans_trainset_fraction={self.kmeans_trainset_fraction})")


class SearchParams:
    """cuvs.neighbors.ivf_flat.SearchParams (cuVS default n_probes = 20)."""

    def __init__(self, n_probes: int = 20):
        if int(n_probes) < 1:
            raise ValueError(f"n_probes must be >= 1, got {n_probes}")
        self.n_probes = int(n_probes)

    def __repr__(self):
        return f"SearchParams(n_probes={self.n_probes})"


class Index:
    """Handle to an IVF-Flat index resident on one GPU (owned by libmivs)."""

    def __init__(self, handle: int, metric: str):
        self._h = ctypes.c_void_p(handle)
        self.metric = metric
        n, d, nl, m, dev = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib().mivs_index_info(self._h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(nl),
                                                    ctypes.byref(m), ctypes.byref(dev)))
        self.size = int(n.value)
        self.dim = int(d.value)
        self.n_lists = int(nl.value)
        self.device = int(dev.value)
        self.trained = True

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("index has been closed")
        return self._h

    def __len__(self):
        return self.size

    @property
    def centers(self) -> torch.Tensor:
        out = torch.empty((self.n_lists, self.dim), dtype=torch.float32, device=f"cuda:{self.device}")
        _native.check(_native.lib().mivs_ivf_flat_get_centroids(self.handle, stream_ptr(self.device), ptr(out)))
        return out

    @property
    def list_sizes(self) -> torch.Tensor:
        out = torch.empty(self.n_lists, dtype=torch.int64)
        _native.check(_native.lib().mivs_ivf_flat_get_list_sizes(self.handle, ptr(out)))
        return out

    def list_ids(self) -> torch.Tensor:
        """ids of all lists concatenated in list order (each list ascending by id)."""
        out = torch.empty(self.size, dtype=torch.int64, device=f"cuda:{self.device}")
        _native.check(_native.lib().mivs_ivf_flat_get_list_ids(self.handle, stream_ptr(self.device), ptr(out)))
        return out

    def list_rows(self) -> torch.Tensor:
        out = torch.empty((self.size, self.dim), dtype=torch.float32, device=f"cuda:{self.device}")
        _native.check(_native.lib().mivs_ivf_flat_get_list_rows(self.handle, stream_ptr(self.device), ptr(out)))
        return out

    @property
    def prefilter(self) -> bool:
        """True when the fp16 copy of the lists is kept for the exact-result pre-filter search."""
        v = ctypes.c_int32()
        _native.check(_native.lib().mivs_index_get_prefilter(self.handle, ctypes.byref(v)))
        return bool(v.value)

    def set_prefilter(self, enable: bool) -> None:
        """Build (True) or free (False) the fp16 copy; search results are identical either way."""
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

    def build_phases(self) -> dict:
        """Host wall time (s) of this index's build phases (recorded only while profiling was on)."""
        ph = _native.build_phases(self.handle, 0)
        if getattr(self, "_to_f32_s", None) is not None:
            ph = {"to_fp32": round(self._to_f32_s, 4), **ph}
        return ph

    def build_kernels(self) -> dict:
        """Device time and algorithmic work of this index's build kernels (recorded only while profiling was on)."""
        return _native.build_kernels(self.handle)

    def profile_collect(self) -> dict:
        """Device time of the searches since the last collect (needs mivs._native.set_profiling(True))."""
        pr = _native.Profile()
        _native.check(_native.lib().mivs_index_profile_collect(self.handle, ctypes.byref(pr)))
        return pr.as_dict()

    def close(self):
        if self._h is not None and self._h.value:
            lib = _native._lib
            if lib is not None:
                lib.mivs_index_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self):
        return (f"ivf_flat.Index(size={self.size}, dim={self.dim}, n_lists={self.n_lists}, metric={self.metric!r}, "
                f"device=cuda:{self.device})")


def build(index_params: IndexParams, dataset, resources=None, ids_offset: int = 0) -> Index:
    """Train k-means, assign every row, fill the inverted lists (all on the GPU holding `dataset`)."""
    if not isinstance(index_params, IndexParams):
        raise TypeError("index_params must be an ivf_flat.IndexParams")
    x = as_device_f32(dataset, name="dataset")
    if _cosine.is_cosine(index_params.metric):
        x = _cosine.normalize_rows(x)
    dev = x.device.index
    n, d = x.shape
    if n < index_params.n_lists:
        raise ValueError(f"dataset has {n} rows, fewer than n_lists={index_params.n_lists}")
    h = ctypes.c_void_p()
    p = index_params._c()
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_ivf_flat_build(dev, stream_ptr(dev), ptr(x), n, d, ctypes.byref(p),
                                                        int(ids_offset), ctypes.byref(h)))
    return Index(h.value, index_params.metric)


def build_from_centroids(centroids, dataset, metric: str = "sqeuclidean", ids_offset: int = 0,
                         chunk_rows: int = 0, prefilter: bool = True) -> Index:
    """IVF-Flat lists from given centroids (FAISS IndexIVFFlat with a pre-trained quantizer)."""
    x = as_device_f32(dataset, name="dataset")
    if _cosine.is_cosine(metric):
        x = _cosine.normalize_rows(x)
    dev = x.device.index
    c = as_device_f32(centroids, device=dev, name="centroids")
    if c.shape[1] != x.shape[1]:
        raise ValueError("centroids and dataset dims differ")
    h = ctypes.c_void_p()
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_ivf_flat_build_from_centroids(
            dev, stream_ptr(dev), ptr(x), x.shape[0], x.shape[1], ptr(c), c.shape[0], metric_code(metric),
            int(ids_offset), int(chunk_rows), ctypes.byref(h)))
    idx = Index(h.value, metric)
    if not prefilter:
        idx.set_prefilter(False)
    return idx


def _search(search_params, index, queries, k: int, neighbors=None, distances=None, probes_out=None):
    """search() without the output hook: torch tensors on the index's device (mivs.neighbors.streaming)."""
    if not isinstance(index, Index):
        raise TypeError("index must be an ivf_flat.Index")
    sp = search_params if search_params is not None else SearchParams()
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
        _native.check(_native.lib().mivs_ivf_flat_search(index.handle, stream_ptr(dev), ptr(q), nq, k, sp.n_probes,
                                                         ptr(dist), ptr(nbrs), ptr(probes_out)))
    if index.metric in _SQRT_METRICS:
        dist.sqrt_()  # in place: a caller-provided `distances` holds the final values
    if cos:
        _cosine.to_distance_(dist)
    return dist, nbrs


def _emit2(r):
    return emit(r[0]), emit(r[1])


def search(search_params: SearchParams, index: Index, queries, k: int, neighbors=None, distances=None,
           resources=None, probes_out: torch.Tensor | None = None):
    """k-NN over the n_probes closest lists. Returns ``(distances, neighbors)`` ([nq, k] f32, [nq, k] i64)."""
    return _emit2(_search(search_params, index, queries, k, neighbors, distances, probes_out))


def extend(index: Index, new_vectors, new_indices=None) -> Index:
    """cuvs.neighbors.ivf_flat.extend: append rows to their nearest lists (the build's assign; each list
    keeps its current rows first). ``new_indices`` None: ids ``ids_offset + len(index) ..
    ids_offset + len(index) + n - 1`` (``ids_offset`` as given to ``build``; 0 for a loaded index), so a
    shard of a sharded corpus keeps its new rows inside its own global id range.
    Returns ``index`` (extended in place)."""
    if not isinstance(index, Index):
        raise TypeError("index must be an ivf_flat.Index")
    dev = index.device
    x = as_device_f32(new_vectors, device=dev, name="new_vectors")
    if x.shape[1] != index.dim:
        raise ValueError(f"new_vectors have dim {x.shape[1]}, index has {index.dim}")
    if _cosine.is_cosine(index.metric):
        x = _cosine.normalize_rows(x)
    ids = None
    if new_indices is not None:
        ids = torch.as_tensor(new_indices).to(device=f"cuda:{dev}", dtype=torch.int64).contiguous().reshape(-1)
        if ids.numel() != x.shape[0]:
            raise ValueError(f"new_indices has {ids.numel()} entries, new_vectors {x.shape[0]} rows")
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_ivf_flat_extend(index.handle, stream_ptr(dev), ptr(x), ptr(ids), x.shape[0]))
    index.size += int(x.shape[0])
    return index


_SAVE_MAGIC = "mivs-ivf-flat-v1"


def save(filename: str, index: Index, include_dataset: bool = True):
    """cuvs.neighbors.ivf_flat.save: centroids, list sizes and (with include_dataset) every list's rows and
    ids, in list order, as a numpy .npz (plain arrays, no pickled objects)."""
    import numpy as np

    if not isinstance(index, Index):
        raise TypeError("index must be an ivf_flat.Index")
    torch.cuda.synchronize(index.device)
    sizes = index.list_sizes.numpy()
    if include_dataset:
        rows = index.list_rows().cpu().numpy()
        ids = index.list_ids().cpu().numpy()
    else:
        rows = np.zeros((0, index.dim), np.float32)
        ids = np.zeros((0,), np.int64)
        sizes = np.zeros_like(sizes)
    np.savez(filename, magic=np.array(_SAVE_MAGIC), metric=np.array(index.metric),
             centers=index.centers.cpu().numpy(), list_sizes=sizes.astype(np.int64), ids=ids.astype(np.int64),
             rows=rows.astype(np.float32))


def load(filename: str, resources=None, device: int | None = None, prefilter: bool = True) -> Index:
    """cuvs.neighbors.ivf_flat.load: an index written by `save`, on `device` (default: the current one).
    The lists keep their saved order and ids, so searches return what the saved index returned."""
    import numpy as np

    with np.load(filename, allow_pickle=False) as z:
        if str(z["magic"]) != _SAVE_MAGIC:
            raise ValueError(f"{filename!r} is not an mivs ivf_flat file")
        metric = str(z["metric"])
        centers, sizes, ids, rows = z["centers"], z["list_sizes"], z["ids"], z["rows"]
    dev = torch.cuda.current_device() if device is None else int(device)
    n_lists, dim = centers.shape
    c = torch.from_numpy(np.ascontiguousarray(centers, dtype=np.float32)).to(f"cuda:{dev}")
    r = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.float32).reshape(-1, dim)).to(f"cuda:{dev}")
    i = torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int64)).to(f"cuda:{dev}")
    hs = np.ascontiguousarray(sizes, dtype=np.int64)
    h = ctypes.c_void_p()
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_ivf_flat_build_from_lists(
            dev, stream_ptr(dev), ptr(r), ptr(i), hs.ctypes.data_as(ctypes.c_void_p), r.shape[0], dim, ptr(c),
            n_lists, metric_code(metric), 0, 1 if prefilter else 0, ctypes.byref(h)))
    return Index(h.value, metric)


def default_n_lists(n_rows: int) -> int:
    """The coordinator's default: max(1, min(256, N // 1000 + 1)) (index_building_coordinator.py:394)."""
    return max(1, min(256, n_rows // 1000 + 1))


__all__ = ["IndexParams", "SearchParams", "Index", "build", "build_from_centroids", "search", "extend", "save", "load",
           "default_n_lists", "metric_code"]
_ = math
