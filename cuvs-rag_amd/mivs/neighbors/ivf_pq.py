"""IVF-PQ on MI355X — drop-in for ``cuvs.neighbors.ivf_pq`` (cuVS 25.6.0).

The reference's call shapes:
  * ``ivf_pq.IndexParams(n_lists=..., pq_bits=8, pq_dim=min(64, d // 4))``  index_building_coordinator.py:398-403
  * ``ivf_pq.build(params, embeddings)``                                     index_building_coordinator.py:404
  * ``ivf_pq.IndexParams(n_lists=..., pq_dim=96, pq_bits=8)``                improved_multi_gpu_rag.py:131-136
  * ``ivf_pq.SearchParams()``; ``ivf_pq.search(sp, index, q, k)``           improved_multi_gpu_rag.py:228-230

Algorithm (restated in oracle/mivs_oracle.c orc_ivfpq_*): coarse k-means lists as IVF-Flat;
per subspace of pq_len = ceil(dim / pq_dim) dims a 256-entry codebook trained by k-means on the
residuals x - c_list of min(n, 256 * max_train_points_per_pq_code) strided rows; each row stored
as pq_dim one-byte codes. Search builds a pq_dim x 256 fp32 LUT per (query, probed list) in LDS
and sums LUT entries over the list's codes (hand-written HIP, cuvs-rag_amd/csrc/pq.hip).

This build: L2 and inner-product metrics (the coarse lists and codebooks are trained in L2 either way;
inner product ranks by -(q . c_l) - sum_j q_j . B_j[code_j], distances out are the inner products),
pq_bits = 8, k <= 64, identity rotation (dims past ``dim`` read as 0). For an exact
ranking of the PQ candidates use ``mivs.neighbors.refine`` (cuVS's IVF-PQ + refine pattern).
fp16 datasets (BASELINE config 5) are widened to fp32 on the device before training.
"""
from __future__ import annotations

import ctypes
import time

import numpy as np
import torch

from .. import _native
from .._tensors import as_device_f32, emit, out_tensor, ptr, stream_ptr
from .ivf_flat import metric_code


class IndexParams:
    """cuvs.neighbors.ivf_pq.IndexParams."""

    def __init__(self, n_lists: int = 1024, metric: str = "sqeuclidean", kmeans_n_iters: int = 20,
                 kmeans_trainset_fraction: float = 0.5, pq_bits: int = 8, pq_dim: int = 0,
                 codebook_kind: str = "subspace", force_random_rotation: bool = False,
                 add_data_on_build: bool = True, conservative_memory_allocation: bool = False,
                 max_train_points_per_pq_code: int = 256, kmeans_balance: bool = True):
        if int(n_lists) < 1:
            raise ValueError(f"n_lists must be >= 1, got {n_lists}")
        if metric not in ("sqeuclidean", "l2", "L2Expanded", "inner_product"):
            raise NotImplementedError("ivf_pq: the sqeuclidean and inner_product metrics are supported by this build")
        if int(pq_bits) != 8:
            raise NotImplementedError("ivf_pq: pq_bits must be 8 in this build")
        if codebook_kind not in ("subspace", "per_subspace"):
            raise NotImplementedError("ivf_pq: only per-subspace codebooks are supported by this build")
        if force_random_rotation:
            raise NotImplementedError("ivf_pq: force_random_rotation is not supported by this build")
        if int(pq_dim) < 0:
            raise ValueError(f"pq_dim must be >= 0, got {pq_dim}")
        self.n_lists = int(n_lists)
        self.metric = metric
        self.kmeans_n_iters = int(kmeans_n_iters)
        self.kmeans_trainset_fraction = float(kmeans_trainset_fraction)
        self.pq_bits = int(pq_bits)
        self.pq_dim = int(pq_dim)
        self.codebook_kind = codebook_kind
        self.force_random_rotation = bool(force_random_rotation)
        self.add_data_on_build = bool(add_data_on_build)
        self.conservative_memory_allocation = bool(conservative_memory_allocation)
        self.max_train_points_per_pq_code = int(max_train_points_per_pq_code)
        self.kmeans_balance = bool(kmeans_balance)

    def resolved_pq_dim(self, dim: int) -> int:
        """pq_dim = 0 -> dim // 4 (at least 1), the coordinator's rule without its 64 cap."""
        return self.pq_dim if self.pq_dim > 0 else max(1, dim // 4)

    def _c(self, dim: int) -> _native.IvfPqParams:
        return _native.IvfPqParams(self.n_lists, metric_code(self.metric), self.kmeans_n_iters,
                                   self.kmeans_trainset_fraction, self.resolved_pq_dim(dim), self.pq_bits,
                                   self.max_train_points_per_pq_code, 1 if self.kmeans_balance else 0,
                                   1 if self.add_data_on_build else 0)

    def __repr__(self):
        return (f"IndexParams(n_lists={self.n_lists}, pq_dim={self.pq_dim}, pq_bits={self.pq_bits}, "
                f"metric={self.metric!r}, kmeans_n_iters={self.kmeans_n_iters})")


class SearchParams:
    """cuvs.neighbors.ivf_pq.SearchParams (cuVS defaults: n_probes 20, fp32 LUT and distances).

    ``lut_dtype=np.float16`` stores every LUT entry as fp16 (rounded to nearest even when the LUT is built) and
    keeps the row sums in fp32, as cuVS's half-precision LUT does; the K9r scan then reads half the LDS bytes
    (DESIGN.md §8). It is served for the L2 metric with pq_len a multiple of 4 in 4..16; other indexes raise
    NotImplementedError at search. ``internal_distance_dtype`` is fp32 only."""

    def __init__(self, n_probes: int = 20, lut_dtype=np.float32, internal_distance_dtype=np.float32):
        if int(n_probes) < 1:
            raise ValueError(f"n_probes must be >= 1, got {n_probes}")
        if np.dtype(lut_dtype) not in (np.float32, np.float16):
            raise NotImplementedError(f"ivf_pq: lut_dtype {np.dtype(lut_dtype)} (this build: float32 or float16)")
        if np.dtype(internal_distance_dtype) != np.float32:
            raise NotImplementedError("ivf_pq: this build accumulates distances in fp32")
        self.n_probes = int(n_probes)
        self.lut_dtype = np.dtype(lut_dtype).type
        self.internal_distance_dtype = np.float32

    def __repr__(self):
        lut = "" if self.lut_dtype == np.float32 else ", lut_dtype=float16"
        return f"SearchParams(n_probes={self.n_probes}{lut})"


class Index:
    """Handle to an IVF-PQ index resident on one GPU (owned by libmivs)."""

    def __init__(self, handle: int, metric: str):
        self._h = ctypes.c_void_p(handle)
        self.metric = metric
        n, d, nl, m, dev = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib().mivs_index_info(self._h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(nl),
                                                    ctypes.byref(m), ctypes.byref(dev)))
        pd, pb, pl = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib().mivs_ivf_pq_info(self._h, ctypes.byref(pd), ctypes.byref(pb), ctypes.byref(pl)))
        self.size = int(n.value)
        self.dim = int(d.value)
        self.n_lists = int(nl.value)
        self.device = int(dev.value)
        self.pq_dim = int(pd.value)
        self.pq_bits = int(pb.value)
        self.pq_len = int(pl.value)
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
    def pq_centers(self) -> torch.Tensor:
        """Codebooks [pq_dim, 2^pq_bits, pq_len] (cuVS ``pq_centers`` for per-subspace codebooks)."""
        out = torch.empty((self.pq_dim, 1 << self.pq_bits, self.pq_len), dtype=torch.float32,
                          device=f"cuda:{self.device}")
        _native.check(_native.lib().mivs_ivf_pq_get_codebooks(self.handle, stream_ptr(self.device), ptr(out)))
        return out

    @property
    def list_sizes(self) -> torch.Tensor:
        out = torch.empty(self.n_lists, dtype=torch.int64)
        _native.check(_native.lib().mivs_ivf_flat_get_list_sizes(self.handle, ptr(out)))
        return out

    def list_ids(self) -> torch.Tensor:
        out = torch.empty(self.size, dtype=torch.int64, device=f"cuda:{self.device}")
        _native.check(_native.lib().mivs_ivf_flat_get_list_ids(self.handle, stream_ptr(self.device), ptr(out)))
        return out

    def codes(self) -> torch.Tensor:
        """[size, pq_dim] uint8 codes in list order (row t belongs to list_ids()[t])."""
        out = torch.empty((self.size, self.pq_dim), dtype=torch.uint8, device=f"cuda:{self.device}")
        _native.check(_native.lib().mivs_ivf_pq_get_codes(self.handle, stream_ptr(self.device), ptr(out)))
        return out

    def memory(self) -> dict:
        """Bytes the index holds in HBM by part (mivs_index_memory_info): the fp32 rows, norms / ids / offsets,
        centroids, the fp16 and fp8 copies, PQ codes; copies_skipped = 1 when the fp8 copy was left out (HBM
        budget, MIVS_INDEX_HBM_FRAC)."""
        m = _native.IndexMemory()
        _native.check(_native.lib().mivs_index_memory_info(self.handle, ctypes.byref(m)))
        return m.as_dict()

    def build_phases(self) -> dict:
        """Host wall time (s) of this index's build phases (recorded only while profiling was on)."""
        ph = _native.build_phases(self.handle, 2)
        if getattr(self, "_to_f32_s", None) is not None:
            ph = {"to_fp32": round(self._to_f32_s, 4), **ph}
        return ph

    def profile_collect(self) -> dict:
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
        return (f"ivf_pq.Index(size={self.size}, dim={self.dim}, n_lists={self.n_lists}, pq_dim={self.pq_dim}, "
                f"pq_bits={self.pq_bits}, device=cuda:{self.device})")


def build(index_params: IndexParams, dataset, resources=None, ids_offset: int = 0) -> Index:
    """Coarse k-means, list assignment, per-subspace codebooks and encoding, on the GPU holding `dataset`."""
    if not isinstance(index_params, IndexParams):
        raise TypeError("index_params must be an ivf_pq.IndexParams")
    prof = _native.profiling()
    t0 = time.perf_counter()
    x = as_device_f32(dataset, name="dataset")  # (fp16 input is widened exactly; the kernels read fp32)
    dev = x.device.index
    if prof:
        torch.cuda.synchronize(dev)
    t_conv = time.perf_counter() - t0
    n, d = x.shape
    if n < index_params.n_lists:
        raise ValueError(f"dataset has {n} rows, fewer than n_lists={index_params.n_lists}")
    h = ctypes.c_void_p()
    p = index_params._c(d)
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_ivf_pq_build(dev, stream_ptr(dev), ptr(x), n, d, ctypes.byref(p),
                                                      int(ids_offset), ctypes.byref(h)))
    idx = Index(h.value, index_params.metric)
    idx._to_f32_s = t_conv if prof else None
    return idx


def _search(search_params, index, queries, k: int, neighbors=None, distances=None, probes_out=None):
    """search() without the output hook: torch tensors on the index's device (mivs.neighbors.streaming)."""
    if not isinstance(index, Index):
        raise TypeError("index must be an ivf_pq.Index")
    sp = search_params if search_params is not None else SearchParams()
    k = int(k)
    if k < 1:
        raise ValueError(f"k must be >= 1, got {k}")
    dev = index.device
    q = as_device_f32(queries, device=dev, name="queries")
    if q.shape[1] != index.dim:
        raise ValueError(f"queries have dim {q.shape[1]}, index has {index.dim}")
    nq = q.shape[0]
    dist = out_tensor(distances, (nq, k), torch.float32, dev, "distances")
    nbrs = out_tensor(neighbors, (nq, k), torch.int64, dev, "neighbors")
    lut = 1 if getattr(sp, "lut_dtype", np.float32) == np.float16 else 0  # (MIVS_LUT_FP16 / MIVS_LUT_FP32)
    with torch.cuda.device(dev):
        rc = _native.lib().mivs_ivf_pq_search_ex(index.handle, stream_ptr(dev), ptr(q), nq, k, sp.n_probes, lut,
                                                 ptr(dist), ptr(nbrs), ptr(probes_out))
    if rc == _native.MIVS_ERR_UNSUPPORTED and lut:  # the fp16 LUT is not served for this index
        raise NotImplementedError(_native.lib().mivs_last_error().decode(errors="replace"))
    _native.check(rc)
    return dist, nbrs


def _emit2(r):
    return emit(r[0]), emit(r[1])


def search(search_params: SearchParams, index: Index, queries, k: int, neighbors=None, distances=None,
           resources=None, probes_out: torch.Tensor | None = None):
    """Approximate k-NN from the PQ codes of the n_probes closest lists -> ``(distances, neighbors)``."""
    return _emit2(_search(search_params, index, queries, k, neighbors, distances, probes_out))


def default_pq_dim(dim: int) -> int:
    """The coordinator's default: min(64, d // 4) (index_building_coordinator.py:402)."""
    return min(64, dim // 4)


__all__ = ["IndexParams", "SearchParams", "Index", "build", "search", "default_pq_dim"]
