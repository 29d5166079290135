"""numpy front-end of the CPU oracle (liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; it is the checker, never the thing measured or shipped. Every
function documents the reference behaviour it restates (see mivs_oracle.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
L2, IP = 0, 1

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        i32, i64, f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        sig = {
            "orc_dim_pad": (i32, [i32]),
            "orc_dot": (ctypes.c_float, [P, P, i32]),
            "orc_norms": (None, [P, i64, i32, P]),
            "orc_normalize_rows": (None, [P, i64, i32, P]),
            "orc_knn": (None, [P, i64, P, i64, i32, i32, i32, i64, P, P]),
            "orc_refine": (None, [P, i64, i32, P, i64, P, i32, i32, i32, P, P]),
            "orc_merge": (None, [P, P, i64, i32, i32, i32, i32, P, P]),
            "orc_kmeans_assign": (None, [P, P, i64, P, i32, i32, i32, P]),
            "orc_kmeans_update": (None, [P, P, i64, P, i32, i32, P]),
            "orc_kmeans_rebalance": (None, [P, P, i64, P, i32, i32, i32, P]),
            "orc_kmeans_fit": (None, [P, P, i64, i32, i32, i32, i32, P]),
            "orc_kmeans_fit_ex": (None, [P, P, i64, i32, i32, i32, i32, i32, P]),
            "orc_train_count": (i64, [i64, i32, f64, i64]),
            "orc_train_rows": (None, [i64, i64, P]),
            "orc_init_rows": (None, [i64, i32, P]),
            "orc_ivf_build": (None, [P, i64, i32, i32, i32, f64, i64, i32, i32, i64, P, P, P]),
            "orc_ivf_lists_from_centroids": (None, [P, i64, i32, P, i32, i32, i64, P, P]),
            "orc_ivf_search": (None, [P, i64, i32, P, i32, P, P, P, i64, i32, i32, i32, P, P, P]),
            "orc_pq_len": (i32, [i32, i32]),
            "orc_pq_train_count": (i64, [i64, i32, i64]),
            "orc_ivfpq_build": (None, [P, i64, i32, i32, i32, f64, i32, i32, i64, i32, i64, P, P, P, P, P]),
            "orc_ivfpq_search": (None, [P, i32, i32, P, i32, i32, P, P, P, P, i64, i32, i32, i32, P, P, P]),
            "orc_ivfpq_search_ex": (None, [P, i32, i32, P, i32, i32, P, P, P, P, i64, i32, i32, i32, P, P, P, i32]),
            "orc_round_f16": (ctypes.c_float, [ctypes.c_float]),
            "orc_fast_threads": (i32, []),
            "orc_fast_set_threads": (None, [i32]),
            "orc_fast_knn": (None, [P, i64, P, i64, i32, i32, P, P]),
            "orc_fast_ivf_search": (None, [P, P, P, P, i32, i32, P, i64, i32, i32, P, P]),
            "orc_parallel_copy": (None, [P, P, i64]),
            "orc_fast_isa": (ctypes.c_char_p, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def metric_code(metric) -> int:
    if isinstance(metric, int):
        return metric
    if metric in ("cosine", "CosineExpanded"):
        raise ValueError("cosine: normalize_rows() both sides, search with inner_product, report 1 - ip")
    return IP if metric in ("inner_product", "ip", "IP") else L2


def dot(a, b) -> np.float32:
    a, b = _f32(a), _f32(b)
    return np.float32(lib().orc_dot(_p(a), _p(b), a.shape[0]))


def norms(x) -> np.ndarray:
    x = _f32(x)
    out = np.empty(x.shape[0], np.float32)
    lib().orc_norms(_p(x), x.shape[0], x.shape[1], _p(out))
    return out


def normalize_rows(x) -> np.ndarray:
    """x / sqrt(pinned ||x||^2) per row; zero rows stay zero (mivs_oracle.c orc_normalize_rows)."""
    x = _f32(x)
    out = np.empty_like(x)
    lib().orc_normalize_rows(_p(x), x.shape[0], x.shape[1], _p(out))
    return out


def cosine_knn(x, q, k, id_offset=0):
    """Exact k-NN by cosine distance 1 - cos(q, x) (sklearn NearestNeighbors(metric='cosine',
    algorithm='brute'), VectorSearch_QuestionRetrieval.ipynb:878): inner-product top-k of the
    normalised rows, distance 1 - ip in fp32."""
    d, i = knn(normalize_rows(x), normalize_rows(q), k, "inner_product", id_offset)
    return (np.float32(1.0) - d).astype(np.float32), i


def knn(x, q, k, metric="sqeuclidean", id_offset=0):
    """Exact kNN with the engine's arithmetic (bit-exact parity target)."""
    x, q = _f32(x), _f32(q)
    nq = q.shape[0]
    od = np.empty((nq, k), np.float32)
    oi = np.empty((nq, k), np.int64)
    lib().orc_knn(_p(x), x.shape[0], _p(q), nq, x.shape[1], k, metric_code(metric), id_offset, _p(od), _p(oi))
    return od, oi


def refine(x, q, candidates, k, metric="sqeuclidean"):
    """Exact top-k over each query's candidate rows (cuvs.neighbors.refine semantics, ties by id)."""
    x, q, c = _f32(x), _f32(q), _i64(candidates)
    nq = q.shape[0]
    od = np.empty((nq, k), np.float32)
    oi = np.empty((nq, k), np.int64)
    lib().orc_refine(_p(x), x.shape[0], x.shape[1], _p(q), nq, _p(np.ascontiguousarray(c)), c.shape[1], k,
                     metric_code(metric), _p(od), _p(oi))
    return od, oi


def merge(dist, ids, k, metric="sqeuclidean"):
    """[nq, m, k_in] candidate lists -> global top-k by (key, id)."""
    d, i = _f32(dist), _i64(ids)
    if d.ndim == 2:
        d, i = d[:, None, :], i[:, None, :]
    nq, m, kin = d.shape
    od = np.empty((nq, k), np.float32)
    oi = np.empty((nq, k), np.int64)
    lib().orc_merge(_p(np.ascontiguousarray(d)), _p(np.ascontiguousarray(i)), nq, m, kin, k, metric_code(metric),
                    _p(od), _p(oi))
    return od, oi


def kmeans_assign(x, c, rows=None, metric="sqeuclidean"):
    x, c = _f32(x), _f32(c)
    r = None if rows is None else _i64(rows)
    nr = x.shape[0] if r is None else r.shape[0]
    out = np.empty(nr, np.int32)
    lib().orc_kmeans_assign(_p(x), _p(r), nr, _p(c), c.shape[0], x.shape[1], metric_code(metric), _p(out))
    return out


def kmeans_update(x, labels, c, rows=None):
    """One Lloyd centroid update from given labels (orc_kmeans_update: fp64 sums over fixed 256-member
    chunks in ascending train position); c is updated in place and returned. Empty clusters keep c."""
    x = _f32(x)
    lab = np.ascontiguousarray(labels, dtype=np.int32)
    r = None if rows is None else _i64(rows)
    assert c.dtype == np.float32 and c.flags.c_contiguous
    lib().orc_kmeans_update(_p(x), _p(r), lab.shape[0], _p(lab), c.shape[0], x.shape[1], _p(c))
    return c


def kmeans_rebalance(x, labels, it, c, rows=None):
    """The IVF build's balancing step of iteration `it` (orc_kmeans_rebalance, cuVS adjust_centers
    restated); c is updated in place and returned."""
    x = _f32(x)
    lab = np.ascontiguousarray(labels, dtype=np.int32)
    r = None if rows is None else _i64(rows)
    assert c.dtype == np.float32 and c.flags.c_contiguous
    lib().orc_kmeans_rebalance(_p(x), _p(r), lab.shape[0], _p(lab), c.shape[0], x.shape[1], int(it), _p(c))
    return c


def kmeans_fit(x, c0, iters, rows=None, metric="sqeuclidean", balance=False):
    """Lloyd from c0; balance=True adds the under-filled-cluster re-seeding of the IVF build."""
    x = _f32(x)
    c = _f32(c0).copy()
    r = None if rows is None else _i64(rows)
    nr = x.shape[0] if r is None else r.shape[0]
    lib().orc_kmeans_fit_ex(_p(x), _p(r), nr, c.shape[0], x.shape[1], iters, metric_code(metric), int(balance),
                            _p(c))
    return c


def train_count(n, n_lists, fraction=0.5, max_per_list=0) -> int:
    return int(lib().orc_train_count(n, n_lists, fraction, max_per_list))


def train_rows(n, n_train) -> np.ndarray:
    out = np.empty(n_train, np.int64)
    lib().orc_train_rows(n, n_train, _p(out))
    return out


def ivf_build(x, n_lists, iters=20, fraction=0.5, max_per_list=0, metric="sqeuclidean", id_offset=0, balance=True):
    """-> (centroids [n_lists, d], list_sizes [n_lists], list_ids [n])."""
    x = _f32(x)
    n, d = x.shape
    cents = np.empty((n_lists, d), np.float32)
    sizes = np.empty(n_lists, np.int64)
    ids = np.empty(n, np.int64)
    lib().orc_ivf_build(_p(x), n, d, n_lists, iters, fraction, max_per_list, metric_code(metric), int(balance),
                        id_offset, _p(cents), _p(sizes), _p(ids))
    return cents, sizes, ids


def ivf_lists(x, centroids, metric="sqeuclidean", id_offset=0):
    x, c = _f32(x), _f32(centroids)
    sizes = np.empty(c.shape[0], np.int64)
    ids = np.empty(x.shape[0], np.int64)
    lib().orc_ivf_lists_from_centroids(_p(x), x.shape[0], x.shape[1], _p(c), c.shape[0], metric_code(metric),
                                       id_offset, _p(sizes), _p(ids))
    return sizes, ids


def ivf_search(x, centroids, sizes, ids, q, n_probes, k, metric="sqeuclidean", id_offset=0):
    """-> (dist [nq,k], ids [nq,k], probes [nq, n_probes])."""
    x, c, q = _f32(x), _f32(centroids), _f32(q)
    sizes, ids = _i64(sizes), _i64(ids)
    nq = q.shape[0]
    np_ = min(n_probes, c.shape[0])
    od = np.empty((nq, k), np.float32)
    oi = np.empty((nq, k), np.int64)
    op = np.empty((nq, np_), np.int32)
    lib().orc_ivf_search(_p(x), id_offset, x.shape[1], _p(c), c.shape[0], _p(sizes), _p(ids), _p(q), nq, np_, k,
                         metric_code(metric), _p(od), _p(oi), _p(op))
    return od, oi, op


# ---- IVF-PQ (cuVS ivf_pq restated; parity unpinned beyond the Lloyd k-means it builds on) ----
def pq_len(d, pq_dim) -> int:
    return int(lib().orc_pq_len(d, pq_dim))


def ivfpq_build(x, n_lists, pq_dim, pq_bits=8, iters=20, fraction=0.5, max_per_code=256, balance=True,
                id_offset=0):
    """-> (centroids [n_lists, d], codebooks [pq_dim, 2^pq_bits, pq_len], list_sizes [n_lists],
    list_ids [n], codes [n, pq_dim] uint8 in list order)."""
    x = _f32(x)
    n, d = x.shape
    pl = pq_len(d, pq_dim)
    cents = np.empty((n_lists, d), np.float32)
    cbs = np.empty((pq_dim, 1 << pq_bits, pl), np.float32)
    sizes = np.empty(n_lists, np.int64)
    ids = np.empty(n, np.int64)
    codes = np.empty((n, pq_dim), np.uint8)
    lib().orc_ivfpq_build(_p(x), n, d, n_lists, iters, fraction, pq_dim, pq_bits, max_per_code, int(balance),
                          id_offset, _p(cents), _p(cbs), _p(sizes), _p(ids), _p(codes))
    return cents, cbs, sizes, ids, codes


def round_f16(v) -> float:
    """orc_round_f16: fp32 -> nearest fp16 (ties to even) -> fp32."""
    return float(lib().orc_round_f16(float(v)))


def ivfpq_search(centroids, codebooks, sizes, ids, codes, q, n_probes, k, metric="sqeuclidean", lut_fp16=False):
    """-> (dist [nq,k], ids [nq,k], probes [nq, n_probes]); metric sqeuclidean or inner_product. lut_fp16: LUT entries
    rounded to fp16 (cuvs SearchParams.lut_dtype = float16; sqeuclidean only)."""
    c, cb, q = _f32(centroids), _f32(codebooks), _f32(q)
    sizes, ids = _i64(sizes), _i64(ids)
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    nq = q.shape[0]
    pq_dim, ncodes, _ = cb.shape
    np_ = min(n_probes, c.shape[0])
    od = np.empty((nq, k), np.float32)
    oi = np.empty((nq, k), np.int64)
    op = np.empty((nq, np_), np.int32)
    lib().orc_ivfpq_search_ex(_p(c), c.shape[0], c.shape[1], _p(cb), pq_dim, int(ncodes).bit_length() - 1, _p(sizes),
                              _p(ids), _p(codes), _p(q), nq, np_, k, metric_code(metric), _p(od), _p(oi), _p(op),
                              1 if lut_fp16 else 0)
    return od, oi, op


# ---- FAISS-algorithm CPU baseline (not bit-exact) ----
def fast_threads() -> int:
    return int(lib().orc_fast_threads())


def fast_set_threads(t: int) -> None:
    lib().orc_fast_set_threads(int(t))


def fast_isa() -> str:
    """the ISA the baseline's workers run with on this host (target_clones dispatch)"""
    return lib().orc_fast_isa().decode()


def parallel_copy(dst: np.ndarray, src: np.ndarray) -> None:
    """dst[...] = src, first-touched by every OpenMP thread (NUMA spread); both C-contiguous, same nbytes"""
    assert dst.flags.c_contiguous and src.flags.c_contiguous and dst.nbytes == src.nbytes
    lib().orc_parallel_copy(_p(dst), _p(src), dst.nbytes)


def fast_knn(x, q, k):
    x, q = _f32(x), _f32(q)
    od = np.empty((q.shape[0], k), np.float32)
    oi = np.empty((q.shape[0], k), np.int64)
    lib().orc_fast_knn(_p(x), x.shape[0], _p(q), q.shape[0], x.shape[1], k, _p(od), _p(oi))
    return od, oi


def fast_ivf_search(list_rows, list_ids, offsets, centroids, q, n_probes, k):
    lr, li, off, c, q = _f32(list_rows), _i64(list_ids), _i64(offsets), _f32(centroids), _f32(q)
    od = np.empty((q.shape[0], k), np.float32)
    oi = np.empty((q.shape[0], k), np.int64)
    lib().orc_fast_ivf_search(_p(lr), _p(li), _p(off), _p(c), c.shape[0], c.shape[1], _p(q), q.shape[0], n_probes, k,
                              _p(od), _p(oi))
    return od, oi
