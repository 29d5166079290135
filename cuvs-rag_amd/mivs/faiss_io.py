"""FAISS index files: read ``IndexFlat`` / ``IndexIVFFlat`` into mivs indexes, write them back
(SURVEY.md §8(f) rank 3).

The reference loads a prebuilt FAISS index with ``faiss.read_index(path)``
(``Latest/faiss.ipynb:682-693``, ``Latest/cuVS-2-gpu/faiss.ipynb:194``; the Wikipedia 2023-07 index,
6,286,775 × 384) and shards it over the GPUs (``index_cpu_to_gpus_list`` with ``shard=True``, a
contiguous row split). ``read_index`` gives the mivs equivalent: an ``IndexFlat*`` file becomes a
``brute_force.Index`` (optionally one contiguous shard of its rows, ids offset by the shard start),
an ``IndexIVFFlat`` file an ``ivf_flat.Index`` with the file's centroids, lists and ids (so its
searches rank the same rows the FAISS index would).

Format: FAISS 1.7.2 (``Latest/faiss.ipynb:29``) ``faiss/impl/index_write.cpp`` /
``index_read.cpp``, little-endian. faiss is not installed here and the reference holds no index
file, so the layout below is restated from the published writer and tested by round trips and a
hand-assembled byte stream (``tests/test_faiss_io.py``): parity unpinned against faiss itself.

  index header  : i32 d, i64 ntotal, i64 dummy, i64 dummy, u8 is_trained, i32 metric_type
                  (+ f32 metric_arg when metric_type > 1); metric 0 = inner product, 1 = L2
  vector<T>     : u64 count, count × T
  IndexFlat     : fourcc "IxFI" (IP) | "IxF2" (L2) | "IxFl"; header; vector<f32> (ntotal × d)
  IndexIVFFlat  : fourcc "IwFl"; header; u64 nlist; u64 nprobe; quantizer (an IndexFlat);
                  direct map (u8 type, vector<i64>, + vector<(i64, i64)> when type == 2);
                  inverted lists: fourcc "ilar", u64 nlist, u64 code_size, fourcc "full" with
                  vector<u64> sizes[nlist] | "sprs" with vector<u64> (list, size) pairs; then per
                  non-empty list its codes (size × code_size bytes = rows as f32) and ids (size × i64)
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np
import torch

from . import _native
from ._tensors import ptr, stream_ptr

_METRIC_IP, _METRIC_L2 = 0, 1


def _fourcc(s: str) -> int:
    return struct.unpack("<I", s.encode("ascii"))[0]


class _In:
    def __init__(self, f):
        self.f = f

    def raw(self, n: int) -> bytes:
        b = self.f.read(n)
        if len(b) != n:
            raise ValueError(f"truncated FAISS file: wanted {n} bytes at offset {self.f.tell() - len(b)}")
        return b

    def scalar(self, fmt: str):
        return struct.unpack("<" + fmt, self.raw(struct.calcsize(fmt)))[0]

    def fourcc(self) -> str:
        return self.raw(4).decode("latin-1")

    def array(self, dtype, count: int, out: np.ndarray | None = None) -> np.ndarray:
        dt = np.dtype(dtype)
        a = np.empty(count, dt) if out is None else out
        if count:
            mv = memoryview(a.reshape(-1)).cast("B")
            if self.f.readinto(mv) != count * dt.itemsize:
                raise ValueError("truncated FAISS file")
        return a

    def vector(self, dtype, expect: int | None = None) -> np.ndarray:
        n = self.scalar("Q")
        if expect is not None and n != expect:
            raise ValueError(f"FAISS vector holds {n} entries, expected {expect}")
        return self.array(dtype, n)

    def skip(self, n: int) -> None:
        self.f.seek(n, 1)


def _read_header(r: _In) -> dict:
    h = {"d": r.scalar("i"), "ntotal": r.scalar("q")}
    r.scalar("q"), r.scalar("q")  # two dummies (1 << 20)
    h["is_trained"] = bool(r.scalar("B"))
    h["metric"] = r.scalar("i")
    if h["metric"] > 1:
        h["metric_arg"] = r.scalar("f")
    if h["d"] < 1 or h["ntotal"] < 0:
        raise ValueError(f"bad FAISS index header {h}")
    return h


def _metric_name(m: int) -> str:
    if m == _METRIC_L2:
        return "sqeuclidean"
    if m == _METRIC_IP:
        return "inner_product"
    raise ValueError(f"FAISS metric_type {m} is not supported (0 = inner product, 1 = L2)")


_FLAT = ("IxFI", "IxF2", "IxFl")


def _read_flat_body(r: _In, h: dict, row_range=None) -> np.ndarray:
    n, d = h["ntotal"], h["d"]
    count = r.scalar("Q")
    if count != n * d:
        raise ValueError(f"IndexFlat holds {count} floats, expected ntotal*d = {n * d}")
    lo, hi = (0, n) if row_range is None else row_range
    if not (0 <= lo <= hi <= n):
        raise ValueError(f"row_range {row_range} outside [0, {n}]")
    r.skip(lo * d * 4)
    x = r.array(np.float32, (hi - lo) * d).reshape(hi - lo, d)
    r.skip((n - hi) * d * 4)
    return x


def _read_direct_map(r: _In) -> None:
    t = r.scalar("B")
    n = r.scalar("Q")
    r.skip(n * 8)
    if t == 2:  # hashtable: vector<pair<i64, i64>>
        n = r.scalar("Q")
        r.skip(n * 16)


class IvfFlatLists:
    """Host image of an IndexIVFFlat file."""

    def __init__(self, d, metric, centroids, sizes, ids, rows, nprobe):
        self.d, self.metric, self.centroids, self.sizes, self.ids, self.rows, self.nprobe = \
            d, metric, centroids, sizes, ids, rows, nprobe


def _read_ivf_flat(r: _In) -> IvfFlatLists:
    h = _read_header(r)
    nlist, nprobe = r.scalar("Q"), r.scalar("Q")
    qk = r.fourcc()
    if qk not in _FLAT:
        raise ValueError(f"IVF quantizer {qk!r} is not an IndexFlat")
    qh = _read_header(r)
    if qh["d"] != h["d"] or qh["ntotal"] != nlist:
        raise ValueError(f"quantizer {qh} does not match d={h['d']}, nlist={nlist}")
    cents = _read_flat_body(r, qh)
    _read_direct_map(r)
    ik = r.fourcc()
    if ik == "il00":
        sizes = np.zeros(nlist, np.int64)
    elif ik == "ilar":
        if r.scalar("Q") != nlist:
            raise ValueError("inverted lists nlist does not match the index")
        code_size = r.scalar("Q")
        if code_size != 4 * h["d"]:
            raise ValueError(f"code_size {code_size} is not 4*d: not an IndexIVFFlat")
        lt = r.fourcc()
        sizes = np.zeros(nlist, np.int64)
        if lt == "full":
            sizes[:] = r.vector(np.uint64, nlist).astype(np.int64)
        elif lt == "sprs":
            v = r.vector(np.uint64).astype(np.int64)
            if len(v) % 2:
                raise ValueError("sparse list sizes must come in (list, size) pairs")
            sizes[v[0::2]] = v[1::2]
        else:
            raise ValueError(f"unknown inverted-list size encoding {lt!r}")
    else:
        raise ValueError(f"inverted lists {ik!r} are not supported (only in-memory 'ilar')")
    n = int(sizes.sum())
    if n != h["ntotal"]:
        raise ValueError(f"lists hold {n} rows, header says {h['ntotal']}")
    d = h["d"]
    rows = np.empty((n, d), np.float32)
    ids = np.empty(n, np.int64)
    o = 0
    for s in sizes:
        if s:
            r.array(np.float32, int(s) * d, out=rows[o:o + s])
            r.array(np.int64, int(s), out=ids[o:o + s])
            o += s
    return IvfFlatLists(d, _metric_name(h["metric"]), cents, sizes, ids, rows, nprobe)


def read_index(path: str, device: int | None = None, row_range: tuple[int, int] | None = None,
               prefilter: bool = True):
    """``faiss.read_index`` for IndexFlat / IndexIVFFlat files -> ``brute_force.Index`` /
    ``ivf_flat.Index`` on ``device`` (default: the current one).

    ``row_range=(lo, hi)`` (IndexFlat only) loads rows [lo, hi) with ids lo..hi-1: one shard of the
    ``index_cpu_to_gpus_list(shard=True)`` split, without reading the other rows. For an IVF file the
    returned index carries ``faiss_nprobe`` (the file's nprobe)."""
    from .neighbors import brute_force, ivf_flat

    dev = torch.cuda.current_device() if device is None else int(device)
    with open(path, "rb") as f:
        r = _In(f)
        kind = r.fourcc()
        if kind in _FLAT:
            h = _read_header(r)
            x = _read_flat_body(r, h, row_range)
            lo = 0 if row_range is None else row_range[0]
            idx = brute_force.build(torch.from_numpy(x).to(f"cuda:{dev}"), metric=_metric_name(h["metric"]),
                                    ids_offset=lo)
            return idx
        if kind == "IwFl":
            if row_range is not None:
                raise ValueError("row_range applies to IndexFlat files only")
            L = _read_ivf_flat(r)
        else:
            raise ValueError(f"FAISS index type {kind!r} is not supported (IndexFlat*, IndexIVFFlat)")
    c = torch.from_numpy(np.ascontiguousarray(L.centroids)).to(f"cuda:{dev}")
    rows = torch.from_numpy(L.rows).to(f"cuda:{dev}")
    ids = torch.from_numpy(L.ids).to(f"cuda:{dev}")
    hs = np.ascontiguousarray(L.sizes, np.int64)
    h = ctypes.c_void_p()
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_ivf_flat_build_from_lists(
            dev, stream_ptr(dev), ptr(rows), ptr(ids), hs.ctypes.data_as(ctypes.c_void_p), rows.shape[0], L.d,
            ptr(c), c.shape[0], ivf_flat.metric_code(L.metric), 0, 1 if prefilter else 0, ctypes.byref(h)))
    idx = ivf_flat.Index(h.value, L.metric)
    idx.faiss_nprobe = int(L.nprobe)
    return idx


# ---------------------------------------------------------------------------------------------- write
def _header(d: int, ntotal: int, metric: int) -> bytes:
    return struct.pack("<iqqqBi", d, ntotal, 1 << 20, 1 << 20, 1, metric)


def _metric_code(metric: str) -> int:
    from .neighbors import ivf_flat

    m = ivf_flat.metric_code(metric)
    return _METRIC_L2 if m == _native.METRIC_L2 else _METRIC_IP


def _flat_bytes(x: np.ndarray, metric: int) -> list:
    x = np.ascontiguousarray(x, np.float32)
    return [b"IxF2" if metric == _METRIC_L2 else b"IxFI", _header(x.shape[1], x.shape[0], metric),
            struct.pack("<Q", x.size), x.tobytes()]


def write_flat(path: str, dataset, metric: str = "sqeuclidean") -> None:
    """``faiss.write_index(IndexFlatL2 / IndexFlatIP)`` of a ``[n, d]`` dataset (host or device)."""
    x = dataset.detach().cpu().numpy() if isinstance(dataset, torch.Tensor) else np.asarray(dataset)
    if x.ndim != 2:
        raise ValueError("dataset must be 2-D")
    with open(path, "wb") as f:
        for b in _flat_bytes(x, _metric_code(metric)):
            f.write(b)


def write_index(index, path: str, nprobe: int = 20) -> None:
    """``faiss.write_index`` of an ``ivf_flat.Index`` as an IndexIVFFlat file (centroids, lists in
    list order with their ids; the quantizer an IndexFlat of the same metric)."""
    from .neighbors import ivf_flat

    if not isinstance(index, ivf_flat.Index):
        raise TypeError("write_index takes an ivf_flat.Index (use write_flat for a dataset)")
    m = _metric_code(index.metric)
    cents = index.centers.cpu().numpy()
    sizes = index.list_sizes.numpy().astype(np.int64)
    rows = index.list_rows().cpu().numpy()
    ids = index.list_ids().cpu().numpy().astype(np.int64)
    nlist, d = cents.shape
    with open(path, "wb") as f:
        f.write(b"IwFl")
        f.write(_header(d, int(sizes.sum()), m))
        f.write(struct.pack("<QQ", nlist, int(nprobe)))
        for b in _flat_bytes(cents, m):
            f.write(b)
        f.write(struct.pack("<BQ", 0, 0))  # no direct map
        f.write(b"ilar")
        f.write(struct.pack("<QQ", nlist, 4 * d))
        nz = int((sizes > 0).sum())
        if nz > nlist // 2:
            f.write(b"full")
            f.write(struct.pack("<Q", nlist))
            f.write(sizes.astype(np.uint64).tobytes())
        else:
            f.write(b"sprs")
            pairs = np.stack([np.nonzero(sizes)[0], sizes[sizes > 0]], 1).astype(np.uint64).reshape(-1)
            f.write(struct.pack("<Q", pairs.size))
            f.write(pairs.tobytes())
        o = 0
        for s in sizes:
            if s:
                f.write(np.ascontiguousarray(rows[o:o + s], np.float32).tobytes())
                f.write(np.ascontiguousarray(ids[o:o + s], np.int64).tobytes())
                o += s


def read_ivf_flat_lists(path: str) -> IvfFlatLists:
    """The host image of an IndexIVFFlat file (no GPU needed): centroids, sizes, ids, rows, nprobe."""
    with open(path, "rb") as f:
        r = _In(f)
        if r.fourcc() != "IwFl":
            raise ValueError("not an IndexIVFFlat file")
        return _read_ivf_flat(r)


def read_flat_rows(path: str, row_range: tuple[int, int] | None = None) -> tuple[np.ndarray, str]:
    """The rows and metric of an IndexFlat file (no GPU needed)."""
    with open(path, "rb") as f:
        r = _In(f)
        if r.fourcc() not in _FLAT:
            raise ValueError("not an IndexFlat file")
        h = _read_header(r)
        return _read_flat_body(r, h, row_range), _metric_name(h["metric"])


__all__ = ["read_index", "write_index", "write_flat", "read_ivf_flat_lists", "read_flat_rows", "IvfFlatLists"]
