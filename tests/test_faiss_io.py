"""FAISS index files (mivs.faiss_io; SURVEY.md §8(f) rank 3, the reference's faiss.read_index at
Latest/faiss.ipynb:686).

faiss is not installed and the reference holds no index file, so parity is unpinned against faiss
itself: the CPU tests assemble files byte by byte from the published FAISS 1.7.2 layout
(index_write.cpp: header, vectors as u64 count + data, 'ilar' inverted lists in 'full' and 'sprs'
size encodings) and check the reader; the GPU tests check write -> read round trips through the
engine bit for bit and against the oracle.
"""
import struct

import numpy as np
import pytest
import torch

import oracle as O


def _hdr(d, n, metric):
    h = struct.pack("<i", d) + struct.pack("<q", n) + struct.pack("<qq", 1 << 20, 1 << 20) + b"\x01" + \
        struct.pack("<i", metric)
    return h + (struct.pack("<f", 2.0) if metric > 1 else b"")  # metric_arg follows for metric_type > 1


def _flat(x, metric):
    tag = b"IxF2" if metric == 1 else b"IxFI"
    return tag + _hdr(x.shape[1], x.shape[0], metric) + struct.pack("<Q", x.size) + x.astype("<f4").tobytes()


def _ivf(cents, lists, metric, nprobe, sparse):
    """lists: [(list_no, rows [s, d], ids [s])] in list order."""
    nlist, d = cents.shape
    n = sum(len(i) for _, _, i in lists)
    out = b"IwFl" + _hdr(d, n, metric) + struct.pack("<QQ", nlist, nprobe) + _flat(cents, metric)
    out += b"\x00" + struct.pack("<Q", 0)  # direct map: none
    out += b"ilar" + struct.pack("<QQ", nlist, 4 * d)
    sizes = np.zeros(nlist, np.uint64)
    for l_, _, i in lists:
        sizes[l_] = len(i)
    if sparse:
        pairs = [v for l_, _, i in lists if len(i) for v in (l_, len(i))]
        out += b"sprs" + struct.pack("<Q", len(pairs)) + np.array(pairs, "<u8").tobytes()
    else:
        out += b"full" + struct.pack("<Q", nlist) + sizes.astype("<u8").tobytes()
    for _, r, i in lists:
        if len(i):
            out += r.astype("<f4").tobytes() + np.asarray(i, "<i8").tobytes()
    return out


def _rand(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


def test_read_flat_file(tmp_path):
    from mivs import faiss_io

    x = _rand((37, 12), 0)
    p = tmp_path / "flat.index"
    p.write_bytes(_flat(x, 1))
    rows, metric = faiss_io.read_flat_rows(str(p))
    assert metric == "sqeuclidean"
    np.testing.assert_array_equal(rows, x)
    rows, _ = faiss_io.read_flat_rows(str(p), row_range=(10, 25))
    np.testing.assert_array_equal(rows, x[10:25])
    p.write_bytes(_flat(x, 0))
    assert faiss_io.read_flat_rows(str(p))[1] == "inner_product"
    with pytest.raises(ValueError, match="row_range"):
        faiss_io.read_flat_rows(str(p), row_range=(5, 40))


@pytest.mark.parametrize("sparse", [False, True])
def test_read_ivf_flat_file(tmp_path, sparse):
    from mivs import faiss_io

    d, nlist = 8, 6
    cents = _rand((nlist, d), 1)
    lists = [(0, _rand((3, d), 2), [5, 9, 1]), (2, _rand((1, d), 3), [7]), (5, _rand((4, d), 4), [0, 2, 3, 4])]
    if not sparse:
        lists.append((4, _rand((2, d), 5), [11, 12]))
        lists.sort(key=lambda t: t[0])
    p = tmp_path / "ivf.index"
    p.write_bytes(_ivf(cents, lists, 1, 17, sparse))
    L = faiss_io.read_ivf_flat_lists(str(p))
    assert (L.d, L.metric, L.nprobe) == (d, "sqeuclidean", 17)
    np.testing.assert_array_equal(L.centroids, cents)
    want = np.zeros(nlist, np.int64)
    for l_, _, i in lists:
        want[l_] = len(i)
    np.testing.assert_array_equal(L.sizes, want)
    np.testing.assert_array_equal(L.ids, np.concatenate([np.asarray(i, np.int64) for _, _, i in lists]))
    np.testing.assert_array_equal(L.rows, np.concatenate([r for _, r, _ in lists]))


def test_bad_files(tmp_path):
    from mivs import faiss_io

    x = _rand((10, 4), 6)
    p = tmp_path / "t.index"
    p.write_bytes(_flat(x, 1)[:-7])
    with pytest.raises(ValueError, match="truncated"):
        faiss_io.read_flat_rows(str(p))
    p.write_bytes(b"IxPQ" + _flat(x, 1)[4:])
    with pytest.raises(ValueError, match="not an IndexFlat"):
        faiss_io.read_flat_rows(str(p))
    cents = _rand((2, 4), 7)
    good = _ivf(cents, [(0, x[:3], [0, 1, 2]), (1, x[3:5], [3, 4])], 1, 1, False)
    p.write_bytes(good.replace(b"ilar", b"ilod"))
    with pytest.raises(ValueError, match="not supported"):
        faiss_io.read_ivf_flat_lists(str(p))
    p.write_bytes(_ivf(cents, [(0, x[:3], [0, 1, 2])], 3, 1, False))
    with pytest.raises(ValueError, match="metric"):
        faiss_io.read_ivf_flat_lists(str(p))


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _unit(n, d, seed):
    x = _rand((n, d), seed)
    return x / np.linalg.norm(x, axis=1, keepdims=True).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["sqeuclidean", "inner_product"])
def test_ivf_flat_write_read_roundtrip(mivs_lib, tmp_path, metric):
    from mivs import faiss_io
    from mivs.neighbors import ivf_flat

    x, q = _unit(7000, 64, 10), _unit(90, 64, 11)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=20, kmeans_n_iters=3, metric=metric),
                         torch.from_numpy(x).cuda(), ids_offset=100)
    p = str(tmp_path / "ivf.index")
    faiss_io.write_index(idx, p, nprobe=7)
    L = faiss_io.read_ivf_flat_lists(p)
    assert L.nprobe == 7 and L.metric == metric
    back = faiss_io.read_index(p)
    assert back.faiss_nprobe == 7 and back.metric == metric and back.size == idx.size
    np.testing.assert_array_equal(back.list_ids().cpu().numpy(), idx.list_ids().cpu().numpy())
    np.testing.assert_array_equal(back.list_sizes.numpy(), idx.list_sizes.numpy())
    sp = ivf_flat.SearchParams(n_probes=5)
    d0, i0 = ivf_flat.search(sp, idx, torch.from_numpy(q).cuda(), 10)
    d1, i1 = ivf_flat.search(sp, back, torch.from_numpy(q).cuda(), 10)
    np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d0.cpu().numpy()))
    od, oi, _ = O.ivf_search(x, L.centroids, L.sizes, L.ids, q, 5, 10, metric=metric, id_offset=100)
    np.testing.assert_array_equal(i1.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(od))


@pytest.mark.gpu
def test_flat_file_to_brute_force_shards(mivs_lib, tmp_path):
    from mivs import faiss_io
    from mivs.neighbors import brute_force

    x, q = _unit(3000, 48, 12), _unit(40, 48, 13)
    p = str(tmp_path / "flat.index")
    faiss_io.write_flat(p, x, metric="inner_product")
    full = faiss_io.read_index(p)
    assert full.metric == "inner_product" and full.size == 3000
    d0, i0 = brute_force.search(full, torch.from_numpy(q).cuda(), 8)
    od, oi = O.knn(x, q, 8, metric="inner_product")
    np.testing.assert_array_equal(i0.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(d0.cpu().numpy()), _bits(od))
    shard = faiss_io.read_index(p, row_range=(1000, 2000))
    d1, i1 = brute_force.search(shard, torch.from_numpy(q).cuda(), 8)
    od, oi = O.knn(x[1000:2000], q, 8, metric="inner_product", id_offset=1000)
    np.testing.assert_array_equal(i1.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(od))
