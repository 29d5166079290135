"""ivf_flat.save / load / extend (cuvs.neighbors.ivf_flat API).

* save -> load reproduces the index exactly: centroids, list sizes, list ids and rows, and the search
  results bit for bit.
* extend appends rows to their nearest lists after each list's current rows: building on half the
  rows and extending with the rest equals the one-shot build from the same centroids, and the oracle's
  IVF lists (oracle.ivf_search over the lists) give the same search results.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _data(n, d, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, d)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True).astype(np.float32)


def _gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("metric", ["sqeuclidean", "inner_product"])
def test_save_load_roundtrip_bitexact(mivs_lib, tmp_path, metric):
    from mivs.neighbors import ivf_flat

    x, q = _data(9000, 96, 1), _data(80, 96, 2)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=24, kmeans_n_iters=4, metric=metric), _gpu(x), ids_offset=3)
    path = str(tmp_path / "idx.npz")
    ivf_flat.save(path, idx)
    back = ivf_flat.load(path)
    assert (back.size, back.dim, back.n_lists, back.metric) == (idx.size, idx.dim, idx.n_lists, idx.metric)
    np.testing.assert_array_equal(_bits(back.centers.cpu().numpy()), _bits(idx.centers.cpu().numpy()))
    np.testing.assert_array_equal(back.list_sizes.numpy(), idx.list_sizes.numpy())
    np.testing.assert_array_equal(back.list_ids().cpu().numpy(), idx.list_ids().cpu().numpy())
    np.testing.assert_array_equal(back.list_rows().cpu().numpy(), idx.list_rows().cpu().numpy())
    for k in (1, 10, 100):
        d0, i0 = ivf_flat.search(ivf_flat.SearchParams(n_probes=6), idx, _gpu(q), k)
        d1, i1 = ivf_flat.search(ivf_flat.SearchParams(n_probes=6), back, _gpu(q), k)
        np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
        np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d0.cpu().numpy()))


def test_save_without_dataset_then_extend(mivs_lib, tmp_path):
    from mivs.neighbors import ivf_flat

    x = _data(4000, 64, 3)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=8, kmeans_n_iters=3), _gpu(x))
    path = str(tmp_path / "empty.npz")
    ivf_flat.save(path, idx, include_dataset=False)
    back = ivf_flat.load(path)
    assert back.size == 0 and back.n_lists == 8
    ivf_flat.extend(back, _gpu(x))
    assert back.size == x.shape[0]
    np.testing.assert_array_equal(back.list_ids().cpu().numpy(), idx.list_ids().cpu().numpy())
    np.testing.assert_array_equal(back.list_sizes.numpy(), idx.list_sizes.numpy())


@pytest.mark.parametrize("split", [1, 2500, 5999])
def test_extend_equals_one_shot_build_and_oracle(mivs_lib, split):
    from mivs.neighbors import ivf_flat

    x, q = _data(6000, 128, 4), _data(50, 128, 5)
    cents = _data(16, 128, 6)
    full = ivf_flat.build_from_centroids(_gpu(cents), _gpu(x))
    part = ivf_flat.build_from_centroids(_gpu(cents), _gpu(x[:split]))
    ivf_flat.extend(part, _gpu(x[split:]))  # ids continue at `split`
    assert part.size == full.size
    np.testing.assert_array_equal(part.list_sizes.numpy(), full.list_sizes.numpy())
    np.testing.assert_array_equal(part.list_ids().cpu().numpy(), full.list_ids().cpu().numpy())
    np.testing.assert_array_equal(part.list_rows().cpu().numpy(), full.list_rows().cpu().numpy())
    oids = full.list_ids().cpu().numpy()
    osz = full.list_sizes.numpy()
    od, oi, _ = O.ivf_search(x, cents, osz, oids, q, 5, 10)
    dist, ids = ivf_flat.search(ivf_flat.SearchParams(n_probes=5), part, _gpu(q), 10)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


@pytest.mark.parametrize("dim", [128, 768])
def test_search_extend_search_rebuilds_prepass_copies(mivs_lib, dim):
    """a search builds K13's fp8 pre-pass copy of the lists on first use; extend changes the lists, so the next
    search must score the new lists' copy (the old one is released with the fp16 copy): results equal the
    oracle's after the extend"""
    from mivs.neighbors import ivf_flat

    x, q = _data(6000, dim, 7), _data(40, dim, 8)
    cents = _data(16, dim, 9)
    part = ivf_flat.build_from_centroids(_gpu(cents), _gpu(x[:2000]))
    ivf_flat.search(ivf_flat.SearchParams(n_probes=5), part, _gpu(q), 10)  # (builds the copies)
    ivf_flat.extend(part, _gpu(x[2000:]))
    full = ivf_flat.build_from_centroids(_gpu(cents), _gpu(x))
    od, oi, _ = O.ivf_search(x, cents, full.list_sizes.numpy(), full.list_ids().cpu().numpy(), q, 5, 10)
    dist, ids = ivf_flat.search(ivf_flat.SearchParams(n_probes=5), part, _gpu(q), 10)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


def test_extend_with_explicit_ids(mivs_lib):
    from mivs.neighbors import ivf_flat

    x = _data(3000, 64, 7)
    cents = _data(6, 64, 8)
    idx = ivf_flat.build_from_centroids(_gpu(cents), _gpu(x[:1000]))
    new_ids = np.arange(10_000_000, 10_002_000, dtype=np.int64)
    ivf_flat.extend(idx, _gpu(x[1000:]), new_ids)
    ids = idx.list_ids().cpu().numpy()
    assert set(ids.tolist()) == set(range(1000)) | set(new_ids.tolist())
    # a new row finds itself at distance 0 under its explicit id
    d, i = ivf_flat.search(ivf_flat.SearchParams(n_probes=6), idx, _gpu(x[2500:2501]), 1)
    assert int(i[0, 0]) == 10_001_500 and float(d[0, 0]) <= 1e-5


def test_rebuild_reuses_cached_blocks_same_index(mivs_lib):
    """Buf's block cache (capi_util.hpp; opt-in, enabled here): an index built after another was closed gets the closed one's device
    blocks back (the sizes match) and must come out identical -- lists, rows, footprint and search bits -- as must
    a third build while the second is alive (fresh allocations)."""
    from mivs import _native
    from mivs.neighbors import ivf_flat

    x, q = _data(120000, 768, 5), _data(64, 768, 6)  # (rows 370 MB: above the cache's 64 MB block floor)
    p = ivf_flat.IndexParams(n_lists=64, kmeans_n_iters=3)
    _native.set_block_cache_limit(8 << 30, 0)  # (the cache is opt-in)
    a = ivf_flat.build(p, _gpu(x))
    da, ia = ivf_flat.search(ivf_flat.SearchParams(n_probes=8), a, _gpu(q), 10)
    ref = (a.list_sizes.numpy().copy(), a.list_ids().cpu().numpy(), a.memory())
    a.close()
    b = ivf_flat.build(p, _gpu(x))  # (takes a's cached blocks)
    c = ivf_flat.build(p, _gpu(x))  # (b is alive: new blocks)
    for idx in (b, c):
        d, i = ivf_flat.search(ivf_flat.SearchParams(n_probes=8), idx, _gpu(q), 10)
        np.testing.assert_array_equal(i.cpu().numpy(), ia.cpu().numpy())
        np.testing.assert_array_equal(_bits(d.cpu().numpy()), _bits(da.cpu().numpy()))
        np.testing.assert_array_equal(idx.list_sizes.numpy(), ref[0])
        np.testing.assert_array_equal(idx.list_ids().cpu().numpy(), ref[1])
        assert idx.memory() == ref[2]
    b.close()
    c.close()
    assert _native.cached_memory(0)["bytes"] > 0
    _native.set_block_cache_limit(0, 0)  # (lowering the limit frees what it held)
    assert _native.cached_memory(0)["bytes"] == 0
