"""streaming.search_host: host queries with H2D / search / D2H overlapped on three HIP streams
(SURVEY.md §8(f) rank 2). The results must equal one device-side search per batch, bit for bit,
for every index kind, ragged last batches, unpinned and numpy inputs; and, for IVF-Flat, equal
the oracle's IVF search.
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


def _per_batch(search, q, k, B):
    ds, is_ = [], []
    for s in range(0, len(q), B):
        d, i = search(torch.from_numpy(q[s:s + B]).cuda(), k)
        ds.append(d.cpu().numpy())
        is_.append(i.cpu().numpy())
    return np.concatenate(ds), np.concatenate(is_)


@pytest.mark.parametrize("metric", ["sqeuclidean", "inner_product", "euclidean"])
@pytest.mark.parametrize("nq,B", [(1000, 256), (300, 1000), (777, 100), (1, 1)])
def test_ivf_flat_stream_equals_batches(mivs_lib, metric, nq, B):
    from mivs.neighbors import ivf_flat, streaming

    x, q = _data(12000, 128, 1), _data(nq, 128, 2)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=32, kmeans_n_iters=4, metric=metric), torch.from_numpy(x).cuda())
    sp = ivf_flat.SearchParams(n_probes=5)
    d, i = streaming.search_host(idx, q, 10, sp, batch_size=B)
    assert d.is_pinned() and i.is_pinned() and d.shape == (nq, 10)
    d0, i0 = _per_batch(lambda qq, k: ivf_flat.search(sp, idx, qq, k), q, 10, B)
    np.testing.assert_array_equal(i.numpy(), i0)
    np.testing.assert_array_equal(_bits(d.numpy()), _bits(d0))


def test_ivf_flat_stream_matches_oracle(mivs_lib):
    from mivs.neighbors import ivf_flat, streaming

    x, q = _data(6000, 64, 3), _data(500, 64, 4)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=16, kmeans_n_iters=3), torch.from_numpy(x).cuda())
    d, i = streaming.search_host(idx, torch.from_numpy(q), 7, ivf_flat.SearchParams(n_probes=4), batch_size=128)
    cents = idx.centers.cpu().numpy()
    od, oi, _ = O.ivf_search(x, cents, idx.list_sizes.numpy(), idx.list_ids().cpu().numpy(), q, 4, 7)
    np.testing.assert_array_equal(i.numpy(), oi)
    np.testing.assert_array_equal(_bits(d.numpy()), _bits(od))


def test_brute_force_and_ivf_pq_stream(mivs_lib):
    from mivs.neighbors import brute_force, ivf_pq, streaming

    x, q = _data(5000, 64, 5), _data(333, 64, 6)
    bf = brute_force.build(torch.from_numpy(x).cuda())
    d, i = streaming.search_host(bf, q, 12, batch_size=100)
    d0, i0 = _per_batch(lambda qq, k: brute_force.search(bf, qq, k), q, 12, 100)
    np.testing.assert_array_equal(i.numpy(), i0)
    np.testing.assert_array_equal(_bits(d.numpy()), _bits(d0))

    pq = ivf_pq.build(ivf_pq.IndexParams(n_lists=8, pq_dim=16, kmeans_n_iters=3), torch.from_numpy(x).cuda())
    sp = ivf_pq.SearchParams(n_probes=3)
    d, i = streaming.search_host(pq, q, 5, sp, batch_size=64)
    d0, i0 = _per_batch(lambda qq, k: ivf_pq.search(sp, pq, qq, k), q, 5, 64)
    np.testing.assert_array_equal(i.numpy(), i0)
    np.testing.assert_array_equal(_bits(d.numpy()), _bits(d0))


def test_stream_empty_and_errors(mivs_lib):
    from mivs.neighbors import brute_force, streaming

    bf = brute_force.build(torch.from_numpy(_data(100, 32, 7)).cuda())
    d, i = streaming.search_host(bf, np.zeros((0, 32), np.float32), 3)
    assert d.shape == (0, 3) and i.shape == (0, 3)
    with pytest.raises(ValueError, match="dim"):
        streaming.search_host(bf, np.zeros((4, 31), np.float32), 3)
    with pytest.raises(ValueError, match="host-resident"):
        streaming.search_host(bf, torch.zeros((4, 32)).cuda(), 3)
    with pytest.raises(ValueError, match="batch_size"):
        streaming.search_host(bf, np.zeros((4, 32), np.float32), 3, batch_size=0)


def test_stream_reuses_host_outputs(mivs_lib):
    from mivs.neighbors import brute_force, streaming

    x, q = _data(3000, 32, 8), _data(250, 32, 9)
    bf = brute_force.build(torch.from_numpy(x).cuda())
    d0, i0 = streaming.search_host(bf, q, 4, batch_size=64)
    od = torch.full((250, 4), -1.0).pin_memory()
    oi = torch.full((250, 4), -7, dtype=torch.int64).pin_memory()
    d1, i1 = streaming.search_host(bf, q, 4, batch_size=100, distances=od, neighbors=oi)
    assert d1.data_ptr() == od.data_ptr() and i1.data_ptr() == oi.data_ptr()
    np.testing.assert_array_equal(i1.numpy(), i0.numpy())
    np.testing.assert_array_equal(_bits(d1.numpy()), _bits(d0.numpy()))
    with pytest.raises(ValueError, match="distances"):
        streaming.search_host(bf, q, 4, distances=torch.empty((250, 5)))
