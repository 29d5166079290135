"""GPU parity: every kernel of the hot path vs the CPU oracle, BIT-EXACT.

The oracle (oracle/mivs_oracle.c) restates the reference's cuVS/FAISS algorithm
with the engine's pinned arithmetic order,
so distances are compared bitwise (np.float32 views as int32) and ids exactly.
All calls go through libmivs.so (the C-ABI); nothing here has a CPU fallback.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _data(n, d, seed, scale=1.0, normalize=False):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, d)) * scale).astype(np.float32)
    if normalize:
        x /= np.linalg.norm(x, axis=1, keepdims=True).astype(np.float32)
    return x


def _gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("d", [1, 7, 32, 64, 100, 128, 384, 768, 1000])
def test_row_norms_bitexact(mivs_lib, d):
    from mivs import ops

    x = _data(257, d, seed=d)
    got = ops.row_norms(_gpu(x)).cpu().numpy()
    np.testing.assert_array_equal(_bits(got), _bits(O.norms(x)))


BF_CASES = [
    # n, d, nq, k, metric
    (1, 8, 3, 1, "sqeuclidean"),
    (5, 16, 7, 10, "sqeuclidean"),        # n < k: padded with (-1, +inf)
    (1000, 64, 33, 10, "sqeuclidean"),
    (3001, 100, 65, 1, "sqeuclidean"),
    (3001, 100, 65, 16, "sqeuclidean"),
    (4096, 128, 100, 32, "sqeuclidean"),
    (2500, 384, 40, 64, "sqeuclidean"),   # k=64: merge area in global scratch
    (5000, 768, 64, 10, "sqeuclidean"),
    (2000, 128, 50, 10, "inner_product"),
    (777, 33, 31, 5, "inner_product"),
]


@pytest.mark.parametrize("n,d,nq,k,metric", BF_CASES)
def test_brute_force_bitexact(mivs_lib, n, d, nq, k, metric):
    from mivs.neighbors import brute_force

    x = _data(n, d, seed=n + d)
    q = _data(nq, d, seed=n + d + 1)
    idx = brute_force.build(_gpu(x), metric=metric)
    dist, ids = brute_force.search(idx, _gpu(q), k)
    od, oi = O.knn(x, q, k, metric=metric)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


def test_brute_force_id_offset_and_self_match(mivs_lib):
    from mivs.neighbors import brute_force

    x = _data(1500, 96, seed=3, normalize=True)
    idx = brute_force.build(_gpu(x), ids_offset=1000)
    dist, ids = brute_force.search(idx, _gpu(x[:200]), 3)
    ids = ids.cpu().numpy()
    dist = dist.cpu().numpy()
    # a row queried against its own index is returned first at distance exactly 0
    np.testing.assert_array_equal(ids[:, 0], np.arange(200) + 1000)
    assert (dist[:, 0] == 0.0).all()
    assert (np.diff(dist, axis=1) >= 0).all()


@pytest.mark.parametrize("m,kin,k,metric", [(1, 3, 2, "sqeuclidean"), (8, 10, 10, "sqeuclidean"),
                                            (40, 16, 10, "inner_product"), (3, 5, 12, "sqeuclidean"),
                                            (7, 64, 64, "sqeuclidean")])
def test_merge_topk_matches_oracle(mivs_lib, m, kin, k, metric):
    from mivs import ops

    rng = np.random.default_rng(m * 100 + k)
    nq = 77
    d = rng.random((nq, m, kin)).astype(np.float32)
    d = np.round(d * 50) / 50  # force ties, broken by id
    if metric == "inner_product":
        d = -np.sort(-d, axis=2)
    else:
        d = np.sort(d, axis=2)
    ids = rng.permutation(nq * m * kin).reshape(nq, m, kin).astype(np.int64)
    ids[:, :, -1] = -1  # padding entries are skipped
    od, oi = O.merge(d, ids, k, metric=metric)
    gd, gi = ops.merge_topk(_gpu(d), _gpu(ids), k, metric=metric)
    np.testing.assert_array_equal(gi.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(gd.cpu().numpy()), _bits(od))


def test_reference_merge_fixture_on_gpu(mivs_lib):
    """test_search_result_aggregator.py:330-358 — two shards merged at k=3."""
    from mivs import ops

    d = np.array([[[2, 4], [1, 3]], [[6, 8], [5, 7]]], np.float32)
    i = np.array([[[20, 40], [10, 30]], [[60, 80], [50, 70]]], np.int64)
    gd, gi = ops.merge_topk(_gpu(d), _gpu(i), 3)
    np.testing.assert_array_equal(gd.cpu().numpy(), [[1, 2, 3], [5, 6, 7]])
    np.testing.assert_array_equal(gi.cpu().numpy(), [[10, 20, 30], [50, 60, 70]])


@pytest.mark.parametrize("n,d,nc,iters", [(3000, 32, 16, 5), (6000, 100, 40, 3), (20000, 64, 300, 2)])
def test_kmeans_fit_bitexact(mivs_lib, n, d, nc, iters):
    from mivs.cluster import kmeans

    x = _data(n, d, seed=nc)
    c0 = x[(np.arange(nc) * n) // nc]
    got, _ = kmeans.fit(kmeans.KMeansParams(n_clusters=nc, max_iter=iters), _gpu(x), centroids=_gpu(c0))
    exp = O.kmeans_fit(x, c0, iters)
    np.testing.assert_array_equal(_bits(got.cpu().numpy()), _bits(exp))
    lab = kmeans.predict(kmeans.KMeansParams(n_clusters=nc), got, _gpu(x)).cpu().numpy()
    np.testing.assert_array_equal(lab, O.kmeans_assign(x, exp))


IVF_BUILD_CASES = [
    # n, d, n_lists, iters, fraction, chunk_rows
    (5000, 100, 16, 5, 0.5, 0),
    (8000, 128, 64, 4, 0.3, 64),     # several chunks per list
    (12000, 768, 32, 2, 0.5, 0),
    (9000, 64, 1100, 1, 1.0, 0),     # > 1024 lists: coarse step merges centroid chunks
]


@pytest.mark.parametrize("n,d,n_lists,iters,fraction,chunk_rows", IVF_BUILD_CASES)
def test_ivf_flat_build_and_search_bitexact(mivs_lib, n, d, n_lists, iters, fraction, chunk_rows):
    from mivs.neighbors import ivf_flat

    x = _data(n, d, seed=n_lists, normalize=True)
    q = _data(97, d, seed=n_lists + 7, normalize=True)
    params = ivf_flat.IndexParams(n_lists=n_lists, kmeans_n_iters=iters, kmeans_trainset_fraction=fraction,
                                  chunk_rows=chunk_rows)
    idx = ivf_flat.build(params, _gpu(x), ids_offset=5)
    oc, osz, oids = O.ivf_build(x, n_lists, iters=iters, fraction=fraction, id_offset=5)
    np.testing.assert_array_equal(_bits(idx.centers.cpu().numpy()), _bits(oc))
    np.testing.assert_array_equal(idx.list_sizes.numpy(), osz)
    np.testing.assert_array_equal(idx.list_ids().cpu().numpy(), oids)
    np.testing.assert_array_equal(idx.list_rows().cpu().numpy(), x[oids - 5])
    for n_probes, k in [(1, 1), (4, 10), (min(20, n_lists), 32), (min(64, n_lists), 64)]:
        probes = torch.empty((q.shape[0], n_probes), dtype=torch.int32, device="cuda")
        dist, ids = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, _gpu(q), k, probes_out=probes)
        od, oi, op = O.ivf_search(x, oc, osz, oids, q, n_probes, k, id_offset=5)
        np.testing.assert_array_equal(probes.cpu().numpy(), op)
        np.testing.assert_array_equal(ids.cpu().numpy(), oi)
        np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


def test_ivf_flat_unbalanced_lloyd_bitexact(mivs_lib):
    from mivs.neighbors import ivf_flat

    x = _data(9000, 64, seed=41, normalize=True)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=48, kmeans_n_iters=6, kmeans_balance=False), _gpu(x))
    oc, osz, oids = O.ivf_build(x, 48, iters=6, balance=False)
    np.testing.assert_array_equal(_bits(idx.centers.cpu().numpy()), _bits(oc))
    np.testing.assert_array_equal(idx.list_ids().cpu().numpy(), oids)


def test_kmeans_rebalance_reseeds_starved_clusters(mivs_lib):
    """Skewed init (most centroids on one cluster): balancing must leave no starved list; bit-exact."""
    from mivs.neighbors import ivf_flat

    rng = np.random.default_rng(51)
    centers = rng.standard_normal((16, 32)).astype(np.float32) * 4
    lab = np.sort(rng.integers(0, 16, 16000))  # rows sorted by cluster: strided init is skewed
    x = (centers[lab] + rng.standard_normal((16000, 32))).astype(np.float32)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=16, kmeans_n_iters=12, kmeans_trainset_fraction=1.0),
                         _gpu(x))
    oc, osz, oids = O.ivf_build(x, 16, iters=12, fraction=1.0)
    np.testing.assert_array_equal(_bits(idx.centers.cpu().numpy()), _bits(oc))
    np.testing.assert_array_equal(idx.list_sizes.numpy(), osz)
    assert osz.min() > 0.25 * 1000


def test_ivf_flat_inner_product_bitexact(mivs_lib):
    from mivs.neighbors import ivf_flat

    x = _data(6000, 96, seed=11, normalize=True)
    q = _data(50, 96, seed=12, normalize=True)
    c0 = x[(np.arange(24) * 6000) // 24]
    idx = ivf_flat.build_from_centroids(_gpu(c0), _gpu(x), metric="inner_product")
    osz, oids = O.ivf_lists(x, c0, metric="inner_product")
    np.testing.assert_array_equal(idx.list_sizes.numpy(), osz)
    np.testing.assert_array_equal(idx.list_ids().cpu().numpy(), oids)
    dist, ids = ivf_flat.search(ivf_flat.SearchParams(n_probes=6), idx, _gpu(q), 10)
    od, oi, _ = O.ivf_search(x, c0, osz, oids, q, 6, 10, metric="inner_product")
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


def test_ivf_full_probe_equals_brute_force(mivs_lib):
    """n_probes = n_lists scans everything: IVF must return exactly the brute-force answer."""
    from mivs.neighbors import brute_force, ivf_flat

    x = _data(7000, 64, seed=21, normalize=True)
    q = _data(120, 64, seed=22, normalize=True)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=32, kmeans_n_iters=3), _gpu(x))
    d1, i1 = ivf_flat.search(ivf_flat.SearchParams(n_probes=32), idx, _gpu(q), 10)
    bf = brute_force.build(_gpu(x))
    d2, i2 = brute_force.search(bf, _gpu(q), 10)
    np.testing.assert_array_equal(i1.cpu().numpy(), i2.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d2.cpu().numpy()))


def test_distances_within_1e4_of_fp64(mivs_lib):
    """north_star tolerance: L2 distances within 1e-4 of the exact (fp64) value."""
    from mivs.neighbors import brute_force

    x = _data(4000, 768, seed=31, normalize=True)
    q = _data(64, 768, seed=32, normalize=True)
    dist, ids = brute_force.search(brute_force.build(_gpu(x)), _gpu(q), 10)
    ids = ids.cpu().numpy()
    exact = ((x[ids].astype(np.float64) - q[:, None, :].astype(np.float64)) ** 2).sum(-1)
    assert np.abs(dist.cpu().numpy() - exact).max() < 1e-4


def test_synth_slices_are_row_pure(mivs_lib):
    """synth_mixture launches in 2^24-row slices; rows must be a pure function of the global row index."""
    from mivs import ops

    n = (1 << 24) + 1000
    whole = ops.synth_mixture(n, 8, seed=5, n_centers=64)
    tail = ops.synth_mixture(2000, 8, seed=5, n_centers=64, row_begin=(1 << 24) - 1000)
    assert torch.equal(whole[(1 << 24) - 1000:], tail)


def test_list_export_beyond_2p32_elements(mivs_lib):
    """list_rows()/list_ids() on an index whose n*d exceeds 2^32 (one launch's work-item limit)."""
    from mivs import ops
    from mivs.neighbors import ivf_flat

    n, d = 5_700_000, 768  # n*d = 4.38e9
    x = ops.synth_mixture(n, d, seed=9, n_centers=1024, sigma=0.5)
    cents = x[torch.arange(0, n, n // 256, device=x.device)[:256]].contiguous()
    idx = ivf_flat.build_from_centroids(cents, x)
    ids = idx.list_ids()
    assert torch.equal(torch.sort(ids).values, torch.arange(n, device=ids.device))
    rows = idx.list_rows()
    g = torch.Generator(device="cpu").manual_seed(0)
    sel = torch.cat([torch.randint(0, n, (20000,), generator=g), torch.arange(n - 4096, n)]).to(x.device)
    assert torch.equal(rows[sel], x[ids[sel]])
    del rows
    # self-queries from the tail of the corpus find themselves at distance 0 with one probe per nearest list
    q = x[n - 64:].contiguous()
    dist, nid = ivf_flat.search(ivf_flat.SearchParams(n_probes=4), idx, q, 1)
    assert torch.equal(nid[:, 0].cpu(), torch.arange(n - 64, n))
    assert float(dist.abs().max()) < 1e-4


# ---- large k (K8 select: DUMP scan + per-query range-refining select), reference top_k = 2000 ----
BF_LARGE_K = [
    # n, d, nq, k, metric
    (3000, 64, 20, 2000, "sqeuclidean"),     # n <= CAP: select-all path
    (1500, 64, 9, 2000, "sqeuclidean"),      # n < k: padded with (-1, +inf)
    (20000, 96, 37, 100, "sqeuclidean"),     # refinement passes (CAP 1024)
    (30000, 128, 16, 2000, "sqeuclidean"),
    (50000, 32, 8, 4096, "sqeuclidean"),     # CAP 8192
    (12000, 64, 25, 777, "inner_product"),
]


@pytest.mark.parametrize("n,d,nq,k,metric", BF_LARGE_K)
def test_brute_force_large_k_bitexact(mivs_lib, n, d, nq, k, metric):
    from mivs.neighbors import brute_force

    x = _data(n, d, seed=n + k)
    q = _data(nq, d, seed=n + k + 1)
    dist, ids = brute_force.search(brute_force.build(_gpu(x), metric=metric), _gpu(q), k)
    od, oi = O.knn(x, q, k, metric=metric)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


def test_large_k_duplicate_rows_tie_break_by_id(mivs_lib):
    """Duplicated corpus rows give equal keys: order by id, also when ties overflow the LDS capacity."""
    from mivs.neighbors import brute_force

    base = _data(3000, 48, seed=77)
    x = np.concatenate([base] * 4)                      # every row 4 times
    same = np.repeat(_data(1, 48, seed=78), 9000, 0)    # 9000 identical rows (id-phase refinement)
    x = np.concatenate([x, same])
    q = np.concatenate([base[:5], same[:2], _data(4, 48, seed=79)])
    for k in (300, 1500, 4096):
        dist, ids = brute_force.search(brute_force.build(_gpu(x)), _gpu(q), k)
        od, oi = O.knn(x, q, k)
        np.testing.assert_array_equal(ids.cpu().numpy(), oi)
        np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


@pytest.mark.parametrize("n_probes,k,metric", [(8, 100, "sqeuclidean"), (128, 2000, "sqeuclidean"),
                                                (100, 10, "sqeuclidean"), (40, 500, "inner_product")])
def test_ivf_flat_large_k_and_probes_bitexact(mivs_lib, n_probes, k, metric):
    from mivs.neighbors import ivf_flat

    x = _data(40000, 64, seed=91, normalize=True)
    q = _data(70, 64, seed=92, normalize=True)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=256, kmeans_n_iters=3, metric=metric), _gpu(x))
    oc, osz, oids = O.ivf_build(x, 256, iters=3, metric=metric)
    np.testing.assert_array_equal(_bits(idx.centers.cpu().numpy()), _bits(oc))
    probes = torch.empty((q.shape[0], n_probes), dtype=torch.int32, device="cuda")
    dist, ids = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, _gpu(q), k, probes_out=probes)
    od, oi, op = O.ivf_search(x, oc, osz, oids, q, n_probes, k, metric=metric)
    np.testing.assert_array_equal(probes.cpu().numpy(), op)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


def test_large_k_query_batching(mivs_lib, monkeypatch):
    """A tiny select workspace forces many query batches; results must not change."""
    from mivs.neighbors import brute_force, ivf_flat

    x = _data(20000, 64, seed=95, normalize=True)
    q = _data(300, 64, seed=96, normalize=True)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=64, kmeans_n_iters=2), _gpu(x))
    bf = brute_force.build(_gpu(x))
    ref = [ivf_flat.search(ivf_flat.SearchParams(n_probes=16), idx, _gpu(q), 200),
           brute_force.search(bf, _gpu(q), 200)]
    monkeypatch.setenv("MIVS_SELECT_WORKSPACE_MB", "1")
    got = [ivf_flat.search(ivf_flat.SearchParams(n_probes=16), idx, _gpu(q), 200),
           brute_force.search(bf, _gpu(q), 200)]
    for (rd, ri), (gd, gi) in zip(ref, got):
        assert torch.equal(ri, gi) and torch.equal(rd, gd)


@pytest.mark.parametrize("m,kin,k,metric", [(4, 600, 1000, "sqeuclidean"), (8, 2000, 2000, "sqeuclidean"),
                                            (3, 300, 4096, "inner_product")])
def test_merge_topk_large_k_matches_oracle(mivs_lib, m, kin, k, metric):
    from mivs import ops

    rng = np.random.default_rng(m * 1000 + k)
    nq = 13
    d = (np.round(rng.random((nq, m, kin)) * 200) / 200).astype(np.float32)  # many ties, broken by id
    d = -np.sort(-d, axis=2) if metric == "inner_product" else np.sort(d, axis=2)
    ids = rng.permutation(nq * m * kin).reshape(nq, m, kin).astype(np.int64)
    ids[:, :, -3:] = -1
    od, oi = O.merge(d, ids, k, metric=metric)
    gd, gi = ops.merge_topk(_gpu(d), _gpu(ids), k, metric=metric)
    np.testing.assert_array_equal(gi.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(gd.cpu().numpy()), _bits(od))


# ---- K3w (64-query tiles, slab-staged queries): same arithmetic, must be bit-identical ----
WIDE_CASES = [
    # n, d, nq, k, metric, n_lists (0 = brute force)
    (5000, 768, 100, 10, "sqeuclidean", 0),
    (3001, 128, 65, 1, "sqeuclidean", 0),
    (4096, 256, 129, 16, "sqeuclidean", 0),
    (2000, 128, 50, 8, "inner_product", 0),
    (777, 124, 31, 4, "sqeuclidean", 0),      # d % 4 == 0, dp = 128, tail dims zero
    (20000, 768, 300, 10, "sqeuclidean", 64),
    (12000, 384, 97, 16, "sqeuclidean", 32),
    (9000, 256, 70, 10, "inner_product", 40),
]


@pytest.mark.parametrize("waves", ["4", "8"])
@pytest.mark.parametrize("n,d,nq,k,metric,n_lists", WIDE_CASES)
def test_wide_scan_bitexact(mivs_lib, monkeypatch, n, d, nq, k, metric, n_lists, waves):
    from mivs.neighbors import brute_force, ivf_flat

    monkeypatch.setenv("MIVS_SCAN_WIDE", "1")
    monkeypatch.setenv("MIVS_SCAN_WIDE_WAVES", waves)
    x = _data(n, d, seed=n + d + 3, normalize=True)
    q = _data(nq, d, seed=n + d + 4, normalize=True)
    if n_lists == 0:
        dist, ids = brute_force.search(brute_force.build(_gpu(x), metric=metric), _gpu(q), k)
        od, oi = O.knn(x, q, k, metric=metric)
    else:
        idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=n_lists, kmeans_n_iters=3, metric=metric), _gpu(x))
        oc, osz, oids = O.ivf_build(x, n_lists, iters=3, metric=metric)
        np.testing.assert_array_equal(_bits(idx.centers.cpu().numpy()), _bits(oc))
        np.testing.assert_array_equal(idx.list_ids().cpu().numpy(), oids)
        n_probes = min(8, n_lists)
        dist, ids = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, _gpu(q), k)
        od, oi, _ = O.ivf_search(x, oc, osz, oids, q, n_probes, k, metric=metric)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


# ---- IVF-PQ (K9 LUT scan): codebooks, codes and search bit-exact vs oracle orc_ivfpq_* ----
PQ_CASES = [
    # n, d, n_lists, pq_dim, iters, nq, n_probes, k
    (6000, 64, 16, 16, 4, 40, 4, 10),
    (9000, 128, 24, 32, 3, 33, 8, 16),
    (4000, 100, 8, 20, 3, 17, 8, 5),      # pq_len 5, rot_dim 100: no padding dims
    (5000, 96, 12, 40, 2, 29, 5, 32),     # pq_len 3, rot_dim 120 > d: zero-padded dims
    (12000, 768, 32, 96, 2, 20, 6, 10),   # the reference's pq_dim = 96 at d = 768
    (9000, 32, 2, 8, 3, 15, 2, 10),       # lists > 4096 rows (K9s row blocks), one LUT half only
    (8000, 768, 16, 96, 2, 21, 6, 64),    # k = 64: the candidate pool of IVF-PQ + refine
    (7000, 64, 16, 16, 3, 19, 5, 40),
    (6000, 64, 16, 16, 4, 40, 8, 200),    # 64 < k <= 256: K9r candidate-superset slots + K8 (IVF-PQ + refine pools)
    (12000, 768, 32, 96, 2, 20, 6, 120),  # the bench's refine pool (12 x k = 120) at the reference's pq_dim
    (9000, 32, 2, 8, 3, 15, 2, 100),      # lists > 4096 rows: two chunks, two candidate slots per probe
    (6000, 64, 32, 16, 3, 25, 20, 100),   # 20 slots per query (> 4096 entries): K8c reloads its keys per pass
    (12000, 768, 32, 96, 2, 20, 6, 300),  # k > 256: K9r DUMP + K8
]


@pytest.mark.parametrize("n,d,n_lists,pq_dim,iters,nq,n_probes,k", PQ_CASES)
def test_ivf_pq_build_and_search_bitexact(mivs_lib, n, d, n_lists, pq_dim, iters, nq, n_probes, k):
    _pq_case(n, d, n_lists, pq_dim, iters, nq, n_probes, k)


@pytest.mark.parametrize("case", [c for c in PQ_CASES if 16 < c[-1] <= 64])
def test_ivf_pq_register_lists_bitexact(mivs_lib, monkeypatch, case):
    """k in (16, 64] through the 32/64-entry register lists of K9s (MIVS_PQ_DUMP_K=64) instead of the
    default path (K9r; K9s DUMP + K8 without it): the same bits."""
    monkeypatch.setenv("MIVS_PQ_RT", "0")
    monkeypatch.setenv("MIVS_PQ_DUMP_K", "64")
    _pq_case(*case)


@pytest.mark.parametrize("pq_len", [4, 8, 12, 16])
def test_ivf_pq_k9r_mfma_lut_every_pq_len(mivs_lib, monkeypatch, pq_len):
    """K9r builds each LUT on v_mfma_f32_16x16x4_f32 and stores the results to LDS after hand-counted wait states
    (pq.hip): for every pq_len it serves (pq_rt_supported: 4, 8, 12, 16) its search equals the oracle and
    K9s (MIVS_PQ_RT=0) bit for bit, so a toolchain that schedules a store closer to its MFMA fails here"""
    pq_dim = 8
    _pq_case(3000, pq_dim * pq_len, 8, pq_dim, 2, 24, 4, 10)
    monkeypatch.setenv("MIVS_PQ_RT", "0")
    _pq_case(3000, pq_dim * pq_len, 8, pq_dim, 2, 24, 4, 10)


PQ_LUT16_CASES = [
    # n, d, n_lists, pq_dim, iters, nq, n_probes, k
    (6000, 64, 16, 16, 4, 40, 4, 10),     # pq_len 4
    (9000, 128, 24, 16, 3, 33, 8, 16),    # pq_len 8
    (4000, 96, 8, 8, 3, 17, 8, 5),        # pq_len 12
    (5000, 128, 12, 8, 2, 29, 5, 1),      # pq_len 16, k = 1
    (7000, 64, 16, 16, 3, 19, 5, 40),     # k in (16, 64]
    (6000, 64, 16, 16, 4, 40, 8, 200),    # k > 64: DUMP + K8 select
    (12000, 768, 32, 192, 2, 20, 6, 10),  # d = 768, pq_len 4
]


@pytest.mark.parametrize("n,d,n_lists,pq_dim,iters,nq,n_probes,k", PQ_LUT16_CASES)
def test_ivf_pq_fp16_lut_bitexact(mivs_lib, n, d, n_lists, pq_dim, iters, nq, n_probes, k):
    """SearchParams(lut_dtype=float16): K9r stores each LUT entry rounded to fp16 (nearest even) and sums them in
    fp32 -- probes, ids and distance bits equal to oracle orc_ivfpq_search_ex(lut_fp16=1)"""
    _pq_case(n, d, n_lists, pq_dim, iters, nq, n_probes, k, lut16=True)


def test_ivf_pq_fp16_lut_unsupported_and_recall(mivs_lib, monkeypatch):
    """the fp16 LUT is served by K9r for L2 only: inner product, pq_len 3 and MIVS_PQ_RT=0 raise
    NotImplementedError; on clustered data its recall stays within 0.02 of the fp32 LUT's"""
    from mivs import ops
    from mivs.neighbors import brute_force, ivf_pq

    sp16 = ivf_pq.SearchParams(n_probes=4, lut_dtype=np.float16)
    x = _data(3000, 64, seed=5, normalize=True)
    q = _gpu(_data(8, 64, seed=6, normalize=True))
    ip = ivf_pq.build(ivf_pq.IndexParams(n_lists=8, metric="inner_product", pq_dim=16, kmeans_n_iters=2), _gpu(x))
    with pytest.raises(NotImplementedError):
        ivf_pq.search(sp16, ip, q, 10)
    x96 = _data(3000, 96, seed=7, normalize=True)
    l3 = ivf_pq.build(ivf_pq.IndexParams(n_lists=8, pq_dim=32, kmeans_n_iters=2), _gpu(x96))
    with pytest.raises(NotImplementedError):
        ivf_pq.search(sp16, l3, _gpu(_data(8, 96, seed=8, normalize=True)), 10)
    l2 = ivf_pq.build(ivf_pq.IndexParams(n_lists=8, pq_dim=16, kmeans_n_iters=2), _gpu(x))
    ivf_pq.search(sp16, l2, q, 10)
    monkeypatch.setenv("MIVS_PQ_RT", "0")
    with pytest.raises(NotImplementedError):
        ivf_pq.search(sp16, l2, q, 10)
    monkeypatch.delenv("MIVS_PQ_RT")
    with pytest.raises(NotImplementedError):
        ivf_pq.SearchParams(lut_dtype=np.float64)

    xs = ops.synth_mixture(50000, 128, 4, n_centers=256, sigma=0.35)
    qs = ops.synth_mixture(300, 128, 4, n_centers=256, sigma=0.35, row_begin=1 << 40)
    idx = ivf_pq.build(ivf_pq.IndexParams(n_lists=64, pq_dim=32, kmeans_n_iters=5), xs)
    _, gt = brute_force.search(brute_force.build(xs), qs, 10)
    gt = gt.cpu().numpy()
    rec = {}
    for lut in (np.float32, np.float16):
        _, ids = ivf_pq.search(ivf_pq.SearchParams(n_probes=16, lut_dtype=lut), idx, qs, 10)
        rec[lut] = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(ids.cpu().numpy(), gt)])
    assert rec[np.float16] > rec[np.float32] - 0.02, rec


def _pq_case(n, d, n_lists, pq_dim, iters, nq, n_probes, k, lut16=False):
    from mivs.neighbors import ivf_pq

    x = _data(n, d, seed=n + pq_dim, normalize=True)
    q = _data(nq, d, seed=n + pq_dim + 1, normalize=True)
    params = ivf_pq.IndexParams(n_lists=n_lists, pq_dim=pq_dim, kmeans_n_iters=iters, max_train_points_per_pq_code=32)
    idx = ivf_pq.build(params, _gpu(x), ids_offset=3)
    oc, ocb, osz, oids, ocodes = O.ivfpq_build(x, n_lists, pq_dim, iters=iters, max_per_code=32, id_offset=3)
    np.testing.assert_array_equal(_bits(idx.centers.cpu().numpy()), _bits(oc))
    np.testing.assert_array_equal(_bits(idx.pq_centers.cpu().numpy()), _bits(ocb))
    np.testing.assert_array_equal(idx.list_sizes.numpy(), osz)
    np.testing.assert_array_equal(idx.list_ids().cpu().numpy(), oids)
    np.testing.assert_array_equal(idx.codes().cpu().numpy(), ocodes)
    probes = torch.empty((nq, n_probes), dtype=torch.int32, device="cuda")
    sp = ivf_pq.SearchParams(n_probes=n_probes, lut_dtype=np.float16 if lut16 else np.float32)
    dist, ids = ivf_pq.search(sp, idx, _gpu(q), k, probes_out=probes)
    od, oi, op = O.ivfpq_search(oc, ocb, osz, oids, ocodes, q, n_probes, k, lut_fp16=lut16)
    np.testing.assert_array_equal(probes.cpu().numpy(), op)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


@pytest.mark.parametrize("k", [10, 40, 100, 200])
def test_ivf_pq_tied_keys_bitexact(mivs_lib, k):
    """every row 250 times: the best key of a list chunk is tied 250 times, more than K9r's 128-entry
    candidate list at k <= 16 (its block-wide fallback rounds run), within the 512 list at k = 40, and at
    k = 100 / 200 more than a 256-entry candidate slot holds (the slot's exact top-k) with K8c's id digit passes
    ordering the ties -- ids (ties by id) and bits equal to the oracle"""
    from mivs.neighbors import ivf_pq

    base = _data(40, 64, seed=91, normalize=True)
    x = np.concatenate([base] * 250)
    q = np.concatenate([base[:9], _data(9, 64, seed=92, normalize=True)])
    params = ivf_pq.IndexParams(n_lists=4, pq_dim=16, kmeans_n_iters=3, max_train_points_per_pq_code=32)
    idx = ivf_pq.build(params, _gpu(x), ids_offset=0)
    oc, ocb, osz, oids, ocodes = O.ivfpq_build(x, 4, 16, iters=3, max_per_code=32, id_offset=0)
    np.testing.assert_array_equal(idx.codes().cpu().numpy(), ocodes)
    dist, ids = ivf_pq.search(ivf_pq.SearchParams(n_probes=2), idx, _gpu(q), k)
    od, oi, _ = O.ivfpq_search(oc, ocb, osz, oids, ocodes, q, 2, k)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


PQ_IP_CASES = [
    # n, d, n_lists, pq_dim, iters, nq, n_probes, k, split
    (6000, 64, 16, 16, 4, 40, 4, 10, True),
    (12000, 768, 32, 96, 2, 20, 6, 10, True),     # K9s at the reference's pq_dim
    (9000, 32, 2, 8, 3, 15, 2, 10, True),         # lists > 4096 rows: K9s row blocks
    (5000, 96, 12, 40, 2, 29, 5, 32, False),      # K9 (MIVS_PQ_SPLIT=0), pq_len 3, padded dims
    (8000, 768, 16, 96, 2, 21, 6, 64, True),      # k = 64
    (5000, 96, 12, 40, 2, 29, 5, 150, True),      # k > 64: DUMP + K8
]


@pytest.mark.parametrize("n,d,n_lists,pq_dim,iters,nq,n_probes,k,split", PQ_IP_CASES)
def test_ivf_pq_inner_product_bitexact(mivs_lib, monkeypatch, n, d, n_lists, pq_dim, iters, nq, n_probes, k, split):
    """metric inner_product: probes by q . c_l, LUT -(q_j . B_j[c]) with the coarse key in subspace 0,
    inner products out -- ids, probes and distance bits equal to oracle orc_ivfpq_search(ORC_IP)."""
    from mivs.neighbors import ivf_pq

    if not split:
        monkeypatch.setenv("MIVS_PQ_SPLIT", "0")
    x = _data(n, d, seed=n + pq_dim + 7, normalize=True)
    q = _data(nq, d, seed=n + pq_dim + 8, normalize=True)
    params = ivf_pq.IndexParams(n_lists=n_lists, metric="inner_product", pq_dim=pq_dim, kmeans_n_iters=iters,
                                max_train_points_per_pq_code=32)
    idx = ivf_pq.build(params, _gpu(x), ids_offset=5)
    oc, ocb, osz, oids, ocodes = O.ivfpq_build(x, n_lists, pq_dim, iters=iters, max_per_code=32, id_offset=5)
    np.testing.assert_array_equal(idx.codes().cpu().numpy(), ocodes)
    probes = torch.empty((nq, n_probes), dtype=torch.int32, device="cuda")
    dist, ids = ivf_pq.search(ivf_pq.SearchParams(n_probes=n_probes), idx, _gpu(q), k, probes_out=probes)
    od, oi, op = O.ivfpq_search(oc, ocb, osz, oids, ocodes, q, n_probes, k, metric="inner_product")
    np.testing.assert_array_equal(probes.cpu().numpy(), op)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))
    assert (np.diff(dist.cpu().numpy(), axis=1) <= 0).all()  # inner products, descending


def test_ivf_pq_fp16_dataset_and_recall(mivs_lib):
    """fp16 input (BASELINE config 5) is widened on the device: the index equals the one built from the
    widened fp32 copy, and PQ recall against exact neighbours is in the expected range for pq_len 4."""
    from mivs import ops
    from mivs.neighbors import brute_force, ivf_pq

    x = ops.synth_mixture(50000, 128, 4, n_centers=256, sigma=0.35)
    q = ops.synth_mixture(200, 128, 4, n_centers=256, sigma=0.35, row_begin=1 << 40)
    params = ivf_pq.IndexParams(n_lists=64, pq_dim=32, kmeans_n_iters=5)
    idx = ivf_pq.build(params, x.half())
    ref = ivf_pq.build(params, x.half().float())
    assert idx.size == 50000 and idx.pq_len == 4
    assert torch.equal(idx.codes(), ref.codes()) and torch.equal(idx.pq_centers, ref.pq_centers)
    d1, i1 = ivf_pq.search(ivf_pq.SearchParams(n_probes=16), idx, q, 10)
    d2, i2 = ivf_pq.search(ivf_pq.SearchParams(n_probes=16), ref, q, 10)
    assert torch.equal(i1, i2) and torch.equal(d1, d2)
    _, gt = brute_force.search(brute_force.build(x.half().float()), q, 10)
    ids, gt = i1.cpu().numpy(), gt.cpu().numpy()
    rec = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(ids, gt)])
    assert rec > 0.3, rec
