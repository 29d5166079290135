"""fp16 pre-filter scan (K10) + exact fp32 refine (K11): results BIT-EXACT with the oracle and with the
fp32 scan, on shapes, metrics and magnitudes that stress the refine window.

The pre-filter is on by default for ivf_flat indexes and serves k <= 16; these tests check that it
actually served the search (last_search_stats()['prefilter']), that queries it cannot prove go
through the exact fallback (overflow_queries), and that either way the answer equals the oracle's.
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


def _check_vs_oracle(x, q, n_lists, n_probes, k, metric="sqeuclidean", iters=3, expect_pf=True):
    from mivs.neighbors import ivf_flat

    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=n_lists, kmeans_n_iters=iters, metric=metric), _gpu(x))
    assert idx.prefilter
    dist, ids = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, _gpu(q), k)
    st = idx.last_search_stats()
    assert st["prefilter"] == (1 if expect_pf else 0), st
    oc, osz, oids = O.ivf_build(x, n_lists, iters=iters, metric=metric)
    od, oi, _ = O.ivf_search(x, oc, osz, oids, q, n_probes, k, metric=metric)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))
    return idx, st


PF_CASES = [
    # n, d, nq, n_lists, n_probes, k, metric
    (8000, 64, 70, 32, 4, 10, "sqeuclidean"),
    (6000, 100, 65, 16, 5, 1, "sqeuclidean"),      # d % 64 != 0: zero-padded dims
    (40, 64, 9, 8, 2, 16, "sqeuclidean"),          # fewer probed rows than k: padded (-1, +inf)
    (40, 64, 9, 8, 2, 16, "inner_product"),
    (12000, 768, 130, 24, 6, 10, "sqeuclidean"),   # the benchmark's d
    (9000, 384, 33, 20, 8, 16, "sqeuclidean"),     # k = kPfMaxK
    (7000, 128, 90, 24, 6, 10, "inner_product"),
    (5000, 33, 40, 8, 3, 7, "inner_product"),
    (4000, 1000, 40, 8, 3, 10, "sqeuclidean"),     # dp = 1024: the LDS-capped work-item size
]


@pytest.mark.parametrize("n,d,nq,n_lists,n_probes,k,metric", PF_CASES)
def test_prefilter_bitexact_vs_oracle(mivs_lib, n, d, nq, n_lists, n_probes, k, metric):
    x = _data(n, d, seed=n + d, normalize=True)
    q = _data(nq, d, seed=n + d + 1, normalize=True)
    _, st = _check_vs_oracle(x, q, n_lists, n_probes, k, metric)
    if n >= 1000:  # (the tiny cases probe fewer than k rows: their windows hold all of them)
        assert st["window_candidates"] >= k * nq - st["overflow_queries"] * k


@pytest.mark.parametrize("scale", [1e4, 3e-7, 1.0])
def test_prefilter_magnitudes(mivs_lib, scale):
    """Unnormalised rows far outside (and far below) the fp16 range: the power-of-two scaling keeps the
    approximate keys within the proven window."""
    x = _data(6000, 96, seed=5, scale=scale)
    q = _data(50, 96, seed=6, scale=scale)
    _check_vs_oracle(x, q, 16, 4, 10)


def test_prefilter_mixed_row_norms(mivs_lib):
    """Rows whose norms span 4 orders of magnitude (the window uses the index-wide maxima)."""
    x = _data(6000, 64, seed=8) * np.logspace(-2, 2, 6000, dtype=np.float32)[:, None]
    q = _data(40, 64, seed=9)
    _check_vs_oracle(x.astype(np.float32), q, 16, 6, 10)


def test_prefilter_overflow_falls_back_exactly(mivs_lib):
    """Many exact duplicates: the window holds more candidates than the refine capacity, so the
    pre-filter must hand those queries to the exact scan — and the answer must not change."""
    base = _data(500, 64, seed=12, normalize=True)
    # every row 80 times: 80 equal keys per neighbour, more than the refine's 64-candidate window
    x = np.concatenate([base] * 80)
    q = np.concatenate([base[:20], _data(20, 64, seed=13, normalize=True)])
    idx, st = _check_vs_oracle(x, q, 8, 8, 10)
    assert st["overflow_queries"] > 0, st


def test_prefilter_toggle_identical(mivs_lib):
    from mivs import ops
    from mivs.neighbors import ivf_flat

    x = ops.synth_mixture(60000, 768, 0, n_centers=512, sigma=0.75)
    q = ops.synth_mixture(700, 768, 0, n_centers=512, sigma=0.75, row_begin=1 << 40)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=64, kmeans_n_iters=4), x)
    sp = ivf_flat.SearchParams(n_probes=12)
    d1, i1 = ivf_flat.search(sp, idx, q, 10)
    assert idx.last_search_stats()["prefilter"] == 1
    idx.set_prefilter(False)
    assert not idx.prefilter
    d2, i2 = ivf_flat.search(sp, idx, q, 10)
    assert idx.last_search_stats()["prefilter"] == 0
    assert torch.equal(i1, i2) and torch.equal(d1, d2)
    idx.set_prefilter(True)
    d3, i3 = ivf_flat.search(sp, idx, q, 10)
    assert torch.equal(i1, i3) and torch.equal(d1, d3)
    # k above kPfMaxK: K13 + K16, the same bits as the fp32 scan (MIVS_LARGE_K_PF=0)
    d4, i4 = ivf_flat.search(sp, idx, q, 20)
    assert idx.last_search_stats()["prefilter"] == 1 and idx.last_search_stats()["scan_kernel"] == 13
    import os

    os.environ["MIVS_LARGE_K_PF"] = "0"
    try:
        d5, i5 = ivf_flat.search(sp, idx, q, 20)
        assert idx.last_search_stats()["prefilter"] == 0
    finally:
        del os.environ["MIVS_LARGE_K_PF"]
    assert torch.equal(i4, i5) and torch.equal(d4, d5)


def test_prefilter_matches_fp32_scan_at_scale(mivs_lib):
    """The bench's corpus family (mixture, sigma 0.75, 768 dims) at 400k rows: pre-filter == fp32 scan."""
    from mivs import ops
    from mivs.neighbors import ivf_flat

    x = ops.synth_mixture(400_000, 768, 0, n_centers=4096, sigma=0.75)
    q = ops.synth_mixture(3000, 768, 0, n_centers=4096, sigma=0.75, row_begin=1 << 40)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=256, kmeans_n_iters=5), x)
    for n_probes, k in [(32, 10), (8, 16), (64, 1)]:
        sp = ivf_flat.SearchParams(n_probes=n_probes)
        idx.set_prefilter(True)
        d1, i1 = ivf_flat.search(sp, idx, q, k)
        st = idx.last_search_stats()
        assert st["prefilter"] == 1 and st["overflow_queries"] < 3000 // 100, st
        idx.set_prefilter(False)
        d2, i2 = ivf_flat.search(sp, idx, q, k)
        assert torch.equal(i1, i2) and torch.equal(d1, d2)


@pytest.mark.parametrize("metric", ["sqeuclidean", "inner_product"])
@pytest.mark.parametrize("k", [1, 10, 16])
def test_brute_force_prefilter_bitexact(mivs_lib, metric, k):
    """brute_force.search with k <= 16 runs the fp16 pre-filter over the one list (three 16384-row
    work items here) + the exact refine: identical to the fp32 scan and to the oracle."""
    from mivs.neighbors import brute_force

    rng = np.random.default_rng(77 + k)
    x = rng.standard_normal((40000, 128)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    q = rng.standard_normal((300, 128)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    idx = brute_force.build(torch.from_numpy(x).cuda(), metric=metric, ids_offset=11)
    assert idx.prefilter
    d1, i1 = brute_force.search(idx, torch.from_numpy(q).cuda(), k)
    st = idx.last_search_stats()
    idx.set_prefilter(False)
    assert not idx.prefilter
    d0, i0 = brute_force.search(idx, torch.from_numpy(q).cuda(), k)
    np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
    np.testing.assert_array_equal(d1.cpu().numpy().view(np.int32), d0.cpu().numpy().view(np.int32))
    od, oi = O.knn(x, q, k, metric=metric, id_offset=11)
    np.testing.assert_array_equal(i1.cpu().numpy(), oi)
    np.testing.assert_array_equal(d1.cpu().numpy().view(np.int32), od.view(np.int32))
    assert st["overflow_queries"] <= 300


@pytest.mark.parametrize("metric", ["sqeuclidean", "inner_product"])
def test_brute_force_prefilter_overflow_falls_back_exactly(mivs_lib, metric):
    """Brute force through the pre-filter with every row duplicated 80 times: the refine window of a
    query whose neighbour is a base row holds > 64 candidates, so those queries take the exact
    single-list fallback (rows gathered, norms recomputed, scattered back) -- and the answer is still
    the oracle's (the brute-force overflow branch)."""
    from mivs.neighbors import brute_force

    base = _data(400, 64, seed=21, normalize=True)
    x = np.concatenate([base] * 80)
    q = np.concatenate([base[:24], _data(24, 64, seed=22, normalize=True)])
    idx = brute_force.build(torch.from_numpy(x).cuda(), metric=metric, ids_offset=5)
    d1, i1 = brute_force.search(idx, torch.from_numpy(q).cuda(), 10)
    st = idx.last_search_stats()
    assert st["prefilter"] == 1 and st["overflow_queries"] > 0, st
    od, oi = O.knn(x, q, 10, metric=metric, id_offset=5)
    np.testing.assert_array_equal(i1.cpu().numpy(), oi)
    np.testing.assert_array_equal(d1.cpu().numpy().view(np.int32), od.view(np.int32))
    idx.close()
