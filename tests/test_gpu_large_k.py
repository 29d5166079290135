"""Large k through the fp16 pre-filter (K13 + K16): the reference's top_k = 2000 and k * 2 per
shard (Latest/cuVS-2-gpu/improved_multi_gpu_rag.py:40,247).

The answer must be the oracle's (orc_ivf_search) bit for bit and equal the exact fp32 path (K3 DUMP + K8,
MIVS_LARGE_K_PF=0) whatever the sample says: T_q only decides which queries K16 can prove, the rest take the
exact scan. So the tests also drive the sample to both extremes and force every query into the fallback."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _data(n, d, seed, normalize=True):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, d)).astype(np.float32)
    if normalize:
        x /= np.linalg.norm(x, axis=1, keepdims=True).astype(np.float32)
    return x


def _mixture(n, d, seed, centers=64, sigma=0.6):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((centers, d)).astype(np.float32)
    x = c[rng.integers(0, centers, n)] + sigma * rng.standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True).astype(np.float32)
    return x


def _gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _search(idx, q, k, n_probes):
    from mivs.neighbors import ivf_flat

    d, i = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, _gpu(q), k)
    return d.cpu().numpy(), i.cpu().numpy()


CASES = [
    # n, d, n_lists, n_probes, nq, k, metric
    (40000, 64, 128, 16, 57, 17, "sqeuclidean"),
    (40000, 64, 128, 16, 57, 100, "sqeuclidean"),
    (60000, 128, 96, 24, 33, 2000, "sqeuclidean"),
    (30000, 96, 64, 8, 41, 777, "inner_product"),
    (50000, 768, 64, 12, 29, 4000, "sqeuclidean"),
    (8000, 32, 16, 16, 19, 4096, "sqeuclidean"),   # every probed row: fewer than k -> padded
]


@pytest.fixture(scope="module")
def built():
    cache = {}

    def get(n, d, n_lists, metric, seed):
        from mivs.neighbors import ivf_flat

        key = (n, d, n_lists, metric, seed)
        if key not in cache:
            x = _mixture(n, d, seed)
            idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=n_lists, kmeans_n_iters=3, metric=metric), _gpu(x))
            cache[key] = (x, idx)
        return cache[key]

    yield get
    for _, idx in cache.values():
        idx.close()


@pytest.mark.parametrize("n,d,n_lists,n_probes,nq,k,metric", CASES)
def test_large_k_prefilter_bitexact_vs_oracle_and_exact(mivs_lib, built, monkeypatch, n, d, n_lists, n_probes, nq, k,
                                                        metric):
    x, idx = built(n, d, n_lists, metric, n + d)
    q = _mixture(nq, d, n + d + 1)
    dist, ids = _search(idx, q, k, n_probes)
    st = idx.last_search_stats()
    assert st["prefilter"] == 1 and st["scan_kernel"] == 13 and st["k"] == k, st
    od, oi, _ = O.ivf_search(x, idx.centers.cpu().numpy(), idx.list_sizes.numpy(), idx.list_ids().cpu().numpy(), q,
                             n_probes, k, metric=metric)
    np.testing.assert_array_equal(ids, oi)
    np.testing.assert_array_equal(_bits(dist), _bits(od))
    monkeypatch.setenv("MIVS_LARGE_K_PF", "0")
    ed, ei = _search(idx, q, k, n_probes)
    assert idx.last_search_stats()["prefilter"] == 0
    np.testing.assert_array_equal(ei, ids)
    np.testing.assert_array_equal(_bits(ed), _bits(dist))


@pytest.mark.parametrize("env", [{"MIVS_LK_SAMPLE_DIV": "1"}, {"MIVS_LK_SAMPLE_DIV": "7"},
                                 {"MIVS_LK_SAMPLE_DIV": "100000"}, {"MIVS_RS_WAVE_CAP": "2"},
                                 {"MIVS_LK_WORKSPACE_MB": "1"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_large_k_switches_same_bits(mivs_lib, built, monkeypatch, env):
    """the whole list as the sample (T_q from the exact k-th: every query provable), a 1/7 sample, a one-group
    sample (T_q loose or +inf), record streams of 2 (every query lost: the exact fallback), query batches of one
    query, the T_q statistics: the same bits"""
    x, idx = built(60000, 128, 96, "sqeuclidean", 60000 + 128)
    q = _mixture(45, 128, 7)
    d0, i0 = _search(idx, q, 1500, 24)
    for kk, v in env.items():
        monkeypatch.setenv(kk, v)
    d1, i1 = _search(idx, q, 1500, 24)
    st = idx.last_search_stats()
    if "MIVS_RS_WAVE_CAP" in env:
        assert st["cand_overflow"] == st["n_queries"] and st["overflow_queries"] == st["n_queries"], st
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))


def test_large_k_duplicate_rows_tie_break_by_id(mivs_lib):
    """equal keys (every row 3 times, and 5000 copies of one row) are ordered by id inside K16's sort"""
    from mivs.neighbors import ivf_flat

    base = _data(6000, 48, 77)
    same = np.repeat(_data(1, 48, 78), 5000, 0)
    x = np.concatenate([base, base, base, same])
    q = np.concatenate([base[:6], same[:2], _data(5, 48, 79)])
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=32, kmeans_n_iters=2), _gpu(x))
    for k in (300, 1500, 4096):
        d, i = _search(idx, q, k, 8)
        od, oi, _ = O.ivf_search(x, idx.centers.cpu().numpy(), idx.list_sizes.numpy(), idx.list_ids().cpu().numpy(),
                                 q, 8, k)
        np.testing.assert_array_equal(i, oi)
        np.testing.assert_array_equal(_bits(d), _bits(od))
    idx.close()


def test_large_k_uses_prefilter_and_reports_window(mivs_lib, built):
    """K16 serves the search: candidates streamed by K13, window rows recomputed, few or no unproven queries"""
    x, idx = built(60000, 128, 96, "sqeuclidean", 60000 + 128)
    q = _mixture(200, 128, 11)
    _search(idx, q, 2000, 24)
    st = idx.last_search_stats()
    assert st["scan_kernel"] == 13 and st["candidates"] >= 200 * 2000, st
    assert st["window_candidates"] >= (200 - st["overflow_queries"]) * 2000, st
    assert st["overflow_queries"] <= 20, st
