"""K13's staggered group transitions give the same bits as the round-4 kernel.

A workgroup scans a segment of one list (a run of its 256-row items) with its eight waves changing row groups at
different tiles, a wave's first group split into two parts. Every (row group, query tile) pair must still be scanned
exactly once, whatever the segment lengths, phases and the static / dynamic split of the work. The index here is
large enough for segments of several items per workgroup and for lists of ~10 query tiles (the benchmark's shape);
n_probes 2 gives lists of 1-3 tiles (no split groups). Each result is compared bitwise with the round-4 kernel
(MIVS_RS_STAGGER=0), with the exact fp32 scan for every query, and with the oracle on a query sample.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


@pytest.fixture(scope="module")
def data(mivs_lib):
    from mivs import ops

    x = ops.synth_mixture(400_000, 768, 3, n_centers=4096, sigma=0.75, device=0)
    q = ops.synth_mixture(2000, 768, 3, n_centers=4096, sigma=0.75, row_begin=1 << 40, device=0)
    yield x, q
    del x, q
    torch.cuda.empty_cache()


@pytest.fixture(scope="module", params=["sqeuclidean", "inner_product"])
def index(request, data):
    from mivs.neighbors import ivf_flat

    x, _ = data
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=48, kmeans_n_iters=6, metric=request.param), x)
    yield idx, request.param
    idx.close()


def _search(idx, q, n_probes, k=10):
    from mivs.neighbors import ivf_flat

    d, i = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, q, k)
    return d.cpu().numpy(), i.cpu().numpy()


@pytest.mark.parametrize("n_probes", [8, 2])
def test_stagger_equals_round4_kernel_and_exact(index, data, monkeypatch, n_probes):
    idx, metric = index
    x, q = data
    d0, i0 = _search(idx, q, n_probes)
    st = idx.last_search_stats()
    assert st["prefilter"] == 1 and st["scan_kernel"] == 13 and st["overflow_queries"] == 0, st
    for env in ({"MIVS_RS_STAGGER": "0"},      # round-4 kernel: items, all waves change groups together
                {"MIVS_RS_STAGGER": "1024"},   # every item in the static ranges (no dynamic tail)
                {"MIVS_RS_STAGGER": "2"},      # almost every item dealt dynamically (one-item segments)
                {"MIVS_RS_FLAGS": "24"}):      # block and phase clocks (stderr only)
        for kk, v in env.items():
            monkeypatch.setenv(kk, v)
        d1, i1 = _search(idx, q, n_probes)
        for kk in env:
            monkeypatch.delenv(kk)
        np.testing.assert_array_equal(i1, i0, err_msg=str(env))
        np.testing.assert_array_equal(_bits(d1), _bits(d0), err_msg=str(env))
    idx.set_prefilter(False)
    try:
        de, ie = _search(idx, q, n_probes)
    finally:
        idx.set_prefilter(True)
    np.testing.assert_array_equal(i0, ie)
    np.testing.assert_array_equal(_bits(d0), _bits(de))
    s = np.arange(0, q.shape[0], 50)
    od, oi, _ = O.ivf_search(x.cpu().numpy(), idx.centers.cpu().numpy(), idx.list_sizes.numpy(),
                             idx.list_ids().cpu().numpy(), q.cpu().numpy()[s], n_probes, 10, metric=metric)
    np.testing.assert_array_equal(i0[s], oi)
    np.testing.assert_array_equal(_bits(d0[s]), _bits(od))


def test_stagger_ragged_batches(index, data):
    """batches of 1..33 queries (lists of one tile, segments of single items) equal the full batch's rows"""
    idx, _ = index
    _, q = data
    d0, i0 = _search(idx, q[:200], 8)
    for a, b in ((0, 1), (1, 8), (8, 41), (41, 200)):
        d1, i1 = _search(idx, q[a:b], 8)
        np.testing.assert_array_equal(i1, i0[a:b])
        np.testing.assert_array_equal(_bits(d1), _bits(d0[a:b]))
