"""The cosine metric (sklearn cosine_similarity / NearestNeighbors(metric=
'cosine') at Attempt_1/VectorSearch_QuestionRetrieval.ipynb:839,878): rows and queries normalised on
the device with the pinned norm, inner-product ranking, distance 1 - ip. Bit-exact vs the oracle
(oracle.normalize_rows / cosine_knn / ivf_search over the normalised rows).
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _rows(n, d, seed, zero_rows=()):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, d)) * rng.uniform(0.01, 30.0, (n, 1))).astype(np.float32)
    for r in zero_rows:
        x[r] = 0.0
    return x


@pytest.mark.parametrize("d", [1, 3, 64, 130, 768])
def test_normalize_rows_bitexact(mivs_lib, d):
    from mivs import _cosine

    x = _rows(513, d, d, zero_rows=(0, 77))
    got = _cosine.normalize_rows(torch.from_numpy(x).cuda()).cpu().numpy()
    want = O.normalize_rows(x)
    np.testing.assert_array_equal(_bits(got), _bits(want))
    assert not got[0].any() and not got[77].any()


@pytest.mark.parametrize("k", [1, 10, 64])
def test_brute_force_cosine(mivs_lib, k):
    from mivs.neighbors import brute_force

    x, q = _rows(4000, 96, 1, zero_rows=(5,)), _rows(70, 96, 2)
    idx = brute_force.build(torch.from_numpy(x).cuda(), metric="cosine", ids_offset=9)
    d, i = brute_force.search(idx, torch.from_numpy(q).cuda(), k)
    od, oi = O.cosine_knn(x, q, k, id_offset=9)
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(d.cpu().numpy()), _bits(od))
    assert (np.diff(d.cpu().numpy(), axis=1) >= 0).all()  # distances ascending
    # ranking agrees with a float64 cosine distance up to near-ties
    xn = x / np.maximum(np.linalg.norm(x.astype(np.float64), axis=1, keepdims=True), 1e-300)
    qn = q / np.linalg.norm(q.astype(np.float64), axis=1, keepdims=True)
    ref = 1.0 - qn @ xn.T
    np.testing.assert_allclose(d.cpu().numpy(), np.sort(ref, axis=1)[:, :k], atol=1e-5)


@pytest.mark.parametrize("prefilter", [True, False])
def test_ivf_flat_cosine(mivs_lib, prefilter):
    from mivs.neighbors import ivf_flat, streaming

    x, q = _rows(9000, 64, 3), _rows(120, 64, 4)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=24, kmeans_n_iters=4, metric="cosine"),
                         torch.from_numpy(x).cuda())
    idx.set_prefilter(prefilter)
    sp = ivf_flat.SearchParams(n_probes=6)
    d, i = ivf_flat.search(sp, idx, torch.from_numpy(q).cuda(), 10)
    xn, qn = O.normalize_rows(x), O.normalize_rows(q)
    np.testing.assert_array_equal(_bits(idx.list_rows().cpu().numpy()),
                                  _bits(xn[idx.list_ids().cpu().numpy()]))
    od, oi, _ = O.ivf_search(xn, idx.centers.cpu().numpy(), idx.list_sizes.numpy(), idx.list_ids().cpu().numpy(),
                             qn, 6, 10, metric="inner_product")
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(d.cpu().numpy()), _bits(np.float32(1.0) - od))
    sd, si = streaming.search_host(idx, q, 10, sp, batch_size=50)
    np.testing.assert_array_equal(si.numpy(), oi)
    np.testing.assert_array_equal(_bits(sd.numpy()), _bits(d.cpu().numpy()))


def test_ivf_flat_cosine_extend_and_merge(mivs_lib):
    from mivs import ops
    from mivs.neighbors import ivf_flat

    x, q = _rows(5000, 32, 5), _rows(40, 32, 6)
    cents = _rows(12, 32, 7)
    full = ivf_flat.build_from_centroids(torch.from_numpy(cents).cuda(), torch.from_numpy(x).cuda(), metric="cosine")
    part = ivf_flat.build_from_centroids(torch.from_numpy(cents).cuda(), torch.from_numpy(x[:2000]).cuda(),
                                         metric="cosine")
    ivf_flat.extend(part, torch.from_numpy(x[2000:]).cuda())
    sp = ivf_flat.SearchParams(n_probes=4)
    d0, i0 = ivf_flat.search(sp, full, torch.from_numpy(q).cuda(), 8)
    d1, i1 = ivf_flat.search(sp, part, torch.from_numpy(q).cuda(), 8)
    np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d0.cpu().numpy()))
    # two "shards" merged: cosine distances merge smallest-first
    md, mi = ops.merge_topk(torch.stack([d0, d0 + 0.5], 1), torch.stack([i0, i0 + 100000], 1), 8, metric="cosine")
    np.testing.assert_array_equal(mi.cpu().numpy(), i0.cpu().numpy())
