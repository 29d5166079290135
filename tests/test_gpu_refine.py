"""K14 exact re-ranking (cuvs.neighbors.refine) and the IVF-PQ + refine pipeline.

``refine`` ranks each query's candidate rows by the pinned fp32 key: bit-exact with
``oracle.refine`` (oracle/mivs_oracle.c orc_refine), for fp32 and fp16 datasets, L2 and inner product,
with missing (-1) candidates. Over an IVF-PQ candidate pool it gives back exact distances, and over the
whole dataset it is exact k-NN.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


@pytest.mark.parametrize("n,d,nq,nc,k,metric,half", [
    (5000, 64, 37, 50, 10, "sqeuclidean", False),
    (3000, 100, 20, 64, 16, "inner_product", False),   # d % 8 != 0: scalar tail
    (4000, 768, 25, 120, 10, "sqeuclidean", True),     # fp16 dataset (BASELINE config 5)
    (2000, 32, 9, 8, 8, "sqeuclidean", False),         # k = n_candidates
    (6000, 128, 11, 200, 64, "inner_product", True),
    (3000, 1024, 9, 70, 10, "sqeuclidean", True),      # fp16 rows past dp 768: K14g without the next-pass prefetch
    (2500, 1000, 7, 45, 12, "inner_product", False),   # fp32, dp 1024 > d: two 64-dim block rounds, padding blocks
])
def test_refine_bitexact_vs_oracle(mivs_lib, n, d, nq, nc, k, metric, half):
    from mivs.neighbors import refine

    rng = np.random.default_rng(n + d + nc)
    x = rng.standard_normal((n, d)).astype(np.float32)
    if half:
        x = x.astype(np.float16).astype(np.float32)  # the values an fp16 dataset holds
    q = rng.standard_normal((nq, d)).astype(np.float32)
    cand = np.stack([rng.choice(n, nc, replace=False) for _ in range(nq)]).astype(np.int64)
    cand[rng.random(cand.shape) < 0.1] = -1
    xd = torch.from_numpy(x).cuda()
    dist, ids = refine(xd.half() if half else xd, torch.from_numpy(q).cuda(), torch.from_numpy(cand).cuda(), k,
                       metric=metric)
    od, oi = O.refine(x, q, cand, k, metric)
    np.testing.assert_array_equal(ids.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(dist.cpu().numpy()), _bits(od))


def test_refine_over_all_rows_is_exact_knn(mivs_lib):
    from mivs.neighbors import brute_force, refine

    rng = np.random.default_rng(3)
    x = rng.standard_normal((300, 48)).astype(np.float32)
    q = rng.standard_normal((7, 48)).astype(np.float32)
    cand = np.tile(np.arange(300, dtype=np.int64)[::-1], (7, 1))
    d1, i1 = refine(torch.from_numpy(x).cuda(), q, cand, 12)
    d2, i2 = brute_force.search(brute_force.build(torch.from_numpy(x).cuda()), torch.from_numpy(q).cuda(), 12)
    np.testing.assert_array_equal(i1.cpu().numpy(), i2.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d2.cpu().numpy()))


def test_ivf_pq_then_refine_recall(mivs_lib):
    """cuVS's IVF-PQ + refine pattern: PQ top-64 candidates re-ranked exactly. The refined answer equals
    the oracle's refine of the oracle's PQ candidates, and beats the plain PQ top-10 on recall."""
    from mivs import ops
    from mivs.neighbors import brute_force, ivf_pq, refine

    x = ops.synth_mixture(40000, 128, 5, n_centers=512, sigma=0.5)
    q = ops.synth_mixture(100, 128, 5, n_centers=512, sigma=0.5, row_begin=1 << 40)
    idx = ivf_pq.build(ivf_pq.IndexParams(n_lists=64, pq_dim=16, kmeans_n_iters=4), x)
    sp = ivf_pq.SearchParams(n_probes=16)
    _, cand = ivf_pq.search(sp, idx, q, 64)
    rd, ri = refine(x, q, cand, 10)
    od, oi = O.refine(x.cpu().numpy(), q.cpu().numpy(), cand.cpu().numpy(), 10)
    np.testing.assert_array_equal(ri.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(rd.cpu().numpy()), _bits(od))
    _, pq10 = ivf_pq.search(sp, idx, q, 10)
    _, gt = brute_force.search(brute_force.build(x), q, 10)
    gt = gt.cpu().numpy()
    rec = lambda f: np.mean([len(set(a) & set(b)) / 10 for a, b in zip(f, gt)])  # noqa: E731
    assert rec(ri.cpu().numpy()) >= rec(pq10.cpu().numpy())
    assert rec(ri.cpu().numpy()) > 0.8


def test_refine_cuvs_argument_order_and_k_from_indices(mivs_lib):
    """cuVS's order refine(dataset, queries, candidates, k=None, indices=None, distances=None,
    metric=...); k omitted -> indices.shape[1]; k > 64 is refused rather than silently capped"""
    from mivs.neighbors import refine

    rng = np.random.default_rng(4)
    x = torch.from_numpy(rng.standard_normal((3000, 64)).astype(np.float32)).cuda()
    q = torch.from_numpy(rng.standard_normal((9, 64)).astype(np.float32)).cuda()
    cand = torch.from_numpy(np.stack([rng.choice(3000, 80, replace=False) for _ in range(9)])).cuda()
    d0, i0 = refine(x, q, cand, 8)
    ib = torch.empty((9, 8), dtype=torch.int64, device="cuda")
    db = torch.empty((9, 8), dtype=torch.float32, device="cuda")
    d1, i1 = refine(x, q, cand, None, ib, db)
    assert torch.equal(i1, i0) and torch.equal(ib, i0) and torch.equal(db, d0)
    with pytest.raises(ValueError):
        refine(x, q, cand, 65)
