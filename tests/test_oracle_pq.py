"""CPU checks of the IVF-PQ oracle restatement (oracle/mivs_oracle.c orc_ivfpq_*).

No reference fixture pins PQ numerics (cuVS is not importable here: parity unpinned beyond the
Lloyd k-means the codebooks are trained with, which test_oracle_golden.py pins against sklearn).
These tests check the restatement against an independent numpy formulation of the same algorithm.
"""
import numpy as np

import oracle as O


def _data(n, d, seed):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((12, d)).astype(np.float32) * 2
    return (c[rng.integers(0, 12, n)] + rng.standard_normal((n, d)).astype(np.float32) * 0.5).astype(np.float32)


def test_codes_are_nearest_codebook_entries():
    x = _data(3000, 24, 1)
    cents, cbs, sizes, ids, codes = O.ivfpq_build(x, 6, pq_dim=8, iters=4, max_per_code=8)
    pl = O.pq_len(24, 8)
    assert cbs.shape == (8, 256, pl) and codes.shape == (3000, 8)
    # label of each stored row = its list; residual sub-vectors -> argmin over the codebook
    lab = np.repeat(np.arange(6), sizes)
    r = (x[ids] - cents[lab]).reshape(3000, 8, pl).astype(np.float64)
    dist = ((r[:, :, None, :] - cbs[None].astype(np.float64)) ** 2).sum(-1)  # [n, pq_dim, 256]
    best = dist.argmin(-1)
    agree = (best == codes).mean()
    assert agree > 0.995, agree  # fp32 vs fp64 near-ties only


def test_full_probe_search_ranks_by_pq_distance():
    x = _data(2500, 32, 2)
    q = _data(15, 32, 3)
    cents, cbs, sizes, ids, codes = O.ivfpq_build(x, 5, pq_dim=16, iters=3, max_per_code=8)
    d, i, p = O.ivfpq_search(cents, cbs, sizes, ids, codes, q, 5, 10)
    pl = O.pq_len(32, 16)
    lab = np.repeat(np.arange(5), sizes)
    recon = (cents[lab].reshape(-1, 16, pl) + cbs[np.arange(16)[None, :], codes]).reshape(-1, 32)
    # PQ distance of (q, row) = || (q - c_l) - (x_hat - c_l) ||^2 = || q - x_hat ||^2
    ref = ((q[:, None, :].astype(np.float64) - recon[None].astype(np.float64)) ** 2).sum(-1)
    order = np.argsort(ref, axis=1, kind="stable")[:, :10]
    np.testing.assert_allclose(d, np.take_along_axis(ref, order, 1), rtol=1e-4, atol=1e-4)
    assert (ids[order] == i).mean() > 0.95


def test_full_probe_inner_product_ranks_by_q_dot_reconstruction():
    """metric inner_product: key = -(q . c_l) - sum_j q_j . B_j[code_j] = -(q . x_hat); distances out are
    the inner products q . x_hat, in descending order."""
    x = _data(2500, 32, 4)
    q = _data(15, 32, 5)
    cents, cbs, sizes, ids, codes = O.ivfpq_build(x, 5, pq_dim=16, iters=3, max_per_code=8)
    d, i, p = O.ivfpq_search(cents, cbs, sizes, ids, codes, q, 5, 10, metric="inner_product")
    pl = O.pq_len(32, 16)
    lab = np.repeat(np.arange(5), sizes)
    recon = (cents[lab].reshape(-1, 16, pl) + cbs[np.arange(16)[None, :], codes]).reshape(-1, 32)
    ref = q.astype(np.float64) @ recon.astype(np.float64).T
    order = np.argsort(-ref, axis=1, kind="stable")[:, :10]
    np.testing.assert_allclose(d, np.take_along_axis(ref, order, 1), rtol=1e-4, atol=1e-4)
    assert (np.diff(d, axis=1) <= 0).all()
    assert (ids[order] == i).mean() > 0.95
    # probes rank the centroids by inner product
    cp = np.argsort(-(q.astype(np.float64) @ cents.astype(np.float64).T), axis=1, kind="stable")
    np.testing.assert_array_equal(p, cp[:, :5])
