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


def test_round_f16_matches_numpy_half():
    """orc_round_f16 (the fp16 LUT rounding of orc_ivfpq_search_ex): round to nearest even, subnormals, overflow to
    inf -- equal to numpy's float32 -> float16 -> float32 on every sampled value"""
    rng = np.random.default_rng(11)
    v = np.concatenate([
        rng.standard_normal(50000).astype(np.float32) * np.float32(10.0) ** rng.integers(-8, 6, 50000),
        np.float32([0.0, -0.0, 65504.0, 65519.99, 65520.0, -65520.0, 6.1e-5, 5.96e-8, 2.98e-8, 1e-9, 1e30]),
        # halfway cases: odd and even mantissas at several exponents
        ((np.arange(1, 2000, dtype=np.float32) + 0.5) * np.float32(2.0 ** -10)).astype(np.float32),
    ]).astype(np.float32)
    got = np.array([O.round_f16(t) for t in v.tolist()], dtype=np.float32)
    with np.errstate(over="ignore"):
        ref = v.astype(np.float16).astype(np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_fp16_lut_search_sums_rounded_entries():
    """lut_fp16: each distance = sum over subspaces of the fp16-rounded LUT entry, accumulated in fp32; the
    ranking stays close to the fp32 LUT's"""
    x = _data(2500, 32, 6)
    q = _data(15, 32, 7)
    cents, cbs, sizes, ids, codes = O.ivfpq_build(x, 5, pq_dim=8, iters=3, max_per_code=8)
    d32, i32, _ = O.ivfpq_search(cents, cbs, sizes, ids, codes, q, 5, 10)
    d16, i16, _ = O.ivfpq_search(cents, cbs, sizes, ids, codes, q, 5, 10, lut_fp16=True)
    pl = O.pq_len(32, 8)
    lab = np.repeat(np.arange(5), sizes)
    pos = {int(r): j for j, r in enumerate(ids)}
    for qi in range(15):
        for c in range(10):
            row = pos[int(i16[qi, c])]
            r = (q[qi] - cents[lab[row]]).reshape(8, pl)
            lut = ((r - cbs[np.arange(8), codes[row]]) ** 2).sum(-1).astype(np.float32)
            ref = np.float64(lut.astype(np.float16).astype(np.float32)).sum()
            assert abs(d16[qi, c] - ref) <= 2e-3 * max(1.0, abs(ref)), (qi, c, d16[qi, c], ref)
    assert (i16 == i32).mean() > 0.8
    assert np.abs(d16 - d32).max() < 0.05 * np.abs(d32).max()
