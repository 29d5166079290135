"""Pin the CPU oracle (oracle/mivs_oracle.c) against the golden fixtures before trusting it.

The fixtures (tests/golden/, made by make_golden.py) come from the reference itself (its shard
arithmetic, its merge fixtures, its sample embeddings) and from the reference's own CPU
baselines (sklearn NearestNeighbors(brute), Lloyd k-means). ANN numerics are otherwise unpinned
by the reference (cuVS/FAISS are not vendored), so these are the anchors.
"""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_oracle_knn_matches_sklearn_on_reference_sample_embeddings():
    g = np.load(os.path.join(GOLD, "knn_sample_embeddings.npz"))
    x = g["x"]
    d, i = O.knn(x, x, int(g["k"]))
    np.testing.assert_array_equal(i, g["ids"])
    np.testing.assert_allclose(d, g["sqdist"], atol=1e-5)
    assert (i[:, 0] == np.arange(x.shape[0])).all() and (d[:, 0] == 0).all()


def test_oracle_knn_matches_sklearn_synthetic_10k():
    g = np.load(os.path.join(GOLD, "knn_synthetic_10k.npz"))
    rng = np.random.default_rng(int(g["seed"]))
    x = rng.standard_normal((int(g["n"]), int(g["d"]))).astype(np.float32)
    q = rng.standard_normal((int(g["nq"]), int(g["d"]))).astype(np.float32)
    d, i = O.knn(x, q, int(g["k"]))
    np.testing.assert_array_equal(i, g["ids"])
    np.testing.assert_allclose(d, g["sqdist"], rtol=1e-5)


def test_oracle_kmeans_matches_sklearn_lloyd():
    g = np.load(os.path.join(GOLD, "kmeans.npz"))
    rng = np.random.default_rng(int(g["seed"]))
    centers = rng.standard_normal((40, 64)).astype(np.float32) * 3
    lab = rng.integers(0, 40, 20_000)
    x = (centers[lab] + rng.standard_normal((20_000, 64)).astype(np.float32)).astype(np.float32)
    assert (np.bincount(O.kmeans_assign(x, g["c0"]), minlength=40) > 0).all()
    c = O.kmeans_fit(x, g["c0"], int(g["iters"]))
    np.testing.assert_allclose(c, g["centroids"], atol=1e-4)
    np.testing.assert_array_equal(O.kmeans_assign(x, c), g["labels"])


@pytest.mark.parametrize("case", ["single_gpu", "two_gpus"])
def test_oracle_merge_matches_reference_fixtures(case):
    fx = _json("merge.json")[case]
    d = np.asarray(fx["distances"], np.float32).transpose(1, 0, 2)  # [shard, q, k] -> [q, shard, k]
    i = np.asarray(fx["indices"], np.int64).transpose(1, 0, 2)
    od, oi = O.merge(d, i, fx["k"])
    np.testing.assert_array_equal(od, fx["expected_distances"])
    np.testing.assert_array_equal(oi, fx["expected_indices"])


def test_oracle_ivf_full_probe_is_exact():
    rng = np.random.default_rng(5)
    x = rng.standard_normal((3000, 48)).astype(np.float32)
    q = rng.standard_normal((40, 48)).astype(np.float32)
    c, sizes, ids = O.ivf_build(x, 12, iters=4)
    assert sizes.sum() == 3000 and sorted(ids.tolist()) == list(range(3000))
    d1, i1, _ = O.ivf_search(x, c, sizes, ids, q, 12, 7)
    d2, i2 = O.knn(x, q, 7)
    np.testing.assert_array_equal(i1, i2)
    np.testing.assert_array_equal(d1, d2)


def test_oracle_lists_are_stable_and_assigned_to_nearest_centroid():
    rng = np.random.default_rng(6)
    x = rng.standard_normal((2000, 32)).astype(np.float32)
    c = x[::100].copy()
    sizes, ids = O.ivf_lists(x, c)
    lab = O.kmeans_assign(x, c)
    off = np.concatenate([[0], np.cumsum(sizes)])
    for l in range(c.shape[0]):
        members = ids[off[l]:off[l + 1]]
        assert (np.diff(members) > 0).all()
        assert (lab[members] == l).all()


def test_oracle_ties_broken_by_id_and_missing_padded():
    x = np.zeros((5, 8), np.float32)
    d, i = O.knn(x, np.zeros((1, 8), np.float32), 8)
    np.testing.assert_array_equal(i[0], [0, 1, 2, 3, 4, -1, -1, -1])
    assert np.isinf(d[0, 5:]).all() and (d[0, :5] == 0).all()


def test_fast_cpu_baseline_agrees_with_oracle():
    rng = np.random.default_rng(8)
    x = rng.standard_normal((4000, 96)).astype(np.float32)
    q = rng.standard_normal((30, 96)).astype(np.float32)
    _, i1 = O.knn(x, q, 10)
    _, i2 = O.fast_knn(x, q, 10)
    assert (i1 == i2).mean() > 0.99
    c, sizes, ids = O.ivf_build(x, 16, iters=3)
    rows = x[ids]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    _, e, _ = O.ivf_search(x, c, sizes, ids, q, 4, 10)
    _, f = O.fast_ivf_search(rows, ids, off, c, q, 4, 10)
    assert (e == f).mean() > 0.99


def test_distribute_workload_matches_reference_outputs():
    """G1: shard boundaries from the imported reference module (gpu_resource_manager.py:170-233)."""
    from gpu_resource_manager import GPUResourceManager

    fx = _json("distribute_workload.json")
    for case in fx["even"]:
        m = GPUResourceManager.__new__(GPUResourceManager)
        m.available_gpus = list(range(case["gpus"]))
        assert [list(r) for r in m.distribute_workload(case["n"])] == case["ranges"], case
    mb = fx["memory_based"]
    m = GPUResourceManager.__new__(GPUResourceManager)
    m.available_gpus = [0, 1]
    m.gpu_memory_info = {g: {"available": a} for g, a in enumerate(mb["available"])}
    assert [list(r) for r in m.distribute_workload(mb["n"], "memory_based")] == mb["ranges"]
