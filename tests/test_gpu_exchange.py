"""The cross-shard exchange on the GPU: K7 over the rank-major all-gather buffer, the single-process
RCCL path (``mivs_comm_init_all`` / ``mivs_merge_topk_allgather``) and what the drivers build on it.

References: the merge contract (Attempt_1/test_search_result_aggregator.py:308-358, 405-457), the
host merge it replaces (Latest/cuVS-2-gpu/improved_multi_gpu_rag.py:239-277,
cuvs-2gpu-main.ipynb:1820-1834), the output hook (improved_multi_gpu_rag.py:111-114) and
batch_search (:279-303). The box has one GPU: the RCCL communicator is exercised with one rank, the
multi-rank buffer layout through ``mivs_merge_topk_gathered`` with up to 8 parts.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _shards(rng, parts, nq, k_in, metric):
    """parts sorted per-shard tiles with global ids (shard p owns ids [p*10^6, (p+1)*10^6)), some ties,
    some missing (-1) tail entries."""
    d = rng.integers(0, 50, size=(parts, nq, k_in)).astype(np.float32) / 4  # many exact ties
    i = rng.integers(0, 1_000_000, size=(parts, nq, k_in)).astype(np.int64) + (np.arange(parts) * 10**6)[:, None, None]
    for p in range(parts):
        for r in range(nq):
            o = np.lexsort((i[p, r], -d[p, r] if metric == "inner_product" else d[p, r]))
            d[p, r], i[p, r] = d[p, r, o], i[p, r, o]
    miss = rng.random((parts, nq)) < 0.2
    i[:, :, -1][miss] = -1
    d[:, :, -1][miss] = -np.inf if metric == "inner_product" else np.inf
    return d, i


@pytest.mark.parametrize("parts,k_in,k,metric", [(1, 10, 10, "sqeuclidean"), (4, 10, 10, "sqeuclidean"),
                                                 (8, 16, 10, "sqeuclidean"), (3, 20, 64, "inner_product"),
                                                 (8, 10, 70, "sqeuclidean"), (2, 100, 150, "inner_product")])
def test_merge_topk_gathered_matches_oracle(mivs_lib, parts, k_in, k, metric):
    from mivs import ops

    rng = np.random.default_rng(parts * 100 + k)
    nq = 97
    d, i = _shards(rng, parts, nq, k_in, metric)
    od, oi = ops.merge_topk_gathered(torch.from_numpy(d).cuda(), torch.from_numpy(i).cuda(), k, metric)
    ed, ei = O.merge(d.transpose(1, 0, 2), i.transpose(1, 0, 2), k, metric)
    np.testing.assert_array_equal(oi.cpu().numpy(), ei)
    np.testing.assert_array_equal(_bits(od.cpu().numpy()), _bits(ed))


def test_local_comm_one_rank_allgather_merge(mivs_lib):
    from mivs import ops
    from mivs.comm import LocalComm

    rng = np.random.default_rng(5)
    d, i = _shards(rng, 1, 300, 12, "sqeuclidean")
    dt, it = torch.from_numpy(d[0]).cuda(), torch.from_numpy(i[0]).cuda()
    comm = LocalComm([0])
    assert comm.size == 1
    for _ in range(3):  # reuse of the receive buffers across calls
        out = comm.merge_topk_allgather({0: dt}, {0: it}, 10)
    ed, ei = ops.merge_topk(dt, it, 10)
    np.testing.assert_array_equal(out[0][1].cpu().numpy(), ei.cpu().numpy())
    np.testing.assert_array_equal(_bits(out[0][0].cpu().numpy()), _bits(ed.cpu().numpy()))
    big = comm.merge_topk_allgather({0: dt}, {0: it}, 12)  # k = k_in: the whole tile back
    np.testing.assert_array_equal(big[0][1].cpu().numpy(), i[0])
    with pytest.raises(ValueError):
        comm.merge_topk_allgather({1: dt}, {1: it}, 10)
    comm.close()


def test_aggregator_rccl_exchange_bitexact_vs_oracle(mivs_lib):
    """perform_distributed_search with the RCCL exchange forced on (one GPU = one rank)."""
    import index_building_coordinator as ibc
    import search_result_aggregator as sra
    from embedding_distribution_manager import EmbeddingDistributionManager
    from gpu_resource_manager import GPUResourceManager

    rng = np.random.default_rng(19)
    x = rng.standard_normal((12000, 96)).astype(np.float32)
    q = rng.standard_normal((41, 96)).astype(np.float32)
    gm = GPUResourceManager()
    dm = EmbeddingDistributionManager(gm)
    dist = dm.distribute_embeddings(torch.from_numpy(x), target_gpus=[0])
    co = ibc.IndexBuildingCoordinator(gm)
    assert co.build_indices_parallel(dist, ibc.IndexBuildConfig("ivf_flat", {"n_lists": 24, "kmeans_n_iters": 3},
                                                                parallel_build=False, max_retries=0)).success
    agg = sra.SearchResultAggregator(gm)
    out = agg.perform_distributed_search(torch.from_numpy(q), co.get_built_indices(),
                                         sra.SearchConfig(k=10, search_params={"nprobe": 7}, exchange="rccl"))
    oc, osz, oids = O.ivf_build(x, 24, iters=3)
    od, oi, _ = O.ivf_search(x, oc, osz, oids, q, 7, 10)
    np.testing.assert_array_equal(out.final_indices, oi)
    np.testing.assert_array_equal(_bits(out.final_distances), _bits(od))
    assert out.gpu_results[0].distances.dtype == np.float32 and out.gpu_results[0].indices.dtype == np.int64
    co.cleanup_all_indices()
    dm.cleanup_distribution()


def test_aggregator_inner_product_merge_order(mivs_lib):
    """IP shards merge by descending inner product: device and host merges agree with the oracle."""
    import search_result_aggregator as sra
    from gpu_resource_manager import GPUResourceManager

    rng = np.random.default_rng(23)
    d, i = _shards(rng, 3, 17, 6, "inner_product")
    res = [sra.SearchResult(d[p], i[p], p, 0.1, 6, 6) for p in range(3)]
    agg = sra.SearchResultAggregator(GPUResourceManager())
    dd, ii = agg.merge_search_results(res, 9, metric="inner_product")
    ed, ei = O.merge(d.transpose(1, 0, 2), i.transpose(1, 0, 2), 9, "inner_product")
    np.testing.assert_array_equal(ii, ei)
    np.testing.assert_array_equal(_bits(dd), _bits(ed))
    hd, hi = sra._host_merge(np.concatenate(list(d), axis=1), np.concatenate(list(i), axis=1), 9, "inner_product")
    np.testing.assert_array_equal(hi, ei)


def test_aggregator_brute_force_ip_index(mivs_lib):
    import search_result_aggregator as sra
    from gpu_resource_manager import GPUResourceManager
    from mivs.neighbors import brute_force

    rng = np.random.default_rng(29)
    x = rng.standard_normal((5000, 64)).astype(np.float32)
    q = rng.standard_normal((13, 64)).astype(np.float32)
    bf = brute_force.build(torch.from_numpy(x).cuda(), metric="inner_product")
    agg = sra.SearchResultAggregator(GPUResourceManager())
    out = agg.perform_distributed_search(torch.from_numpy(q), {0: bf}, sra.SearchConfig(k=8, exchange="rccl"))
    ed, ei = O.knn(x, q, 8, "inner_product")
    np.testing.assert_array_equal(out.final_indices, ei)
    np.testing.assert_array_equal(_bits(out.final_distances), _bits(ed))


def test_parallel_search_engine_with_copy_to_host_hook_and_ragged_batches(mivs_lib):
    """The reference's driver flow: set_output_as(copy_to_host) (improved_multi_gpu_rag.py:114), then
    parallel_search and batch_search. 11 queries in batches of 5 leave a one-query tail: every
    result must still be a (k,) pair."""
    import improved_multi_gpu_rag as imr
    from mivs import config as mcfg
    from mivs.neighbors import ivf_flat

    rng = np.random.default_rng(31)
    x = rng.standard_normal((6000, 64)).astype(np.float32)
    q = rng.standard_normal((11, 64)).astype(np.float32)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=16, kmeans_n_iters=3), torch.from_numpy(x).cuda())
    cfg = imr.SearchConfig(top_k=7, search_batch_size=5, n_probes=16)
    eng = imr.ParallelSearchEngine({0: idx}, imr.IndexType.IVF_FLAT, cfg)
    mcfg.set_output_as(lambda a: a.copy_to_host())
    try:
        d1, i1 = eng.parallel_search(torch.from_numpy(q[0]))
        assert i1.shape == (7,)
        db, ib = eng.parallel_search(torch.from_numpy(q[:1]))
        assert ib.shape == (1, 7)
        out = eng.batch_search([torch.from_numpy(r) for r in q])
        # the hook is still the driver's after the worker searches
        assert isinstance(ivf_flat.search(ivf_flat.SearchParams(n_probes=16), idx, q[:2], 3)[0], np.ndarray)
    finally:
        mcfg.set_output_as("torch")
    assert len(out) == 11 and all(d.shape == (7,) and i.shape == (7,) for d, i in out)
    ed, ei = O.knn(x, q, 7)  # n_probes = n_lists: the exact answer
    np.testing.assert_array_equal(np.stack([i for _, i in out]), ei)
    np.testing.assert_array_equal(i1, ei[0])
    idx.close()


def test_recall_evaluator_exact_ground_truth_ip(mivs_lib):
    import improved_multi_gpu_rag as imr
    from mivs.neighbors import brute_force

    rng = np.random.default_rng(37)
    x = rng.standard_normal((3000, 32)).astype(np.float32)
    q = rng.standard_normal((9, 32)).astype(np.float32)
    qt = torch.from_numpy(q).cuda()
    parts = {}
    for p, (lo, hi) in enumerate([(0, 1400), (1400, 3000)]):
        bf = brute_force.build(torch.from_numpy(x[lo:hi]).cuda(), metric="inner_product", ids_offset=lo)
        parts[p] = brute_force.search(bf, qt, 5)
    # both "shards" live on cuda:0 here; exact_ground_truth merges whatever devices they are on
    gt = imr.RecallEvaluator.exact_ground_truth({0: parts[0], 1: parts[1]}, qt, 5, metric="inner_product")
    _, ei = O.knn(x, q, 5, "inner_product")
    np.testing.assert_array_equal(gt, ei)


def test_extend_default_ids_follow_ids_offset(mivs_lib):
    """extend without ids on a shard built with ids_offset keeps the shard's global range."""
    from mivs.neighbors import ivf_flat

    rng = np.random.default_rng(41)
    x = rng.standard_normal((4000, 64)).astype(np.float32)
    off = 1_000_000
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=8, kmeans_n_iters=2), torch.from_numpy(x[:3000]).cuda(),
                         ids_offset=off)
    ivf_flat.extend(idx, torch.from_numpy(x[3000:]).cuda())
    ids = np.sort(idx.list_ids().cpu().numpy())
    np.testing.assert_array_equal(ids, np.arange(off, off + 4000))
    d, i = ivf_flat.search(ivf_flat.SearchParams(n_probes=8), idx, x[3500:3510], 1)
    np.testing.assert_array_equal(i.cpu().numpy()[:, 0], np.arange(off + 3500, off + 3510))
    idx.close()


def test_brute_force_prefilter_overflow_falls_back_exactly(mivs_lib):
    """force the K11 overflow branch of brute force (300 identical rows next to every query:
    the refine window holds more candidates than it can prove) and check the fallback bit-exact."""
    from mivs.neighbors import brute_force

    rng = np.random.default_rng(43)
    x = rng.standard_normal((20000, 128)).astype(np.float32)
    v = rng.standard_normal(128).astype(np.float32)
    x[5000:5300] = v
    q = (v[None, :] + 1e-3 * rng.standard_normal((40, 128))).astype(np.float32)
    q = np.concatenate([q, rng.standard_normal((24, 128)).astype(np.float32)])
    bf = brute_force.build(torch.from_numpy(x).cuda())
    d, i = brute_force.search(bf, torch.from_numpy(q).cuda(), 10)
    st = bf.last_search_stats()
    assert st["prefilter"] == 1 and st["overflow_queries"] > 0, st
    ed, ei = O.knn(x, q, 10)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(_bits(d.cpu().numpy()), _bits(ed))
    d2, i2 = brute_force.search(bf, torch.from_numpy(q).cuda(), 20)  # exact path resets the pre-filter stats
    st2 = bf.last_search_stats()
    assert st2["prefilter"] == 0 and st2["overflow_queries"] == 0
    bf.close()
