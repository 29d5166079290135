"""End-to-end on the GPU through the drop-in managers: discover -> distribute -> coordinated build ->
distributed search + device merge, checked bit-exact against the oracle."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def test_coordinator_and_aggregator_real_engine(mivs_lib):
    import index_building_coordinator as ibc
    import search_result_aggregator as sra
    from embedding_distribution_manager import EmbeddingDistributionManager
    from gpu_resource_manager import GPUResourceManager

    assert ibc.CUVS_AVAILABLE and sra.CUVS_AVAILABLE
    rng = np.random.default_rng(9)
    x = rng.standard_normal((20000, 64)).astype(np.float32)
    q = rng.standard_normal((33, 64)).astype(np.float32)
    gm = GPUResourceManager()
    assert gm.get_available_gpu_count() >= 1
    dm = EmbeddingDistributionManager(gm)
    dist = dm.distribute_embeddings(torch.from_numpy(x), target_gpus=[0])
    assert dm.validate_distribution(dist) and dist.parts[0].tensor.is_cuda
    co = ibc.IndexBuildingCoordinator(gm)
    res = co.build_indices_parallel(dist, ibc.IndexBuildConfig("ivf_flat", {"n_lists": 20, "kmeans_n_iters": 3},
                                                               parallel_build=False, max_retries=0))
    assert res.success, res.build_results[0].error_message
    agg = sra.SearchResultAggregator(gm)
    out = agg.perform_distributed_search(torch.from_numpy(q), co.get_built_indices(),
                                         sra.SearchConfig(k=10, search_params={"nprobe": 6}))
    oc, osz, oids = O.ivf_build(x, 20, iters=3)
    od, oi, _ = O.ivf_search(x, oc, osz, oids, q, 6, 10)
    np.testing.assert_array_equal(out.final_indices, oi)
    np.testing.assert_array_equal(out.final_distances.view(np.int32), od.view(np.int32))
    assert out.num_queries == 33 and out.k_returned == 10
    co.cleanup_all_indices()
    dm.cleanup_distribution()


def test_aggregator_brute_force_index_and_host_merge_api(mivs_lib):
    import index_building_coordinator as ibc
    import search_result_aggregator as sra
    from embedding_distribution_manager import EmbeddingDistributionManager
    from gpu_resource_manager import GPUResourceManager

    rng = np.random.default_rng(10)
    x = rng.standard_normal((3000, 40)).astype(np.float32)
    q = rng.standard_normal((9, 40)).astype(np.float32)
    gm = GPUResourceManager()
    dist = EmbeddingDistributionManager(gm).distribute_embeddings(torch.from_numpy(x), target_gpus=[0])
    co = ibc.IndexBuildingCoordinator(gm)
    assert co.build_indices_parallel(dist, ibc.IndexBuildConfig("brute_force", {}, parallel_build=False)).success
    agg = sra.SearchResultAggregator(gm)
    out = agg.perform_distributed_search(torch.from_numpy(q), co.get_built_indices(), sra.SearchConfig(k=7))
    ed, ei = O.knn(x, q, 7)
    np.testing.assert_array_equal(out.final_indices, ei)
    # merge_search_results (numpy contract API) runs the K7 device merge when the engine is present
    r0 = sra.SearchResult(np.array([[2, 4], [6, 8]], np.float32), np.array([[20, 40], [60, 80]]), 0, 0.1, 2, 2)
    r1 = sra.SearchResult(np.array([[1, 3], [5, 7]], np.float32), np.array([[10, 30], [50, 70]]), 1, 0.1, 2, 2)
    d, i = agg.merge_search_results([r0, r1], 3)
    np.testing.assert_array_equal(i, [[10, 20, 30], [50, 60, 70]])


def test_improved_driver_main_small(mivs_lib):
    import improved_multi_gpu_rag as imr

    out = imr.main(num_vectors_per_gpu=20000, dim=128, n_queries=16, top_k=20)
    assert out["build"]["success"] and out["recall"] > 0.5


def test_coordinator_ivf_pq_seam(mivs_lib):
    """index_type 'ivf_pq' through the coordinator (reference :398-404 defaults) and the aggregator,
    bit-exact against the oracle's IVF-PQ restatement."""
    import index_building_coordinator as ibc
    import search_result_aggregator as sra
    from embedding_distribution_manager import EmbeddingDistributionManager
    from gpu_resource_manager import GPUResourceManager

    rng = np.random.default_rng(12)
    x = rng.standard_normal((8000, 64)).astype(np.float32)
    q = rng.standard_normal((21, 64)).astype(np.float32)
    gm = GPUResourceManager()
    dm = EmbeddingDistributionManager(gm)
    dist = dm.distribute_embeddings(torch.from_numpy(x), target_gpus=[0])
    co = ibc.IndexBuildingCoordinator(gm)
    cfg = ibc.IndexBuildConfig("ivf_pq", {"n_lists": 16, "kmeans_n_iters": 3, "max_train_points_per_pq_code": 16},
                               parallel_build=False, max_retries=0)
    res = co.build_indices_parallel(dist, cfg)
    assert res.success, res.build_results[0].error_message
    idx = co.get_built_indices()[0]
    assert idx.pq_dim == 16 and idx.pq_bits == 8  # min(64, d // 4)
    agg = sra.SearchResultAggregator(gm)
    out = agg.perform_distributed_search(torch.from_numpy(q), co.get_built_indices(),
                                         sra.SearchConfig(k=10, search_params={"nprobe": 5}))
    oc, ocb, osz, oids, ocodes = O.ivfpq_build(x, 16, 16, iters=3, max_per_code=16)
    od, oi, _ = O.ivfpq_search(oc, ocb, osz, oids, ocodes, q, 5, 10)
    np.testing.assert_array_equal(out.final_indices, oi)
    np.testing.assert_array_equal(out.final_distances.view(np.int32), od.view(np.int32))
    co.cleanup_all_indices()
    dm.cleanup_distribution()


def test_parallel_index_builder_and_search_engine_bitexact_vs_oracle(mivs_lib):
    """§8 row a2: ParallelIndexBuilder.build_indices_parallel (one build per GPU on the thread pool,
    improved_multi_gpu_rag.py:108-190 upstream) and ParallelSearchEngine.parallel_search through the
    engine equal the oracle's IVF-Flat build (centroids, list sizes, list ids) and search (ids, distance
    bits), and the brute-force seam equals the oracle's exact kNN -- on every GPU of the box (one here)."""
    import improved_multi_gpu_rag as imr

    n_gpus = torch.cuda.device_count()
    rng = np.random.default_rng(31)
    n, d, nq, k = 6000 * n_gpus, 96, 40, 15
    x = rng.standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    parts = np.array_split(x, n_gpus)
    builder = imr.ParallelIndexBuilder(num_gpus=n_gpus)
    res = builder.build_indices_parallel([torch.from_numpy(p) for p in parts], imr.IndexType.IVF_FLAT,
                                         {"n_lists": 24, "kmeans_n_iters": 5})
    assert not res.get("failed_gpus"), res
    offs = np.concatenate([[0], np.cumsum([p.shape[0] for p in parts])])
    oracle_shards = [O.ivf_build(p, 24, iters=5, id_offset=int(offs[g])) for g, p in enumerate(parts)]
    for g, (oc, osz, oids) in enumerate(oracle_shards):
        idx = res["indexes"][g]
        np.testing.assert_array_equal(idx.centers.cpu().numpy().view(np.int32), oc.view(np.int32))
        np.testing.assert_array_equal(idx.list_sizes.numpy(), osz)
        np.testing.assert_array_equal(idx.list_ids().cpu().numpy(), oids)
    cfg = imr.SearchConfig(top_k=k, n_probes=6)
    eng = imr.ParallelSearchEngine(res["indexes"], imr.IndexType.IVF_FLAT, cfg)
    dd, ii = eng.parallel_search(torch.from_numpy(q).cuda())
    # the oracle: every shard's top-k, merged by (distance, id)
    per = [O.ivf_search(p, *oracle_shards[g], q, 6, k, id_offset=int(offs[g]))[:2] for g, p in enumerate(parts)]
    md, mi = O.merge(np.stack([r[0] for r in per], axis=1), np.stack([r[1] for r in per], axis=1), k)
    np.testing.assert_array_equal(np.asarray(ii), mi)
    np.testing.assert_array_equal(np.asarray(dd, dtype=np.float32).view(np.int32), md.view(np.int32))
    # brute-force seam
    resb = builder.build_indices_parallel([torch.from_numpy(p) for p in parts], imr.IndexType.BRUTE_FORCE, {})
    engb = imr.ParallelSearchEngine(resb["indexes"], imr.IndexType.BRUTE_FORCE, cfg)
    bd, bi = engb.parallel_search(torch.from_numpy(q).cuda())
    ed, ei = O.knn(x, q, k)
    np.testing.assert_array_equal(np.asarray(bi), ei)
    np.testing.assert_array_equal(np.asarray(bd, dtype=np.float32).view(np.int32), ed.view(np.int32))
