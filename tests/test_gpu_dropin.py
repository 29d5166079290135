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
