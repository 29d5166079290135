"""The reference's Python API contract on the drop-in modules.

Written from the reference's test suites (Attempt_1/test_*.py): same fakes (Mock(spec=...)
GPU managers, patched torch.cuda, the CUVS_AVAILABLE simulation switch), same messages and
golden values. CPU-only: no test here touches a GPU.
"""
import logging
from unittest.mock import MagicMock, Mock, patch

import numpy as np
import pytest
import torch

logging.disable(logging.CRITICAL)

from embedding_distribution_manager import DistributedEmbeddings, EmbeddingDistributionManager, EmbeddingPart  # noqa: E402
from gpu_resource_manager import GPUConfig, GPUResourceManager, MultiGPUConfig  # noqa: E402
from index_building_coordinator import (CoordinatedIndexBuild, IndexBuildConfig, IndexBuildingCoordinator,  # noqa: E402
                                        IndexBuildResult)
from search_result_aggregator import (AggregatedSearchResult, SearchConfig, SearchResult,  # noqa: E402
                                      SearchResultAggregator, combine_search_results,
                                      filter_search_results_by_distance)


def _mgr(gpus=(0, 1)):
    m = GPUResourceManager.__new__(GPUResourceManager)
    m.available_gpus = list(gpus)
    m.gpu_memory_info = {g: {"available": 16 * 2**30} for g in gpus}
    m.gpu_configs = []
    return m


@pytest.fixture
def mock_mgr():
    m = Mock(spec=GPUResourceManager)
    m.get_available_gpu_ids.return_value = [0, 1]
    m.validate_gpu_index.side_effect = lambda g: g in (0, 1)
    m.get_safe_device_string.side_effect = lambda g: f"cuda:{g}"
    m.distribute_workload.return_value = [(0, 0, 50), (1, 50, 100)]
    m.get_gpu_memory_info.return_value = {"allocated": 1 << 20, "reserved": 2 << 20, "total": 16 << 30,
                                          "free": 14 << 30}
    m.cleanup_gpu_resources.return_value = None
    return m


# ---------------- GPUResourceManager (gpu_resource_manager.py) ----------------
class TestGPUResourceManager:
    def test_discovery_without_gpu(self):
        with patch("torch.cuda.is_available", return_value=False), patch("torch.cuda.device_count", return_value=0):
            m = GPUResourceManager()
        assert m.available_gpus == [] and m.gpu_configs == [] and m.get_available_gpu_count() == 0

    @pytest.mark.parametrize("count", [1, 2, 8])
    def test_discovery_with_patched_devices(self, count):
        props = MagicMock()
        props.name, props.total_memory = "AMD Instinct MI355X", 288 * 2**30
        dev = MagicMock()
        dev.return_value.__enter__ = MagicMock()
        dev.return_value.__exit__ = MagicMock()
        with patch("torch.cuda.is_available", return_value=True), \
                patch("torch.cuda.device_count", return_value=count), \
                patch("torch.cuda.get_device_properties", return_value=props), \
                patch("torch.cuda.memory_allocated", return_value=2**30), \
                patch("torch.cuda.empty_cache"), patch("torch.cuda.device", dev):
            m = GPUResourceManager()
        assert m.available_gpus == list(range(count))
        assert m.gpu_configs[0].device_name == "AMD Instinct MI355X" and m.gpu_configs[0].is_available
        assert m.gpu_memory_info[0]["available"] == 287 * 2**30

    def test_validate_and_device_strings(self):
        m = _mgr()
        assert not m.validate_gpu_index(-1)
        assert not m.validate_gpu_index(2)
        with patch("torch.cuda.is_available", return_value=False):
            assert not m.validate_gpu_index(0)
        with patch("torch.cuda.is_available", return_value=True), patch("torch.cuda.device_count", return_value=1):
            assert not m.validate_gpu_index(1)
        with patch("torch.cuda.is_available", return_value=True), patch("torch.cuda.device_count", return_value=2):
            assert m.validate_gpu_index(1)
            assert m.get_safe_device_string(1) == "cuda:1"
        with pytest.raises(ValueError, match=r"Invalid GPU index: 2\. Available GPUs: \[0, 1\]"):
            m.get_safe_device_string(2)

    def test_distribute_workload_golden(self):
        m = _mgr((0, 1, 2))
        assert m.distribute_workload(300) == [(0, 0, 100), (1, 100, 200), (2, 200, 300)]
        assert m.distribute_workload(301) == [(0, 0, 101), (1, 101, 201), (2, 201, 301)]

    def test_distribute_workload_memory_based_covers_everything(self):
        m = _mgr((0, 1))
        m.gpu_memory_info = {0: {"available": 8 * 2**30}, 1: {"available": 16 * 2**30}}
        assert m.distribute_workload(300, "memory_based") == [(0, 0, 100), (1, 100, 300)]
        m.gpu_memory_info = {0: {"available": 3}, 1: {"available": 3}, }
        m.available_gpus = [0, 1]
        r = m.distribute_workload(7, "memory_based")
        assert sum(e - s for _, s, e in r) == 7  # the reference dropped the truncation remainder

    def test_distribute_workload_errors(self):
        with pytest.raises(RuntimeError, match="No GPUs available"):
            _mgr(()).distribute_workload(10)
        for bad in (0, -10):
            with pytest.raises(ValueError):
                _mgr().distribute_workload(bad)
        with pytest.raises(ValueError, match="Unknown distribution strategy"):
            _mgr().distribute_workload(100, strategy="unknown")

    def test_cleanup_and_memory_info(self):
        m = _mgr((0, 1))
        props = MagicMock()
        props.total_memory = 16 * 2**30
        with patch("torch.cuda.is_available", return_value=True), patch("torch.cuda.device_count", return_value=2), \
                patch("torch.cuda.empty_cache") as ec, patch("torch.cuda.synchronize") as sy, \
                patch("torch.cuda.device"), patch("torch.cuda.memory_allocated", return_value=2 * 2**30), \
                patch("torch.cuda.memory_reserved", return_value=4 * 2**30), \
                patch("torch.cuda.get_device_properties", return_value=props):
            m.cleanup_gpu_resources()
            assert ec.call_count == 2 and sy.call_count == 2
            info = m.get_gpu_memory_info(0)
        assert (info["allocated"], info["reserved"], info["total"], info["free"]) == \
               (2 * 2**30, 4 * 2**30, 16 * 2**30, 12 * 2**30)
        with pytest.raises(ValueError):
            _mgr((0,)).get_gpu_memory_info(1)

    def test_multi_config_tensor_distribution_repr(self):
        m = _mgr((0, 1))
        m.gpu_configs = [GPUConfig(0, "MI355X", 1, 1, True), GPUConfig(1, "MI355X", 1, 1, True)]
        cfg = m.get_multi_gpu_config("even")
        assert isinstance(cfg, MultiGPUConfig) and cfg.primary_gpu == 0 and len(cfg.available_gpus) == 2
        assert _mgr(()).get_multi_gpu_config().primary_gpu == -1
        t0, t1, t2 = MagicMock(), MagicMock(), MagicMock()
        t0.device.index, t1.device.index, t2.device.index = 0, 1, 2
        assert m.validate_tensor_distribution([t0, t1])
        assert not m.validate_tensor_distribution([t0])
        assert not m.validate_tensor_distribution([t0, t2])
        assert "available_gpus=[0, 1]" in str(m) and "gpu_count=2" in str(m)
        assert "gpu_configs=2" in repr(m)


# ---------------- EmbeddingDistributionManager ----------------
class TestEmbeddingDistribution:
    def test_part_validation(self):
        t = torch.randn(10, 8)
        assert EmbeddingPart(0, t, 0, 10).num_rows == 10
        for kw, msg in [(dict(start_index=-1, end_index=10), "start_index must be non-negative"),
                        (dict(start_index=10, end_index=5), "end_index .* must be greater than start_index"),
                        (dict(gpu_id=-1, start_index=0, end_index=10), "gpu_id must be non-negative"),
                        (dict(start_index=0, end_index=20), r"Tensor size.*doesn't match index range")]:
            args = dict(gpu_id=0, tensor=t)
            args.update(kw)
            with pytest.raises(ValueError, match=msg):
                EmbeddingPart(**args)

    def test_distributed_validation(self):
        p1, p2 = EmbeddingPart(0, torch.randn(50, 8), 0, 50), EmbeddingPart(1, torch.randn(50, 8), 50, 100)
        assert DistributedEmbeddings([p1, p2], 100, 8).total_size == 100
        with pytest.raises(ValueError, match="parts list cannot be empty"):
            DistributedEmbeddings([], 100, 8)
        with pytest.raises(ValueError, match="total_size must be positive"):
            DistributedEmbeddings([p1], 0, 8)
        with pytest.raises(ValueError, match="has embedding_dim.*expected"):
            DistributedEmbeddings([p1, EmbeddingPart(1, torch.randn(50, 4), 50, 100)], 100, 8)
        with pytest.raises(ValueError, match="Gap or overlap detected"):
            DistributedEmbeddings([p1, EmbeddingPart(1, torch.randn(40, 8), 60, 100)], 100, 8)
        with pytest.raises(ValueError, match="Gap or overlap detected"):
            DistributedEmbeddings([EmbeddingPart(0, torch.randn(60, 8), 0, 60), p2], 100, 8)

    def test_input_errors(self, mock_mgr):
        m = EmbeddingDistributionManager(mock_mgr)
        with pytest.raises(TypeError, match="embeddings must be a torch.Tensor"):
            m.distribute_embeddings("no")
        with pytest.raises(ValueError, match="embeddings must be 2D tensor"):
            m.distribute_embeddings(torch.randn(10))
        with pytest.raises(ValueError, match="embeddings tensor cannot be empty"):
            m.distribute_embeddings(torch.empty(0, 8))
        with pytest.raises(ValueError, match="Target GPU.*is not available"):
            m.distribute_embeddings(torch.randn(10, 8), target_gpus=[5])
        mock_mgr.get_available_gpu_ids.return_value = []
        with pytest.raises(RuntimeError, match="No GPUs available"):
            m.distribute_embeddings(torch.randn(10, 8))
        with pytest.raises(TypeError):
            EmbeddingDistributionManager(object())

    def test_validate_distribution_variants(self, mock_mgr):
        m = EmbeddingDistributionManager(mock_mgr)

        def mk(dev_str=None, dtype=None, idx=0, rows=50, use_shape=True):
            t = Mock()
            t.device = Mock()
            if dev_str is not None:
                t.device.__str__ = Mock(return_value=dev_str)
            else:
                t.device.type, t.device.index = dtype, idx
            if use_shape:
                t.shape = (rows, 8)
            else:
                t.size.side_effect = lambda dim: rows if dim == 0 else 8
            return t

        good = DistributedEmbeddings([EmbeddingPart(0, mk("cuda:0"), 0, 50), EmbeddingPart(1, mk("cuda:1"), 50, 100)],
                                     100, 8)
        assert m.validate_distribution(good)
        typed = DistributedEmbeddings([EmbeddingPart(0, mk(dtype="cuda", idx=0, rows=100, use_shape=False), 0, 100)],
                                      100, 8)
        assert m.validate_distribution(typed)
        cpu = DistributedEmbeddings([EmbeddingPart(0, mk("cpu", rows=100), 0, 100)], 100, 8)
        assert not m.validate_distribution(cpu)
        mock_mgr.validate_gpu_index.side_effect = lambda g: False
        assert not m.validate_distribution(typed)
        mock_mgr.validate_gpu_index.side_effect = lambda g: True
        mock_mgr.get_available_gpu_ids.return_value = []
        assert not m.validate_distribution(good)

    def test_summary_memory_cleanup_repr(self, mock_mgr):
        m = EmbeddingDistributionManager(mock_mgr)
        assert "has_current_distribution=False" in repr(m) and "EmbeddingDistributionManager" in str(m)
        p1, p2 = EmbeddingPart(0, torch.randn(50, 8), 0, 50), EmbeddingPart(1, torch.randn(50, 8), 50, 100)
        d = DistributedEmbeddings([p1, p2], 100, 8)
        assert m.get_total_memory_usage(d) == {0: 1600, 1: 1600} == m.get_total_gpu_memory_usage(d)
        assert m.get_embedding_part_by_gpu(d, 1) is p2 and m.get_embedding_part_by_gpu(d, 5) is None
        s = m.get_distribution_summary(d)
        assert (s["total_embeddings"], s["embedding_dimension"], s["num_gpus"], s["gpu_ids"], s["part_sizes"]) == \
               (100, 8, 2, [0, 1], [50, 50])
        assert "memory_usage_bytes" in s and "memory_usage_mb" in s
        m.current_distribution = d
        m.cleanup_distribution(d)
        mock_mgr.cleanup_gpu_resources.assert_called_once_with([0, 1])
        assert m.current_distribution is None
        m.cleanup_distribution()  # nothing current: no-op

    def test_redistribute_noop_and_target_subset_split(self, mock_mgr):
        m = EmbeddingDistributionManager(mock_mgr)
        p1, p2 = EmbeddingPart(0, torch.randn(50, 8), 0, 50), EmbeddingPart(1, torch.randn(50, 8), 50, 100)
        d = DistributedEmbeddings([p1, p2], 100, 8)
        assert m.redistribute_if_needed(d) is d
        assert m._split(101, [1]) == [(1, 0, 101)]  # a subset now covers N (reference bug :139-141)
        assert m._split(10, [0, 1, 3]) == [(0, 0, 4), (1, 4, 7), (3, 7, 10)]


# ---------------- IndexBuildingCoordinator (simulation mode, like the reference's tests) ----------------
@pytest.fixture
def parts():
    return DistributedEmbeddings([EmbeddingPart(0, torch.randn(500, 16), 0, 500),
                                  EmbeddingPart(1, torch.randn(500, 16), 500, 1000)], 1000, 16)


class TestIndexBuildingCoordinator:
    def test_dataclasses(self):
        assert IndexBuildResult(0, object(), 1.5, True, memory_usage_bytes=1024).success
        for kw, msg in [(dict(gpu_id=-1), "gpu_id must be non-negative"), (dict(build_time=-1.0),
                         "build_time must be non-negative"), (dict(index=None), "index cannot be None"),
                        (dict(success=False, index=None), "error_message cannot be None")]:
            a = dict(gpu_id=0, index=object(), build_time=1.0, success=True)
            a.update(kw)
            with pytest.raises(ValueError, match=msg):
                IndexBuildResult(**a)
        c = IndexBuildConfig("ivf_flat", {"n_lists": 100}, {"nprobe": 10}, True, 3, 60.0)
        assert c.search_params == {"nprobe": 10}
        for kw, msg in [(dict(index_type="hnsw"), "index_type must be one of"),
                        (dict(index_params="x"), "index_params must be a dictionary"),
                        (dict(max_retries=-1), "max_retries must be non-negative"),
                        (dict(timeout_seconds=0), "timeout_seconds must be positive")]:
            a = dict(index_type="ivf_flat", index_params={})
            a.update(kw)
            with pytest.raises(ValueError, match=msg):
                IndexBuildConfig(**a)
        r0 = IndexBuildResult(0, object(), 1.0, True)
        r1 = IndexBuildResult(1, None, 0.0, False, "oom")
        cb = CoordinatedIndexBuild([r0, r1], 2.5, False, [1], [0], c)
        assert cb.failed_gpus == [1]
        with pytest.raises(ValueError, match="build_results cannot be empty"):
            CoordinatedIndexBuild([], 1.0, True, [], [], c)
        with pytest.raises(ValueError, match="failed_gpus and successful_gpus must match"):
            CoordinatedIndexBuild([r0], 1.0, True, [], [0, 1], c)

    @pytest.mark.parametrize("parallel", [False, True])
    def test_simulated_builds(self, mock_mgr, parts, parallel):
        with patch("index_building_coordinator.CUVS_AVAILABLE", False), patch("torch.cuda.is_available",
                                                                              return_value=False):
            co = IndexBuildingCoordinator(mock_mgr)
            r = co.build_indices_parallel(parts, IndexBuildConfig("ivf_flat", {"n_lists": 10},
                                                                  parallel_build=parallel, max_retries=1))
        assert r.success and sorted(r.successful_gpus) == [0, 1] and set(co.built_indices) == {0, 1}
        assert co.get_build_summary()["gpu_success_rates"] == {0: 1.0, 1: 1.0}

    def test_failure_and_retry(self, mock_mgr, parts):
        with patch("index_building_coordinator.CUVS_AVAILABLE", False), patch("torch.cuda.is_available",
                                                                              return_value=False), \
                patch("time.sleep"):
            co = IndexBuildingCoordinator(mock_mgr)
            mock_mgr.validate_gpu_index.side_effect = lambda g: g == 0
            r = co.build_indices_parallel(parts, IndexBuildConfig("ivf_flat", {}, parallel_build=False,
                                                                  max_retries=1))
            assert not r.success and r.failed_gpus == [1] and list(co.built_indices) == [0]
            calls = {"n": 0}

            def flaky(g):
                if g == 0:
                    return True
                calls["n"] += 1
                return calls["n"] > 1

            mock_mgr.validate_gpu_index.side_effect = flaky
            r = co.build_indices_parallel(parts, IndexBuildConfig("ivf_flat", {}, parallel_build=False,
                                                                  max_retries=2))
            assert r.success and len(r.successful_gpus) == 2

    def test_validation_bookkeeping_and_repr(self, mock_mgr):
        co = IndexBuildingCoordinator(mock_mgr)
        with patch("index_building_coordinator.CUVS_AVAILABLE", False):
            assert co.validate_index_build(0, {"type": "ivf_flat", "size": 100, "dim": 8}, torch.randn(100, 8))
            assert not co.validate_index_build(0, None, torch.randn(100, 8))
            assert not co.validate_index_build(0, {"size": 50, "dim": 8}, torch.randn(100, 8))
        co.built_indices.update({0: {"m": 1}, 1: {"m": 1}})
        co._active_builds.update({0: True, 1: True})
        co.cleanup_failed_builds([1])
        assert 0 in co.built_indices and 1 not in co.built_indices and 1 not in co._active_builds
        assert co.get_built_indices() == {0: {"m": 1}} and co.get_built_indices() is not co.built_indices
        assert co.get_index_for_gpu(1) is None
        co._active_builds = {0: True, 1: False, 2: True}
        assert co.has_active_builds() and set(co.get_active_build_gpus()) == {0, 2}
        co._active_builds = {0: True}
        assert "built_indices=1" in str(co) and "active_builds=1" in str(co) and "built_indices=[0]" in repr(co)
        co.built_indices[1] = {"m": 2}
        co.cleanup_all_indices()
        assert co.built_indices == {} and co._active_builds == {}
        mock_mgr.cleanup_gpu_resources.assert_called_with([0, 1])
        with pytest.raises(ValueError, match="distributed_embeddings must be a DistributedEmbeddings instance"):
            co.build_indices_parallel("x", IndexBuildConfig("ivf_flat", {}))

    def test_default_n_lists_and_unimplemented_types_fail_cleanly(self, mock_mgr):
        from mivs.neighbors.ivf_flat import default_n_lists

        assert [default_n_lists(n) for n in (1, 999, 1000, 255_000, 10**7)] == [1, 1, 2, 256, 256]


# ---------------- SearchResultAggregator (contract written from the reference tests) ----------------
def _sr(d, i, g=0, k=None):
    d, i = np.asarray(d, np.float32), np.asarray(i, np.int64)
    return SearchResult(d, i, g, 0.1, k or d.shape[1], k or d.shape[1])


class TestSearchResultAggregator:
    def test_types(self):
        with pytest.raises(ValueError, match="gpu_id must be non-negative"):
            SearchResult(np.zeros((1, 2)), np.zeros((1, 2)), -1, 0.1, 2, 2)
        with pytest.raises(ValueError, match="query_time must be non-negative"):
            SearchResult(np.zeros((1, 2)), np.zeros((1, 2)), 0, -0.1, 2, 2)
        with pytest.raises(ValueError, match="k_requested must be positive"):
            SearchResult(np.zeros((1, 2)), np.zeros((1, 2)), 0, 0.1, 0, 2)
        with pytest.raises(ValueError, match="k_returned.*cannot exceed k_requested"):
            SearchResult(np.zeros((1, 2)), np.zeros((1, 2)), 0, 0.1, 1, 2)
        with pytest.raises(ValueError, match="distances shape.*!= indices shape"):
            SearchResult(np.zeros((1, 2)), np.zeros((1, 3)), 0, 0.1, 2, 2)
        with pytest.raises(ValueError, match="distances must be 2D array"):
            SearchResult(np.zeros(2), np.zeros(2), 0, 0.1, 2, 2)
        r = _sr([[1.0, 2.0]], [[10, 20]])
        with pytest.raises(ValueError, match="k_requested must be positive"):
            AggregatedSearchResult(r.distances, r.indices, 0.2, [r], 0, 2, 1)
        with pytest.raises(ValueError, match="num_queries must be positive"):
            AggregatedSearchResult(r.distances, r.indices, 0.2, [r], 2, 2, 0)
        c = SearchConfig(k=10, search_params={"nprobe": 32}, parallel_search=True, timeout_seconds=30.0)
        assert c.search_params == {"nprobe": 32}
        with pytest.raises(ValueError, match="k must be positive"):
            SearchConfig(k=0)
        with pytest.raises(ValueError, match="timeout_seconds must be positive"):
            SearchConfig(k=10, timeout_seconds=-1.0)

    def test_validate_and_merge_golden(self, mock_mgr):
        a = SearchResultAggregator(mock_mgr)
        assert a.search_history == [] and a._active_searches == {}
        assert a.validate_search_results([_sr([[1, 2], [3, 4]], [[1, 2], [3, 4]]),
                                          _sr([[0.5, 1.5], [2.5, 3.5]], [[5, 15], [25, 35]], g=1)], 2, 2)
        with pytest.raises(ValueError, match="gpu_results cannot be empty"):
            a.validate_search_results([], 2, 2)
        with pytest.raises(ValueError, match="contains NaN distances"):
            a.validate_search_results([_sr([[np.nan, 2.0]], [[10, 20]])], 1, 2)
        d, i = a.merge_search_results([_sr([[1, 2, 3], [4, 5, 6]], [[10, 20, 30], [40, 50, 60]])], k=2)
        np.testing.assert_array_equal(d, [[1, 2], [4, 5]])
        np.testing.assert_array_equal(i, [[10, 20], [40, 50]])
        d, i = a.merge_search_results([_sr([[2, 4], [6, 8]], [[20, 40], [60, 80]]),
                                       _sr([[1, 3], [5, 7]], [[10, 30], [50, 70]], g=1)], k=3)
        np.testing.assert_array_equal(d, [[1, 2, 3], [5, 6, 7]])
        np.testing.assert_array_equal(i, [[10, 20, 30], [50, 60, 70]])
        with pytest.raises(ValueError, match="Cannot merge empty results list"):
            a.merge_search_results([], k=5)
        with pytest.raises(ValueError, match="has.*queries, expected"):
            a.merge_search_results([_sr([[1, 2]], [[10, 20]]), _sr([[1, 2], [3, 4]], [[1, 2], [3, 4]], g=1)], k=2)
        d, i = combine_search_results([_sr([[3, 1]], [[7, 8]])], 5)  # width clamps to min(k, available)
        assert d.shape == (1, 2)

    def test_ties_broken_by_id_not_position(self, mock_mgr):
        a = SearchResultAggregator(mock_mgr)
        d, i = a.merge_search_results([_sr([[1.0, 1.0]], [[9, 3]]), _sr([[1.0]], [[5]], g=1)], k=3)
        np.testing.assert_array_equal(i, [[3, 5, 9]])

    def test_filter_by_distance(self):
        r = filter_search_results_by_distance(_sr([[0.5, 1.5, 2.5]], [[1, 2, 3]]), 1.5)
        np.testing.assert_array_equal(r.indices, [[1, 2, -1]])
        assert np.isinf(r.distances[0, 2]) and r.k_returned == 2

    @patch("search_result_aggregator.CUVS_AVAILABLE", False)
    def test_simulated_search_and_history(self, mock_mgr):
        a = SearchResultAggregator(mock_mgr)
        d, i = a._simulate_search(torch.randn(2, 128), k=5)
        assert d.shape == (2, 5) and i.shape == (2, 5) and (d >= 0).all() and (i >= 0).all()
        assert (d[:, :-1] <= d[:, 1:]).all()
        for parallel in (False, True):
            r = a.perform_distributed_search(torch.randn(2, 128), {0: Mock(), 1: Mock()},
                                             SearchConfig(k=3, parallel_search=parallel))
            assert isinstance(r, AggregatedSearchResult) and r.num_queries == 2 and r.k_requested == 3
            assert len(r.gpu_results) == 2 and r.final_distances.shape == (2, 3) and r.final_indices.shape == (2, 3)
            assert (np.diff(r.final_distances, axis=1) >= 0).all()
        assert len(a.get_search_history()) == 2
        a.clear_search_history()
        assert a.get_search_history() == []
        a._active_searches[0] = True
        act = a.get_active_searches()
        act[1] = True
        assert a.get_active_searches() == {0: True}
        a._active_searches.clear()
        assert "history_size=0" in str(a) and "active_searches=0" in repr(a)

    def test_search_input_errors(self, mock_mgr):
        a = SearchResultAggregator(mock_mgr)
        cfg = SearchConfig(k=5)
        with pytest.raises(ValueError, match="query must be a torch.Tensor"):
            a.perform_distributed_search("x", {0: Mock()}, cfg)
        with pytest.raises(ValueError, match="query must be 2D tensor"):
            a.perform_distributed_search(torch.randn(8), {0: Mock()}, cfg)
        with pytest.raises(ValueError, match="query cannot be empty"):
            a.perform_distributed_search(torch.empty(0, 8), {0: Mock()}, cfg)
        with pytest.raises(ValueError, match="indices dictionary cannot be empty"):
            a.perform_distributed_search(torch.randn(2, 8), {}, cfg)
        mock_mgr.validate_gpu_index.side_effect = lambda g: False
        with pytest.raises(ValueError, match="GPU 99 in indices is not available"):
            a.perform_distributed_search(torch.randn(2, 8), {99: Mock()}, cfg)


def test_streaming_rejects_unknown_index():
    """streaming.search_host checks the index kind before touching the GPU."""
    from mivs.neighbors import streaming

    with pytest.raises(TypeError, match="ivf_flat, ivf_pq or brute_force"):
        streaming.search_host(object(), np.zeros((2, 4), np.float32), 1)
