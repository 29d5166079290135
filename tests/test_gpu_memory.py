"""Device memory at the API boundary (VERDICT r05 missing #3 / next #2): an index's HBM comes back through the
reference's own cleanup paths.

The engine's block cache (capi_util.hpp BlockCache) is opt-in; with it off an index's memory goes back
to the driver on close(), with it on the blocks are kept until a cleanup path -- GPUResourceManager.cleanup_gpu_resources
(reference Attempt_1/gpu_resource_manager.py:235-255), IndexBuildingCoordinator.cleanup_all_indices /
cleanup_failed_builds (Attempt_1/index_building_coordinator.py:472-497,583-603), CUDAMemoryManager's OOM handler
(Latest/cuVS-2-gpu/improved_multi_gpu_rag.py:74-97) -- hands them back. Either way torch.cuda.mem_get_info()
returns to within 1 GB of its pre-build value and torch can allocate the index's footprint.
"""
import gc

import pytest
import torch

pytestmark = pytest.mark.gpu

GB = 1 << 30


def _corpus(n=10_000_000, d=768):
    from mivs import ops

    return ops.synth_mixture(n, d, 0, n_centers=65536, sigma=0.75, device=0)


def _free():
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info(0)[0]


def _check_torch_can_take(nbytes):
    t = torch.empty(int(nbytes) // 4, dtype=torch.float32, device="cuda:0")
    t[-1] = 1.0
    torch.cuda.synchronize()
    del t
    torch.cuda.empty_cache()


@pytest.fixture
def cache_off(mivs_lib):
    from mivs import _native

    _native.set_block_cache_limit(0)
    yield
    _native.set_block_cache_limit(0)


def test_10m_close_returns_memory_without_cache(cache_off):
    """default (cache off): close() alone gives the index's ~54 GB back"""
    from gpu_resource_manager import GPUResourceManager
    from mivs import _native
    from mivs.neighbors import ivf_flat

    x = _corpus()
    free0 = _free()
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024, kmeans_n_iters=2), x)
    foot = idx.memory()["total_bytes"]
    assert foot > 40 * GB
    assert _free() < free0 - 40 * GB
    idx.close()
    assert _native.cached_memory(0)["bytes"] == 0
    assert _free() >= free0 - GB
    GPUResourceManager().cleanup_gpu_resources([0])
    _check_torch_can_take(foot)
    del x
    gc.collect()
    torch.cuda.empty_cache()


def test_10m_cached_blocks_released_by_reference_cleanup(cache_off):
    """cache on: close() keeps the blocks (invisible to torch), the coordinator's cleanup_all_indices -- through
    GPUResourceManager.cleanup_gpu_resources -- returns them, and torch can take the index's footprint"""
    import index_building_coordinator as ibc
    from gpu_resource_manager import GPUResourceManager
    from mivs import _native
    from mivs.neighbors import ivf_flat

    x = _corpus()
    free0 = _free()
    _native.set_block_cache_limit(96 * GB, 0)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024, kmeans_n_iters=2), x)
    foot = idx.memory()["total_bytes"]
    co = ibc.IndexBuildingCoordinator(GPUResourceManager())
    co.built_indices[0] = idx
    idx2 = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024, kmeans_n_iters=2), x)  # (a second, closed at once)
    idx2.close()
    held = _native.cached_memory(0)["bytes"]
    assert held > 20 * GB, held
    assert _free() < free0 - 40 * GB
    co.cleanup_all_indices()
    assert _native.cached_memory(0)["bytes"] == 0
    assert _free() >= free0 - GB
    _check_torch_can_take(foot)
    del x
    gc.collect()
    torch.cuda.empty_cache()


def test_oom_handler_releases_cached_blocks(cache_off):
    """CUDAMemoryManager.managed_allocation's OOM path returns the engine's cached blocks before torch's cache"""
    from improved_multi_gpu_rag import CUDAMemoryManager, GPUConfig
    from mivs import _native
    from mivs.neighbors import ivf_flat

    x = _corpus(2_000_000)
    _native.set_block_cache_limit(32 * GB, 0)
    ivf_flat.build(ivf_flat.IndexParams(n_lists=256, kmeans_n_iters=2), x).close()
    assert _native.cached_memory(0)["bytes"] > 0
    with pytest.raises(MemoryError):
        with CUDAMemoryManager.managed_allocation(GPUConfig(0), "test"):
            raise MemoryError("simulated OOM")
    assert _native.cached_memory(0)["bytes"] == 0
    del x
    torch.cuda.empty_cache()


def test_close_waits_for_own_stream_only(cache_off):
    """close() of one index waits for that index's calls (its done-events): results of a search enqueued on a side
    stream just before close() on another index are intact, and a cached block reused right after close() carries
    the same bits as a fresh build"""
    import numpy as np

    from mivs import _native
    from mivs.neighbors import ivf_flat

    x = _corpus(300_000, 256)
    q = x[:200].clone()
    p = ivf_flat.IndexParams(n_lists=64, kmeans_n_iters=3)
    _native.set_block_cache_limit(8 * GB, 0)
    a = ivf_flat.build(p, x)
    b = ivf_flat.build(p, x)
    d0, i0 = ivf_flat.search(ivf_flat.SearchParams(n_probes=8), a, q, 10)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        d1, i1 = ivf_flat.search(ivf_flat.SearchParams(n_probes=8), a, q, 10)
    b.close()  # (b's blocks go to the cache without a device-wide wait)
    c = ivf_flat.build(p, x)  # (takes b's blocks)
    side.synchronize()
    d2, i2 = ivf_flat.search(ivf_flat.SearchParams(n_probes=8), c, q, 10)
    torch.cuda.synchronize()
    for d, i in ((d1, i1), (d2, i2)):
        np.testing.assert_array_equal(i.cpu().numpy(), i0.cpu().numpy())
        np.testing.assert_array_equal(d.cpu().numpy().view(np.int32), d0.cpu().numpy().view(np.int32))
    a.close()
    c.close()
    assert _native.release_cached_memory(0) > 0
