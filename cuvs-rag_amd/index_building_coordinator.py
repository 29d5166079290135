"""Per-GPU index builds with retries, validation and history.

Drop-in for the reference's ``Attempt_1/index_building_coordinator.py``
(``IndexBuildingCoordinator`` at :106). The build seam ``_create_index`` (reference
:370-420) now calls the mivs HIP engine (``mivs.neighbors.ivf_flat.build``) instead of
``cuvs.neighbors.ivf_flat.build``; everything around it (dataclasses, thread-per-GPU
parallel build, retry with linear back-off, validation, history, cleanup, messages)
keeps the reference's contract so its tests and drivers run unchanged.

Differences: each shard's index is built with
``ids_offset = part.start_index`` so search results carry GLOBAL ids, and validating a
real index runs a self-query (a stored row must come back first at distance 0) instead
of only ``str(index)``.
"""
from __future__ import annotations

import gc
import logging
import time
from concurrent.futures import ThreadPoolExecutor, as_completed
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

import torch

from embedding_distribution_manager import DistributedEmbeddings, EmbeddingDistributionManager  # noqa: F401
from gpu_resource_manager import GPUResourceManager
from mivs.backend import engine_available

logger = logging.getLogger(__name__)

# "the mivs HIP engine is usable" (reference: "cuVS imported", :25-30); patchable by tests
CUVS_AVAILABLE = engine_available()

VALID_INDEX_TYPES = ["ivf_flat", "ivf_pq", "cagra", "brute_force"]
_IVF_FLAT_KEYS = ("metric", "kmeans_n_iters", "kmeans_trainset_fraction", "kmeans_max_train_per_list", "kmeans_balance",
                  "add_data_on_build", "chunk_rows")
_IVF_PQ_KEYS = ("metric", "kmeans_n_iters", "kmeans_trainset_fraction", "max_train_points_per_pq_code",
                "kmeans_balance", "add_data_on_build")


@dataclass
class IndexBuildResult:
    """Outcome of one GPU's build (reference :33-52)."""
    gpu_id: int
    index: Optional[Any]
    build_time: float
    success: bool
    error_message: Optional[str] = None
    memory_usage_bytes: int = 0

    def __post_init__(self):
        if self.gpu_id < 0:
            raise ValueError(f"gpu_id must be non-negative, got {self.gpu_id}")
        if self.build_time < 0:
            raise ValueError(f"build_time must be non-negative, got {self.build_time}")
        if self.success and self.index is None:
            raise ValueError("index cannot be None when success is True")
        if not self.success and self.error_message is None:
            raise ValueError("error_message cannot be None when success is False")


@dataclass
class IndexBuildConfig:
    """What to build (reference :55-75). ``index_params`` keys: 'n_lists', 'pq_bits', 'pq_dim',
    'intermediate_graph_degree', 'graph_degree' (+ mivs: 'kmeans_n_iters', 'kmeans_trainset_fraction',
    'metric', 'chunk_rows'); ``search_params`` key: 'nprobe'."""
    index_type: str
    index_params: Dict[str, Any]
    search_params: Optional[Dict[str, Any]] = None
    parallel_build: bool = True
    max_retries: int = 2
    timeout_seconds: Optional[float] = None

    def __post_init__(self):
        if self.index_type not in VALID_INDEX_TYPES:
            raise ValueError(f"index_type must be one of {VALID_INDEX_TYPES}, got {self.index_type}")
        if not isinstance(self.index_params, dict):
            raise ValueError("index_params must be a dictionary")
        if self.max_retries < 0:
            raise ValueError(f"max_retries must be non-negative, got {self.max_retries}")
        if self.timeout_seconds is not None and self.timeout_seconds <= 0:
            raise ValueError(f"timeout_seconds must be positive, got {self.timeout_seconds}")


@dataclass
class CoordinatedIndexBuild:
    """All GPUs' results of one coordinated build (reference :78-103)."""
    build_results: List[IndexBuildResult]
    total_build_time: float
    success: bool
    failed_gpus: List[int]
    successful_gpus: List[int]
    config: IndexBuildConfig

    def __post_init__(self):
        if not self.build_results:
            raise ValueError("build_results cannot be empty")
        if self.total_build_time < 0:
            raise ValueError(f"total_build_time must be non-negative, got {self.total_build_time}")
        ids = {r.gpu_id for r in self.build_results}
        failed, ok = set(self.failed_gpus), set(self.successful_gpus)
        if failed | ok != ids:
            raise ValueError("failed_gpus and successful_gpus must match build_results GPU IDs")
        if failed & ok:
            raise ValueError("failed_gpus and successful_gpus cannot overlap")


class IndexBuildingCoordinator:
    """Builds one index per corpus shard, one Python thread per GPU (native calls release the GIL)."""

    def __init__(self, gpu_manager: GPUResourceManager):
        self.gpu_manager = gpu_manager
        self.built_indices: Dict[int, Any] = {}
        self.build_history: List[CoordinatedIndexBuild] = []
        self._active_builds: Dict[int, bool] = {}

    # ---- orchestration ---------------------------------------------------------------------
    def build_indices_parallel(self, distributed_embeddings: DistributedEmbeddings,
                               config: IndexBuildConfig) -> CoordinatedIndexBuild:
        if not isinstance(distributed_embeddings, DistributedEmbeddings):
            raise ValueError("distributed_embeddings must be a DistributedEmbeddings instance")
        if not isinstance(config, IndexBuildConfig):
            raise ValueError("config must be an IndexBuildConfig instance")
        parts = distributed_embeddings.parts
        gpu_ids = [p.gpu_id for p in parts]
        logger.info("Building %s indices on %d GPU(s)", config.index_type, len(parts))
        self._cleanup_existing_indices(gpu_ids)
        self._active_builds.update({g: True for g in gpu_ids})
        t0 = time.time()
        try:
            if config.parallel_build and len(parts) > 1:
                results = self._build_parallel(distributed_embeddings, config)
            else:
                results = self._build_sequential(distributed_embeddings, config)
            ok = [r for r in results if r.success]
            bad = [r for r in results if not r.success]
            for r in ok:
                self.built_indices[r.gpu_id] = r.index
            coordinated = CoordinatedIndexBuild(build_results=results, total_build_time=time.time() - t0,
                                                success=not bad, failed_gpus=[r.gpu_id for r in bad],
                                                successful_gpus=[r.gpu_id for r in ok], config=config)
            self.build_history.append(coordinated)
            if bad:
                logger.warning("Index building failed on GPUs: %s", coordinated.failed_gpus)
                self.cleanup_failed_builds(coordinated.failed_gpus)
            return coordinated
        except Exception as e:
            logger.error("Index building coordination failed: %s", e)
            self._cleanup_existing_indices(gpu_ids)
            raise RuntimeError(f"Index building coordination failed: {e}") from e
        finally:
            for g in gpu_ids:
                self._active_builds.pop(g, None)

    def _build_parallel(self, distributed_embeddings: DistributedEmbeddings,
                        config: IndexBuildConfig) -> List[IndexBuildResult]:
        results: List[IndexBuildResult] = []
        with ThreadPoolExecutor(max_workers=len(distributed_embeddings.parts)) as pool:
            futures = {pool.submit(self._build_single_index, p, config): p for p in distributed_embeddings.parts}
            for fut in as_completed(futures, timeout=config.timeout_seconds):
                part = futures[fut]
                try:
                    results.append(fut.result())
                except Exception as e:
                    logger.error("GPU %s build failed with exception: %s", part.gpu_id, e)
                    results.append(IndexBuildResult(part.gpu_id, None, 0.0, False, str(e)))
        return results

    def _build_sequential(self, distributed_embeddings: DistributedEmbeddings,
                          config: IndexBuildConfig) -> List[IndexBuildResult]:
        return [self._build_single_index(p, config) for p in distributed_embeddings.parts]

    def _build_single_index(self, embedding_part, config: IndexBuildConfig) -> IndexBuildResult:
        """Build one shard's index; retries ``max_retries`` times with a 0.5*(attempt+1) s back-off."""
        gpu_id = embedding_part.gpu_id
        last_error = "Unexpected error in build loop"
        for attempt in range(config.max_retries + 1):
            try:
                if not self.gpu_manager.validate_gpu_index(gpu_id):
                    raise RuntimeError(f"GPU {gpu_id} is no longer available")
                t0 = time.time()
                offset = int(getattr(embedding_part, "start_index", 0))
                if CUVS_AVAILABLE and torch.cuda.is_available():
                    with torch.cuda.device(gpu_id):
                        index = self._create_index(embedding_part.tensor, config, id_offset=offset)
                else:
                    index = self._create_index(embedding_part.tensor, config, id_offset=offset)
                build_time = time.time() - t0
                try:
                    mem = self.gpu_manager.get_gpu_memory_info(gpu_id).get("allocated", 0)
                except Exception:
                    mem = 0
                if not self.validate_index_build(gpu_id, index, embedding_part.tensor):
                    raise RuntimeError("Index validation failed")
                return IndexBuildResult(gpu_id, index, build_time, True, memory_usage_bytes=mem)
            except Exception as e:
                last_error = f"GPU {gpu_id} build attempt {attempt + 1} failed: {e}"
                logger.warning(last_error)
                if attempt == config.max_retries:
                    break
                time.sleep(0.5 * (attempt + 1))
                try:
                    self.gpu_manager.cleanup_gpu_resources([gpu_id])
                except Exception as ce:
                    logger.warning("Cleanup failed on GPU %s: %s", gpu_id, ce)
        return IndexBuildResult(gpu_id, None, 0.0, False, last_error)

    # ---- the build seam (reference :370-420) -------------------------------------------------
    def _create_index(self, embeddings: torch.Tensor, config: IndexBuildConfig, id_offset: int = 0) -> Any:
        if not CUVS_AVAILABLE:
            logger.warning("mivs engine not available, simulating index build")
            time.sleep(0.1)
            return {"type": config.index_type, "size": embeddings.shape[0], "dim": embeddings.shape[1]}
        from mivs.neighbors import brute_force, ivf_flat, ivf_pq

        p = config.index_params
        try:
            if config.index_type == "ivf_flat":
                n_lists = p.get("n_lists", ivf_flat.default_n_lists(embeddings.shape[0]))
                extra = {k: p[k] for k in _IVF_FLAT_KEYS if k in p}
                return ivf_flat.build(ivf_flat.IndexParams(n_lists=n_lists, **extra), embeddings,
                                      ids_offset=id_offset)
            if config.index_type == "brute_force":
                return brute_force.build(embeddings, metric=p.get("metric", "sqeuclidean"), ids_offset=id_offset)
            if config.index_type == "ivf_pq":
                # reference :398-404: n_lists default as ivf_flat, pq_bits 8, pq_dim min(64, d // 4)
                n_lists = p.get("n_lists", ivf_flat.default_n_lists(embeddings.shape[0]))
                pq_bits = p.get("pq_bits", 8)
                pq_dim = p.get("pq_dim", ivf_pq.default_pq_dim(embeddings.shape[1]))
                extra = {k: p[k] for k in _IVF_PQ_KEYS if k in p}
                return ivf_pq.build(ivf_pq.IndexParams(n_lists=n_lists, pq_bits=pq_bits, pq_dim=pq_dim, **extra),
                                    embeddings, ids_offset=id_offset)
            if config.index_type == "cagra":
                raise NotImplementedError("cagra is not implemented in mivs (ivf_flat, ivf_pq and brute_force are; "
                                          "SURVEY.md §8(f))")
            raise ValueError(f"Unsupported index type: {config.index_type}")
        except Exception as e:
            raise RuntimeError(f"Failed to create {config.index_type} index: {e}") from e

    def validate_index_build(self, gpu_id: int, index: Any, original_embeddings: torch.Tensor) -> bool:
        try:
            if index is None:
                logger.error("Index on GPU %s is None", gpu_id)
                return False
            if not self.gpu_manager.validate_gpu_index(gpu_id):
                logger.error("GPU %s is no longer accessible", gpu_id)
                return False
            if not CUVS_AVAILABLE:
                if isinstance(index, dict):
                    return (index.get("size") == original_embeddings.shape[0]
                            and index.get("dim") == original_embeddings.shape[1])
                return False
            return self._self_query_ok(index, original_embeddings)
        except Exception as e:
            logger.error("Error during index validation on GPU %s: %s", gpu_id, e)
            return False

    @staticmethod
    def _self_query_ok(index: Any, embeddings: torch.Tensor) -> bool:
        """A stored row queried against its own index must come back at distance 0 (L2 indices)."""
        from mivs.neighbors import brute_force, ivf_flat, ivf_pq

        if getattr(index, "metric", "sqeuclidean") not in ("sqeuclidean", "l2", "L2Expanded"):
            return len(index) == embeddings.shape[0]
        n = embeddings.shape[0]
        if n == 0 or len(index) != n:
            return len(index) == n
        probe = embeddings[[0, n // 2, n - 1]]
        if isinstance(index, ivf_pq.Index):
            # PQ distances are approximate: the probe rows must come back with valid neighbours
            _, i = ivf_pq.search(ivf_pq.SearchParams(n_probes=min(4, index.n_lists)), index, probe, 1)
            i = i.tensor if hasattr(i, "tensor") else i
            return bool((torch.as_tensor(i).reshape(-1).cpu() >= 0).all())
        if isinstance(index, ivf_flat.Index):
            d, _ = ivf_flat.search(ivf_flat.SearchParams(n_probes=1), index, probe, 1)
        else:
            d, _ = brute_force.search(index, probe, 1)
        d = d.tensor if hasattr(d, "tensor") else d
        return bool((torch.as_tensor(d).reshape(-1).float().cpu() == 0).all())

    # ---- cleanup / bookkeeping ---------------------------------------------------------------
    def cleanup_failed_builds(self, failed_gpu_ids: List[int]) -> None:
        for g in failed_gpu_ids:
            self._release(g)
            self._active_builds.pop(g, None)
        try:
            self.gpu_manager.cleanup_gpu_resources(failed_gpu_ids)
        except Exception as e:
            logger.warning("Error during GPU memory cleanup: %s", e)

    def _release(self, gpu_id: int) -> None:
        idx = self.built_indices.pop(gpu_id, None)
        close = getattr(idx, "close", None)
        if callable(close):
            close()

    def _cleanup_existing_indices(self, gpu_ids: List[int]) -> None:
        for g in gpu_ids:
            if g in self.built_indices:
                self._release(g)

    def get_built_indices(self) -> Dict[int, Any]:
        return dict(self.built_indices)

    def get_index_for_gpu(self, gpu_id: int) -> Optional[Any]:
        return self.built_indices.get(gpu_id)

    def has_active_builds(self) -> bool:
        return any(self._active_builds.values())

    def get_active_build_gpus(self) -> List[int]:
        return [g for g, active in self._active_builds.items() if active]

    def get_build_summary(self) -> Dict[str, Any]:
        per_gpu: Dict[int, List[int]] = {}
        for build in self.build_history:
            for r in build.build_results:
                s = per_gpu.setdefault(r.gpu_id, [0, 0])
                s[0] += int(r.success)
                s[1] += 1
        return {
            "total_coordinated_builds": len(self.build_history),
            "successful_coordinated_builds": sum(1 for b in self.build_history if b.success),
            "current_built_indices": len(self.built_indices),
            "active_builds": len(self.get_active_build_gpus()),
            "gpu_success_rates": {g: (s[0] / s[1] if s[1] else 0) for g, s in per_gpu.items()},
        }

    def cleanup_all_indices(self) -> None:
        gpus = list(self.built_indices.keys())
        for g in gpus:
            self._release(g)
        self.built_indices.clear()
        self._active_builds.clear()
        if gpus:
            try:
                self.gpu_manager.cleanup_gpu_resources(gpus)
            except Exception as e:
                logger.warning("Error during final GPU cleanup: %s", e)
        gc.collect()

    def __str__(self) -> str:
        return (f"IndexBuildingCoordinator(built_indices={len(self.built_indices)}, "
                f"active_builds={len(self.get_active_build_gpus())}, gpu_manager={self.gpu_manager})")

    def __repr__(self) -> str:
        return (f"IndexBuildingCoordinator(gpu_manager={self.gpu_manager!r}, "
                f"built_indices={list(self.built_indices.keys())}, build_history={len(self.build_history)} builds)")
