"""Corpus sharding: split an N x D embedding matrix into contiguous per-GPU parts.

Drop-in for the reference's ``Attempt_1/embedding_distribution_manager.py``
(``EmbeddingDistributionManager`` at :73) — the corpus-shard boundary named by the
north star. The class, dataclasses, method names and messages are the union of the
reference implementation and its two test suites:
``get_total_memory_usage``/``get_total_gpu_memory_usage``, ``cleanup_distribution``/
``cleanup_current_distribution``, ``get_distribution_summary``; part sizes are read
from ``.shape`` or ``.size()``.

Differences from the reference, all bug fixes:
  * ``target_gpus`` is split over the TARGET GPUs (the reference split over all GPUs and
    then dropped the others, so a subset could never cover N, :139-141);
  * each part records ``start_index`` so its index can carry global ids
    (``ids_offset = start_index``), replacing the notebooks' ``i * len(parts[i])`` remap.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

import torch

from gpu_resource_manager import GPUResourceManager

logger = logging.getLogger(__name__)


def _rows(t: Any) -> int:
    shape = getattr(t, "shape", None)
    if isinstance(shape, (tuple, list, torch.Size)):
        return int(shape[0])
    return int(t.size(0))


def _cols(t: Any) -> int:
    shape = getattr(t, "shape", None)
    if isinstance(shape, (tuple, list, torch.Size)):
        return int(shape[1])
    return int(t.size(1))


def _on_device(t: Any, gpu_id: int) -> bool:
    dev = getattr(t, "device", None)
    if dev is None:
        return False
    if str(dev) == f"cuda:{gpu_id}":
        return True
    return getattr(dev, "type", None) == "cuda" and getattr(dev, "index", None) == gpu_id


@dataclass
class EmbeddingPart:
    """Rows [start_index, end_index) of the corpus, resident on GPU `gpu_id` (reference :20-37)."""
    gpu_id: int
    tensor: torch.Tensor
    start_index: int
    end_index: int

    def __post_init__(self):
        if self.start_index < 0:
            raise ValueError(f"start_index must be non-negative, got {self.start_index}")
        if self.end_index <= self.start_index:
            raise ValueError(f"end_index ({self.end_index}) must be greater than start_index ({self.start_index})")
        if self.gpu_id < 0:
            raise ValueError(f"gpu_id must be non-negative, got {self.gpu_id}")
        n = _rows(self.tensor)
        if n != self.end_index - self.start_index:
            raise ValueError(f"Tensor size ({n}) doesn't match index range ({self.end_index - self.start_index})")

    @property
    def num_rows(self) -> int:
        return self.end_index - self.start_index


@dataclass
class DistributedEmbeddings:
    """All parts of one corpus; they must tile [0, total_size) exactly (reference :40-70)."""
    parts: List[EmbeddingPart]
    total_size: int
    embedding_dim: int

    def __post_init__(self):
        if not self.parts:
            raise ValueError("parts list cannot be empty")
        if self.total_size <= 0:
            raise ValueError(f"total_size must be positive, got {self.total_size}")
        if self.embedding_dim <= 0:
            raise ValueError(f"embedding_dim must be positive, got {self.embedding_dim}")
        for i, p in enumerate(self.parts):
            if _cols(p.tensor) != self.embedding_dim:
                raise ValueError(f"Part {i} has embedding_dim {_cols(p.tensor)}, expected {self.embedding_dim}")
        cursor = 0
        for i, p in enumerate(sorted(self.parts, key=lambda p: p.start_index)):
            if p.start_index != cursor:
                raise ValueError(f"Gap or overlap detected at part {i}: expected start {cursor}, got {p.start_index}")
            cursor = p.end_index
        if cursor != self.total_size:
            raise ValueError(f"Parts don't cover full range: expected {self.total_size}, got {cursor}")


class EmbeddingDistributionManager:
    """Places corpus shards on GPUs and keeps track of the current placement."""

    def __init__(self, gpu_manager: GPUResourceManager):
        if not isinstance(gpu_manager, GPUResourceManager):
            raise TypeError("gpu_manager must be an instance of GPUResourceManager")
        self.gpu_manager = gpu_manager
        self.current_distribution: Optional[DistributedEmbeddings] = None

    # ---- placement -------------------------------------------------------------------------
    def _split(self, n: int, target_gpus: Optional[List[int]]):
        if target_gpus is None:
            return self.gpu_manager.distribute_workload(n, strategy="even")
        base, extra = divmod(n, len(target_gpus))  # same 'even' arithmetic, over the targets only
        out, start = [], 0
        for i, g in enumerate(target_gpus):
            size = base + (1 if i < extra else 0)
            out.append((g, start, start + size))
            start += size
        return out

    def distribute_embeddings(self, embeddings: torch.Tensor,
                              target_gpus: Optional[List[int]] = None) -> DistributedEmbeddings:
        """Copy contiguous row ranges of `embeddings` (host or device) to their GPUs."""
        if not isinstance(embeddings, torch.Tensor):
            raise TypeError("embeddings must be a torch.Tensor")
        if embeddings.dim() != 2:
            raise ValueError(f"embeddings must be 2D tensor (N x D), got shape {tuple(embeddings.shape)}")
        if embeddings.size(0) == 0:
            raise ValueError("embeddings tensor cannot be empty")
        n, d = embeddings.size(0), embeddings.size(1)
        if target_gpus is None:
            gpus = self.gpu_manager.get_available_gpu_ids()
        else:
            for g in target_gpus:
                if not self.gpu_manager.validate_gpu_index(g):
                    raise ValueError(f"Target GPU {g} is not available")
            gpus = list(target_gpus)
        if not gpus:
            raise RuntimeError("No GPUs available for embedding distribution")
        logger.info("Distributing %d embeddings across %d GPUs", n, len(gpus))
        try:
            ranges = [r for r in self._split(n, None if target_gpus is None else gpus) if r[0] in gpus]
        except Exception as e:
            raise RuntimeError(f"Failed to distribute workload: {e}") from e
        if not ranges:
            raise RuntimeError("No valid distribution found for target GPUs")

        parts: List[EmbeddingPart] = []
        try:
            for g, start, end in ranges:
                if end <= start:
                    logger.warning("Skipping empty range for GPU %s: [%s, %s)", g, start, end)
                    continue
                if start < 0 or end > n:
                    raise ValueError(f"Invalid range [{start}, {end}) for {n} embeddings")
                src = embeddings[start:end]
                moved = src.to(self.gpu_manager.get_safe_device_string(g))
                if isinstance(moved, torch.Tensor) and moved.data_ptr() == src.data_ptr():
                    moved = moved.clone()  # already on that device: the part must own its rows
                parts.append(EmbeddingPart(gpu_id=g, tensor=moved, start_index=start, end_index=end))
        except Exception as e:
            self._cleanup_embedding_parts(parts)
            raise RuntimeError(f"Failed to distribute embeddings: {e}") from e

        try:
            result = DistributedEmbeddings(parts=parts, total_size=n, embedding_dim=d)
        except Exception:
            self._cleanup_embedding_parts(parts)
            raise
        if not self.validate_distribution(result):
            self._cleanup_embedding_parts(parts)
            raise RuntimeError("Distribution validation failed")
        self.current_distribution = result
        return result

    def validate_distribution(self, distributed_embeddings: DistributedEmbeddings) -> bool:
        """Every part on a usable GPU, on the right device, contiguous coverage, consistent shapes."""
        try:
            parts = distributed_embeddings.parts
            if not parts:
                logger.error("No embedding parts found")
                return False
            available = set(self.gpu_manager.get_available_gpu_ids())
            for i, p in enumerate(parts):
                if not self.gpu_manager.validate_gpu_index(p.gpu_id) or p.gpu_id not in available:
                    logger.error("Part %d assigned to invalid GPU %s", i, p.gpu_id)
                    return False
                if not _on_device(p.tensor, p.gpu_id):
                    logger.error("Part %d tensor is on %s, expected cuda:%s", i, p.tensor.device, p.gpu_id)
                    return False
            cursor = 0
            for i, p in enumerate(sorted(parts, key=lambda p: p.start_index)):
                if p.start_index != cursor or p.end_index <= p.start_index:
                    logger.error("Index gap or bad range at part %d", i)
                    return False
                cursor = p.end_index
            if cursor != distributed_embeddings.total_size:
                logger.error("Total size mismatch: expected %s, got %s", distributed_embeddings.total_size, cursor)
                return False
            for i, p in enumerate(parts):
                if _rows(p.tensor) != p.end_index - p.start_index or _cols(p.tensor) != distributed_embeddings.embedding_dim:
                    logger.error("Part %d has an inconsistent shape", i)
                    return False
            return True
        except Exception as e:
            logger.error("Distribution validation failed with exception: %s", e)
            return False

    def redistribute_if_needed(self, distributed_embeddings: DistributedEmbeddings) -> DistributedEmbeddings:
        """Re-shard over the currently available GPUs if any part's GPU vanished (reference :274-305)."""
        available = self.gpu_manager.get_available_gpu_ids()
        lost = [p.gpu_id for p in distributed_embeddings.parts if p.gpu_id not in available]
        if not lost:
            return distributed_embeddings
        logger.warning("GPUs %s are no longer available, redistributing...", lost)
        try:
            return self.distribute_embeddings(self._collect_embeddings_to_cpu(distributed_embeddings),
                                              target_gpus=available)
        except Exception as e:
            raise RuntimeError(f"Redistribution failed: {e}") from e

    def _collect_embeddings_to_cpu(self, distributed_embeddings: DistributedEmbeddings) -> torch.Tensor:
        chunks = [p.tensor.cpu() for p in sorted(distributed_embeddings.parts, key=lambda p: p.start_index)]
        out = torch.cat(chunks, dim=0)
        expected = (distributed_embeddings.total_size, distributed_embeddings.embedding_dim)
        if tuple(out.shape) != expected:
            raise RuntimeError(f"Combined embeddings shape {tuple(out.shape)} != expected {expected}")
        return out

    def _cleanup_embedding_parts(self, embedding_parts: List[EmbeddingPart]) -> None:
        gpus = set()
        for p in embedding_parts:
            try:
                p.tensor = p.tensor.cpu()
                gpus.add(p.gpu_id)
            except Exception as e:
                logger.warning("Failed to cleanup embedding part on GPU %s: %s", p.gpu_id, e)
        if gpus:
            self.gpu_manager.cleanup_gpu_resources(sorted(gpus))

    # ---- queries ---------------------------------------------------------------------------
    def get_embedding_part_by_gpu(self, distributed_embeddings: DistributedEmbeddings,
                                  gpu_id: int) -> Optional[EmbeddingPart]:
        return next((p for p in distributed_embeddings.parts if p.gpu_id == gpu_id), None)

    def get_total_gpu_memory_usage(self, distributed_embeddings: DistributedEmbeddings) -> Dict[int, int]:
        return {p.gpu_id: int(p.tensor.numel() * p.tensor.element_size()) for p in distributed_embeddings.parts}

    get_total_memory_usage = get_total_gpu_memory_usage

    def get_distribution_summary(self, distributed_embeddings: DistributedEmbeddings) -> Dict[str, Any]:
        usage = self.get_total_gpu_memory_usage(distributed_embeddings)
        total = sum(usage.values())
        return {
            "total_embeddings": distributed_embeddings.total_size,
            "embedding_dimension": distributed_embeddings.embedding_dim,
            "num_gpus": len(distributed_embeddings.parts),
            "gpu_ids": [p.gpu_id for p in distributed_embeddings.parts],
            "part_sizes": [p.end_index - p.start_index for p in distributed_embeddings.parts],
            "part_ranges": [(p.start_index, p.end_index) for p in distributed_embeddings.parts],
            "memory_usage_bytes": usage,
            "memory_usage_mb": total / 2**20,
        }

    def cleanup_distribution(self, distributed_embeddings: Optional[DistributedEmbeddings] = None) -> None:
        """Move the parts off their GPUs and release cached memory (current distribution by default)."""
        target = distributed_embeddings if distributed_embeddings is not None else self.current_distribution
        if target is None:
            return
        self._cleanup_embedding_parts(target.parts)
        if target is self.current_distribution:
            self.current_distribution = None

    def cleanup_current_distribution(self) -> None:
        self.cleanup_distribution(None)

    def __str__(self) -> str:
        n = len(self.current_distribution.parts) if self.current_distribution else 0
        return f"EmbeddingDistributionManager(current_parts={n})"

    def __repr__(self) -> str:
        return (f"EmbeddingDistributionManager(gpu_manager={self.gpu_manager}, "
                f"has_current_distribution={self.current_distribution is not None})")
