"""GPU discovery, validation and shard arithmetic on ROCm.

Drop-in for the reference's ``Attempt_1/gpu_resource_manager.py`` (class
``GPUResourceManager`` at :39): same dataclasses, method names, return shapes and
error messages, so the reference's own tests and drivers run unchanged. PyTorch-ROCm
keeps the ``torch.cuda`` namespace and ``"cuda:N"`` device strings, so nothing here
is CUDA-specific.

``distribute_workload`` (reference :170-233) is on the hot path's boundary: it fixes
the corpus shard of every GPU, i.e. the global-id offset (``start_index``) that each
shard's index adds to its local ids.
"""
from __future__ import annotations

import gc
import logging
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

logger = logging.getLogger(__name__)



def even_split(total_items: int, parts: int) -> List[Tuple[int, int]]:
    """The 'even' strategy's contiguous ranges [(start, end)] of [0, total_items) over `parts` shards: floor(N/P)
    rows each, the first N mod P shards one more (reference gpu_resource_manager.py:190-202). bench.py's fixed-corpus
    mode splits its corpus with it."""
    base, extra = divmod(int(total_items), int(parts))
    out, start = [], 0
    for i in range(int(parts)):
        end = start + base + (1 if i < extra else 0)
        out.append((start, end))
        start = end
    return out

@dataclass
class GPUConfig:
    """One device as seen at discovery time (reference :21-28)."""
    gpu_id: int
    device_name: str
    total_memory: int
    available_memory: int
    is_available: bool


@dataclass
class MultiGPUConfig:
    """Snapshot of the whole node (reference :31-36); strategy in {'even', 'memory_based', 'custom'}."""
    available_gpus: List[GPUConfig]
    primary_gpu: int
    distribution_strategy: str


def _probe_device(gpu_id: int) -> Tuple[GPUConfig, Dict[str, int]]:
    with torch.cuda.device(gpu_id):
        props = torch.cuda.get_device_properties(gpu_id)
        torch.cuda.empty_cache()
        allocated = torch.cuda.memory_allocated(gpu_id)
    total = props.total_memory
    info = {"total": total, "available": total - allocated, "allocated": allocated}
    return GPUConfig(gpu_id, props.name, total, total - allocated, True), info


def release_engine_cache(gpu_id: int) -> int:
    """Hand the blocks the mivs engine keeps for reuse on `gpu_id` back to the driver (bytes freed), so that the
    reference's torch-only cleanup (empty_cache after it) and torch.cuda.mem_get_info see that memory free. A process
    that never loaded the engine holds nothing."""
    try:
        from mivs import _native
    except ImportError:
        return 0
    return _native.release_cached_memory(gpu_id)


class GPUResourceManager:
    """Owns the list of usable devices and the row-range split of a corpus over them."""

    def __init__(self):
        self.available_gpus: List[int] = []
        self.gpu_memory_info: Dict[int, Dict] = {}
        self.gpu_configs: List[GPUConfig] = []
        self._discover_gpus()

    # ---- discovery -------------------------------------------------------------------------
    def _discover_gpus(self) -> None:
        try:
            if not torch.cuda.is_available():
                logger.warning("No ROCm/CUDA device visible; running without GPUs.")
                return
            count = torch.cuda.device_count()
        except Exception as e:  # a broken runtime is "no GPUs", never a crash
            logger.error("GPU discovery failed: %s", e)
            return
        logger.info("Detected %d GPU(s)", count)
        for gpu_id in range(count):
            try:
                cfg, info = _probe_device(gpu_id)
            except Exception as e:
                logger.warning("GPU %d is not accessible: %s", gpu_id, e)
                self.gpu_configs.append(GPUConfig(gpu_id, "Unknown", 0, 0, False))
                continue
            self.gpu_configs.append(cfg)
            self.available_gpus.append(gpu_id)
            self.gpu_memory_info[gpu_id] = info
            logger.info("GPU %d: %s - %.1f GB total, %.1f GB available", gpu_id, cfg.device_name,
                        cfg.total_memory / 2**30, cfg.available_memory / 2**30)

    # ---- validation ------------------------------------------------------------------------
    def validate_gpu_index(self, gpu_id: int) -> bool:
        """True iff `gpu_id` is a discovered, still-visible device."""
        if gpu_id < 0:
            logger.error("Invalid GPU index: %s (negative index)", gpu_id)
            return False
        if gpu_id not in self.available_gpus:
            logger.error("GPU %s is not in available GPUs list: %s", gpu_id, self.available_gpus)
            return False
        if not torch.cuda.is_available():
            logger.error("No ROCm/CUDA device visible")
            return False
        n = torch.cuda.device_count()
        if gpu_id >= n:
            logger.error("GPU %s exceeds available GPU count: %s", gpu_id, n)
            return False
        return True

    def get_safe_device_string(self, gpu_id: int) -> str:
        if not self.validate_gpu_index(gpu_id):
            raise ValueError(f"Invalid GPU index: {gpu_id}. Available GPUs: {self.available_gpus}")
        return f"cuda:{gpu_id}"

    def get_available_gpu_count(self) -> int:
        return len(self.available_gpus)

    def get_available_gpu_ids(self) -> List[int]:
        return list(self.available_gpus)

    # ---- shard arithmetic (hot-path boundary) ----------------------------------------------
    def distribute_workload(self, total_items: int, strategy: str = "even") -> List[Tuple[int, int, int]]:
        """Contiguous row ranges ``[(gpu_id, start, end)]`` covering ``[0, total_items)`` in GPU order.

        'even': floor(N/P) rows each, the first N mod P GPUs one more (reference :190-202).
        'memory_based': proportional to available memory with int truncation (reference :204-223);
        unlike the reference, the truncation remainder goes to the last GPU so coverage is exact.
        """
        if not self.available_gpus:
            raise RuntimeError("No GPUs available for workload distribution")
        if total_items <= 0:
            raise ValueError(f"Invalid total_items: {total_items}")
        gpus = self.available_gpus
        if strategy == "even":
            sizes = [e - b for b, e in even_split(total_items, len(gpus))]
        elif strategy == "memory_based":
            mem = [self.gpu_memory_info[g]["available"] for g in gpus]
            total_mem = sum(mem)
            sizes = [int(total_items * m / total_mem) for m in mem]
            sizes[-1] += total_items - sum(sizes)
        else:
            raise ValueError(f"Unknown distribution strategy: {strategy}")
        out, start = [], 0
        for g, s in zip(gpus, sizes):
            if s <= 0 and strategy == "memory_based":
                continue
            out.append((g, start, start + s))
            start += s
        return out

    # ---- resources -------------------------------------------------------------------------
    def cleanup_gpu_resources(self, gpu_ids: Optional[List[int]] = None) -> None:
        for gpu_id in (self.available_gpus if gpu_ids is None else gpu_ids):
            if not self.validate_gpu_index(gpu_id):
                continue
            try:
                release_engine_cache(gpu_id)
                with torch.cuda.device(gpu_id):
                    torch.cuda.empty_cache()
                    torch.cuda.synchronize()
            except Exception as e:
                logger.warning("Failed to cleanup GPU %s: %s", gpu_id, e)
        gc.collect()

    def get_gpu_memory_info(self, gpu_id: int) -> Dict[str, int]:
        """torch-allocator view (allocated/reserved/total/free = total - reserved) plus the
        device-wide free bytes from hipMemGetInfo under 'device_free' when obtainable."""
        if not self.validate_gpu_index(gpu_id):
            raise ValueError(f"Invalid GPU index: {gpu_id}")
        try:
            with torch.cuda.device(gpu_id):
                allocated = torch.cuda.memory_allocated(gpu_id)
                reserved = torch.cuda.memory_reserved(gpu_id)
                total = torch.cuda.get_device_properties(gpu_id).total_memory
        except Exception as e:
            logger.error("Failed to get memory info for GPU %s: %s", gpu_id, e)
            return {"allocated": 0, "reserved": 0, "total": 0, "free": 0}
        info = {"allocated": allocated, "reserved": reserved, "total": total, "free": total - reserved}
        try:
            info["device_free"] = int(torch.cuda.mem_get_info(gpu_id)[0])
        except Exception:
            pass
        return info

    def get_multi_gpu_config(self, strategy: str = "even") -> MultiGPUConfig:
        return MultiGPUConfig(available_gpus=list(self.gpu_configs),
                              primary_gpu=self.available_gpus[0] if self.available_gpus else -1,
                              distribution_strategy=strategy)

    def validate_tensor_distribution(self, tensor_parts: List[torch.Tensor]) -> bool:
        if len(tensor_parts) != len(self.available_gpus):
            logger.error("Tensor parts count (%d) != available GPUs (%d)", len(tensor_parts),
                         len(self.available_gpus))
            return False
        for i, (t, g) in enumerate(zip(tensor_parts, self.available_gpus)):
            if t.device.index != g:
                logger.error("Tensor part %d is on GPU %s, expected GPU %s", i, t.device.index, g)
                return False
        return True

    def __str__(self) -> str:
        return f"GPUResourceManager(available_gpus={self.available_gpus}, gpu_count={len(self.available_gpus)})"

    def __repr__(self) -> str:
        return (f"GPUResourceManager(available_gpus={self.available_gpus}, gpu_configs={len(self.gpu_configs)}, "
                f"cuda_available={torch.cuda.is_available()})")
