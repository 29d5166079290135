"""Cross-shard top-k exchange over torch.distributed (RCCL over xGMI on MI355X).

One process per GPU; each rank holds one corpus shard (a contiguous row range,
``GPUResourceManager.distribute_workload`` — gpu_resource_manager.py:190-202)
with its own index whose ids are already global (``ids_offset = start_index``,
fixing the reference's ``i * len(parts[i])`` remap, cuvs-2gpu-main.ipynb:1803).
After each rank's local search, the per-shard ``[Q, k]`` (distance, id) tiles
are exchanged with ONE all-gather (Q*k*12 bytes per rank) and merged on the
device by the K7 wave merge — replacing the reference's host-side numpy
argsort merge (improved_multi_gpu_rag.py:266-275, cuvs-2gpu-main.ipynb:1820-1834).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def all_gather_raw(distances: torch.Tensor, ids: torch.Tensor, group=None):
    """-> (dist [world, Q, k], ids [world, Q, k]): the rank-major all-gather receive buffers."""
    world = dist.get_world_size(group)
    q, k = distances.shape
    gd = torch.empty((world * q, k), dtype=distances.dtype, device=distances.device)
    gi = torch.empty((world * q, k), dtype=ids.dtype, device=ids.device)
    dist.all_gather_into_tensor(gd, distances.contiguous(), group=group)
    dist.all_gather_into_tensor(gi, ids.contiguous(), group=group)
    return gd.view(world, q, k), gi.view(world, q, k)


def all_gather_topk(distances: torch.Tensor, ids: torch.Tensor, group=None):
    """-> (dist [Q, world, k], ids [Q, world, k]) gathered from every rank (rank order)."""
    gd, gi = all_gather_raw(distances, ids, group)
    return gd.permute(1, 0, 2).contiguous(), gi.permute(1, 0, 2).contiguous()


def merge_across_ranks(distances: torch.Tensor, ids: torch.Tensor, k: int, metric: str = "sqeuclidean",
                       group=None, merge_fn: Optional[Callable] = None):
    """Global top-k over all shards; every rank gets the same result.

    The default merge is K7 reading the rank-major receive buffer in place
    (``mivs.ops.merge_topk_gathered``: no transpose). ``merge_fn(dist[Q, m, k_in], ids[Q, m, k_in],
    k, metric)`` replaces it (tests on the CPU gloo backend pass their own).
    """
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return distances, ids
    if merge_fn is None:
        from .ops import merge_topk_gathered

        gd, gi = all_gather_raw(distances, ids, group)
        return merge_topk_gathered(gd, gi, k, metric)
    gd, gi = all_gather_topk(distances, ids, group)
    return merge_fn(gd, gi, k, metric)


def allreduce_max(value: float, device: torch.device | None = None, group=None) -> float:
    """Max of a host scalar over ranks (the bench's max-over-ranks timing)."""
    if not dist.is_available() or not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def per_rank_values(value: float, device: torch.device | str | None = None, group=None) -> list:
    """[value of rank 0, rank 1, ...]: a host scalar gathered from every rank (diagnostics of the N > 1 line)."""
    if not dist.is_available() or not dist.is_initialized():
        return [float(value)]
    world = dist.get_world_size(group)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return [float(v.item()) for v in out]


def timed_sharded_step(search_fn: Callable, k: int, metric: str = "sqeuclidean", group=None,
                       merge_fn: Optional[Callable] = None):
    """One sharded step -- this rank's search, the all-gather of the per-shard top-k, the merge -- with each part
    timed: hipEvents on the current stream when the results are on a GPU (the all-gather's RCCL work is ordered
    before the event that follows it), the host clock otherwise. -> ((dist, ids), {"search_ms", "allgather_ms",
    "merge_ms"}). The merge is K7 over the rank-major receive buffer (``merge_fn(gd, gi, k, metric)`` replaces it,
    taking the same [world, Q, k] buffers)."""
    import time

    marks = []

    def mark(on_gpu):
        if on_gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks.append(e)
        else:
            marks.append(time.perf_counter())

    gpu = torch.cuda.is_available() and torch.cuda.is_initialized()
    mark(gpu)
    d, i = search_fn()
    gpu = d.is_cuda
    if gpu and not isinstance(marks[0], torch.cuda.Event):  # (the search initialised the GPU: restart the clock)
        marks[0] = torch.cuda.Event(enable_timing=True)
        marks[0].record()
    mark(gpu)
    gd, gi = all_gather_raw(d, i, group)
    mark(gpu)
    if merge_fn is None:
        from .ops import merge_topk_gathered

        out = merge_topk_gathered(gd, gi, k, metric)
    else:
        out = merge_fn(gd, gi, k, metric)
    mark(gpu)
    if gpu:
        marks[-1].synchronize()
        ms = [marks[j].elapsed_time(marks[j + 1]) for j in range(3)]
    else:
        ms = [(marks[j + 1] - marks[j]) * 1e3 for j in range(3)]
    return out, {"search_ms": ms[0], "allgather_ms": ms[1], "merge_ms": ms[2]}
