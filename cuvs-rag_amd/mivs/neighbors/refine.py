"""cuvs.neighbors.refine — exact re-ranking of candidate neighbours (K14, ``refine.hip``).

cuVS pairs IVF-PQ with ``refine(dataset, queries, candidates, k)``: search the PQ codes for r*k
candidates per query, then rank those candidates by their exact distance to the query. The reference
calls ``ivf_pq.search`` (improved_multi_gpu_rag.py:228-230, index_building_coordinator.py:398-404);
``refine`` is what brings that path to the recall the IVF-Flat path reaches. Keys are the pinned fp32
keys of the arithmetic contract, so the result equals an exact search restricted to the
candidates, bit for bit. The dataset may be fp32 or fp16 (widened exactly).
"""
from __future__ import annotations

import torch

from .. import _native
from .._tensors import as_device_f32, emit, out_tensor, ptr, stream_ptr
from .ivf_flat import _SQRT_METRICS, metric_code


def refine(dataset, queries, candidates, k=None, indices=None, distances=None, metric: str = "sqeuclidean",
           resources=None):
    """-> (distances [nq, k] f32, neighbors [nq, k] i64): the exact top-k of each query's candidate rows
    (row numbers of ``dataset``; -1 entries are skipped).

    cuVS's parameter order: ``k`` may be omitted when ``indices`` (the output buffer) is given -- it is then
    ``indices.shape[1]``. This build serves k <= 64 (one wave per query ranks the candidates); larger k
    raises ValueError."""
    ds = dataset.tensor if hasattr(dataset, "tensor") else dataset
    if not isinstance(ds, torch.Tensor):
        ds = torch.as_tensor(ds)
    if ds.dim() != 2:
        raise ValueError("dataset must be 2-D")
    if not ds.is_cuda:
        raise ValueError("dataset must be on a GPU (cuvs.neighbors.refine takes device data)")
    dev = ds.device.index
    half = ds.dtype == torch.float16
    if not half:
        ds = ds.float()
    ds = ds.contiguous()
    q = as_device_f32(queries, device=dev, name="queries")
    if q.shape[1] != ds.shape[1]:
        raise ValueError(f"queries have dim {q.shape[1]}, dataset has {ds.shape[1]}")
    c = candidates.tensor if hasattr(candidates, "tensor") else candidates
    c = torch.as_tensor(c).to(device=f"cuda:{dev}", dtype=torch.int64).contiguous()
    if c.dim() != 2 or c.shape[0] != q.shape[0]:
        raise ValueError("candidates must be [n_queries, n_candidates]")
    if k is None:
        if indices is None:
            raise ValueError("k is required when no indices output is given")
        k = (indices.tensor if hasattr(indices, "tensor") else indices).shape[1]
    k = int(k)
    if not 1 <= k <= min(c.shape[1], 64):
        raise ValueError(f"k must be in [1, min(n_candidates, 64)], got {k}")
    nq = q.shape[0]
    dist = out_tensor(distances, (nq, k), torch.float32, dev, "distances")
    nbrs = out_tensor(indices, (nq, k), torch.int64, dev, "indices")
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_refine(dev, stream_ptr(dev), ptr(ds), 1 if half else 0, ds.shape[0],
                                                ds.shape[1], ptr(q), nq, ptr(c), c.shape[1], k, metric_code(metric),
                                                ptr(dist), ptr(nbrs)))
    if metric in _SQRT_METRICS:
        dist.sqrt_()
    return emit(dist), emit(nbrs)


__all__ = ["refine"]
