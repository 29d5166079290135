"""Low-level device ops exposed for the multi-GPU merge, parity tests and the bench."""
from __future__ import annotations

import torch

from . import _native
from ._tensors import as_device_f32, ptr, stream_ptr
from .neighbors.ivf_flat import metric_code


def merge_topk(dist: torch.Tensor, ids: torch.Tensor, k: int, metric: str = "sqeuclidean"):
    """K7: per query, merge m sorted candidate lists -> top-k. dist/ids: [nq, m, k_in] (or [nq, m*k_in])."""
    if dist.shape != ids.shape or dist.dim() not in (2, 3):
        raise ValueError("dist/ids must have equal shape [nq, m, k_in]")
    if dist.dim() == 2:
        dist = dist.unsqueeze(1)
        ids = ids.unsqueeze(1)
    nq, m, k_in = dist.shape
    dev = dist.device.index
    d = dist.contiguous().float()
    i = ids.contiguous().to(torch.int64)
    od = torch.empty((nq, k), dtype=torch.float32, device=dist.device)
    oi = torch.empty((nq, k), dtype=torch.int64, device=dist.device)
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_merge_topk(dev, stream_ptr(dev), ptr(d), ptr(i), nq, m, k_in, k,
                                                    _merge_order(metric), ptr(od), ptr(oi)))
    return od, oi


def merge_topk_gathered(dist: torch.Tensor, ids: torch.Tensor, k: int, metric: str = "sqeuclidean"):
    """K7 over an all-gather receive buffer: dist/ids [parts, nq, k_in] (rank-major) -> [nq, k]."""
    if dist.shape != ids.shape or dist.dim() != 3:
        raise ValueError("dist/ids must have equal shape [parts, nq, k_in]")
    parts, nq, k_in = dist.shape
    dev = dist.device.index
    d = dist.contiguous().float()
    i = ids.contiguous().to(torch.int64)
    od = torch.empty((nq, k), dtype=torch.float32, device=dist.device)
    oi = torch.empty((nq, k), dtype=torch.int64, device=dist.device)
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_merge_topk_gathered(dev, stream_ptr(dev), ptr(d), ptr(i), parts, nq, k_in, k,
                                                             _merge_order(metric), ptr(od), ptr(oi)))
    return od, oi


def _merge_order(metric: str) -> int:
    """Cosine results are distances 1 - ip (smaller is better): merged in the L2 order."""
    from ._cosine import is_cosine

    return _native.METRIC_L2 if is_cosine(metric) else metric_code(metric)


def row_norms(x) -> torch.Tensor:
    """‖x‖² per row in the engine's k-order (the value the scan kernels use)."""
    t = as_device_f32(x, name="x")
    dev = t.device.index
    out = torch.empty(t.shape[0], dtype=torch.float32, device=t.device)
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_row_norms(dev, stream_ptr(dev), ptr(t), t.shape[0], t.shape[1], ptr(out)))
    return out


def synth_mixture(n: int, d: int, seed: int, n_centers: int = 4096, sigma: float = 0.35, normalize: bool = True,
                  row_begin: int = 0, device: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """On-device clustered corpus: row i = C[H(seed,i) % n_centers] + sigma*N(0,I), L2-normalised.

    Rows are a pure function of (seed, global row index), so shard s of a sharded corpus is generated
    on GPU s with row_begin = its start_index."""
    dev = torch.cuda.current_device() if device is None else device
    if out is None:
        out = torch.empty((n, d), dtype=torch.float32, device=f"cuda:{dev}")
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_synth_mixture(dev, stream_ptr(dev), ptr(out), int(row_begin), int(n), int(d),
                                                       int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_centers), float(sigma),
                                                       1 if normalize else 0))
    return out
