"""The cosine metric: an inner-product index over L2-normalised rows.

sklearn's cosine baselines in the reference (``cosine_similarity`` and
``NearestNeighbors(metric='cosine', algorithm='brute')``,
Attempt_1/VectorSearch_QuestionRetrieval.ipynb:839,878) and cuVS's ``"cosine"`` metric both rank by
1 - cos(q, x). Here rows and queries are normalised on the device with the pinned norm
(``mivs_normalize_rows``; zero rows stay zero, as sklearn's ``normalize``), the inner-product
engine ranks them, and the reported distance is ``1 - ip`` in fp32 (oracle: ``cosine_knn``).
"""
from __future__ import annotations

import torch

from . import _native
from ._tensors import ptr, stream_ptr

COSINE_METRICS = ("cosine", "CosineExpanded")


def is_cosine(metric: str) -> bool:
    return metric in COSINE_METRICS


def normalize_rows(x: torch.Tensor) -> torch.Tensor:
    """A new device tensor: each row of the contiguous f32 CUDA tensor `x` over its pinned norm."""
    out = torch.empty_like(x)
    dev = x.device.index
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_normalize_rows(dev, stream_ptr(dev), ptr(x), x.shape[0], x.shape[1],
                                                        ptr(out)))
    return out


def to_distance_(ip: torch.Tensor) -> torch.Tensor:
    """In place: ip -> 1 - ip (one fp32 rounding, (-ip) + 1 == 1 - ip)."""
    return ip.neg_().add_(1.0)
