"""Lloyd k-means on MI355X (cuvs.cluster.kmeans-style API).

The trainer cuVS runs inside ``ivf_flat::build`` (reached from
index_building_coordinator.py:396) and FAISS runs in ``IndexIVFFlat.train``
(colab_a100_test.ipynb:478). Assign = the fused MFMA distance scan with k=1
(ties to the lower centroid id); update = deterministic fp64 member sums in a
fixed order, so results are bit-exact with
oracle/mivs_oracle.c and reproducible run to run.
"""
from __future__ import annotations

import torch

from .. import _native
from .._tensors import as_device_f32, ptr, stream_ptr
from ..neighbors.ivf_flat import metric_code


class KMeansParams:
    def __init__(self, n_clusters: int = 8, max_iter: int = 20, metric: str = "sqeuclidean"):
        if n_clusters < 1:
            raise ValueError("n_clusters must be >= 1")
        self.n_clusters = int(n_clusters)
        self.max_iter = int(max_iter)
        self.metric = metric


def fit(params: KMeansParams, X, centroids=None, rows: torch.Tensor | None = None):
    """Run `max_iter` Lloyd iterations. `centroids` = initial centres (default: strided rows of X).

    Returns (centroids [n_clusters, d] float32 on X's device, n_iter)."""
    x = as_device_f32(X, name="X")
    dev = x.device.index
    n, d = x.shape
    if centroids is None:
        idx = (torch.arange(params.n_clusters, device=x.device, dtype=torch.int64) * n) // params.n_clusters
        c = x.index_select(0, idx).contiguous()
    else:
        c = as_device_f32(centroids, device=dev, name="centroids").clone()
    if c.shape != (params.n_clusters, d):
        raise ValueError(f"centroids must have shape {(params.n_clusters, d)}")
    n_train = n
    rows_t = None
    if rows is not None:
        rows_t = rows.to(device=x.device, dtype=torch.int64).contiguous()
        n_train = rows_t.shape[0]
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_kmeans_fit(dev, stream_ptr(dev), ptr(x), n, d, ptr(rows_t), n_train,
                                                    params.n_clusters, params.max_iter, ptr(c)))
    return c, params.max_iter


def build_steps(X, centroids, rows: torch.Tensor | None, it_begin: int, n_steps: int, it_total: int,
                balance: bool = True, return_labels: bool = False):
    """Iterations it_begin .. it_begin + n_steps - 1 of the IVF build's k-means (mivs_kmeans_steps: the assign
    through the fp16 pre-filter, the fp64 update, the re-seed on all but the last 2 of it_total iterations),
    from `centroids` (updated in place). Returns (centroids, labels of the last step or None)."""
    x = as_device_f32(X, name="X")
    dev = x.device.index
    n, d = x.shape
    c = as_device_f32(centroids, device=dev, name="centroids")
    rows_t = None if rows is None else rows.to(device=x.device, dtype=torch.int64).contiguous()
    n_train = n if rows_t is None else rows_t.shape[0]
    labels = torch.empty(n_train, dtype=torch.int64, device=x.device) if return_labels else None
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_kmeans_steps(dev, stream_ptr(dev), ptr(x), n, d, ptr(rows_t), n_train,
                                                      c.shape[0], it_begin, n_steps, it_total, int(balance), ptr(c),
                                                      ptr(labels)))
    return c, labels


def predict(params: KMeansParams, centroids, X) -> torch.Tensor:
    x = as_device_f32(X, name="X")
    dev = x.device.index
    c = as_device_f32(centroids, device=dev, name="centroids")
    labels = torch.empty(x.shape[0], dtype=torch.int64, device=x.device)
    with torch.cuda.device(dev):
        _native.check(_native.lib().mivs_kmeans_predict(dev, stream_ptr(dev), ptr(x), x.shape[0], x.shape[1], ptr(c),
                                                        c.shape[0], metric_code(params.metric), ptr(labels)))
    return labels
