"""Pipelined search of host-resident queries.

The reference searches one query at a time from Python and copies every result back before the
next launch (``cuvs-2gpu-main.ipynb:1789-1836``, ``improved_multi_gpu_rag.py:279-303``;
``README_improved.md:166`` lists streams as future work). Here a host query matrix is cut into
batches and three HIP streams overlap the work of neighbouring batches:

  * H2D stream:  batch b+1 into the device query slot (b+1) % 2
  * the caller's current stream: the search of batch b (the same native call as ``search``)
  * D2H stream:  batch b's results into the pinned host output

Two device slots per buffer; events order the slot reuse (a query slot is refilled only after
the search that read it, a result slot is rewritten only after its copy-out). Results are
identical to one device-side ``search`` per batch (``tests/test_gpu_streaming.py``).
"""
from __future__ import annotations

import numpy as np
import torch

from . import brute_force, ivf_flat, ivf_pq


def _host_f32(x, name: str) -> torch.Tensor:
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
    elif not isinstance(x, torch.Tensor):
        x = torch.as_tensor(x)
    if x.dim() != 2:
        raise ValueError(f"{name} must be a 2-D array, got shape {tuple(x.shape)}")
    if x.is_cuda:
        raise ValueError(f"{name} must be host-resident (use search() for device queries)")
    if x.dtype != torch.float32:
        x = x.float()
    return x.contiguous()


def _host_out(out, shape, dtype, pin: bool, name: str) -> torch.Tensor:
    if out is None:
        return torch.empty(shape, dtype=dtype, pin_memory=pin)
    if not isinstance(out, torch.Tensor) or out.is_cuda or tuple(out.shape) != tuple(shape) or out.dtype != dtype \
            or not out.is_contiguous():
        raise ValueError(f"{name} must be a contiguous host {dtype} tensor of shape {tuple(shape)}")
    return out


_side_streams: dict = {}


def _streams(dev: int):
    """The H2D and D2H streams of `dev`, created once: a new HIP stream's first use sets up its hardware
    queue, which cost up to ~7 ms per call when every call took fresh streams from torch's pool."""
    st = _side_streams.get(dev)
    if st is None:
        st = _side_streams[dev] = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
    return st


def _searcher(index, search_params):
    if isinstance(index, ivf_flat.Index):
        return lambda q, k, dd, ii: ivf_flat._search(search_params, index, q, k, ii, dd)
    if isinstance(index, ivf_pq.Index):
        return lambda q, k, dd, ii: ivf_pq._search(search_params, index, q, k, ii, dd)
    if isinstance(index, brute_force.Index):
        return lambda q, k, dd, ii: brute_force._search(index, q, k, ii, dd)
    raise TypeError(f"index must be an ivf_flat, ivf_pq or brute_force Index, got {type(index).__name__}")


def search_host(index, queries, k: int, search_params=None, batch_size: int = 10000, distances=None,
                neighbors=None):
    """k-NN of host queries with copies overlapped with the search.

    ``index``: an ``ivf_flat``, ``ivf_pq`` or ``brute_force`` Index; ``search_params`` as for that
    module's ``search`` (ignored for brute force). ``queries``: host ``[nq, dim]`` (numpy or a CPU
    tensor; copied once into pinned memory if it is not pinned). Returns ``(distances, neighbors)``
    as pinned CPU tensors ``[nq, k]`` (f32, i64), equal to ``search`` on each batch; pass pinned
    ``distances`` / ``neighbors`` of that shape to reuse them (a fresh pinned allocation costs
    milliseconds).
    """
    run = _searcher(index, search_params)
    k = int(k)
    if k < 1:
        raise ValueError(f"k must be >= 1, got {k}")
    batch_size = int(batch_size)
    if batch_size < 1:
        raise ValueError(f"batch_size must be >= 1, got {batch_size}")
    qh = _host_f32(queries, "queries")
    if qh.shape[1] != index.dim:
        raise ValueError(f"queries have dim {qh.shape[1]}, index has {index.dim}")
    nq, dim = qh.shape
    dev = index.device
    pin = torch.cuda.is_available()
    out_d = _host_out(distances, (nq, k), torch.float32, pin, "distances")
    out_i = _host_out(neighbors, (nq, k), torch.int64, pin, "neighbors")
    if nq == 0:
        return out_d, out_i
    if not qh.is_pinned():
        qh = qh.pin_memory()
    B = min(batch_size, nq)
    batches = [(s, min(B, nq - s)) for s in range(0, nq, B)]
    with torch.cuda.device(dev):
        comp = torch.cuda.current_stream(dev)
        h2d, d2h = _streams(dev)
        qbuf = [torch.empty((B, dim), dtype=torch.float32, device=f"cuda:{dev}") for _ in range(2)]
        dbuf = [torch.empty((B, k), dtype=torch.float32, device=f"cuda:{dev}") for _ in range(2)]
        ibuf = [torch.empty((B, k), dtype=torch.int64, device=f"cuda:{dev}") for _ in range(2)]
        ev_in = [torch.cuda.Event() for _ in range(2)]
        ev_done = [torch.cuda.Event() for _ in range(2)]
        ev_out = [torch.cuda.Event() for _ in range(2)]
        # the slots are allocated on `comp`; the copies must finish before `comp` may reuse them
        h2d.wait_stream(comp)
        d2h.wait_stream(comp)

        def load(b: int) -> None:
            slot = b & 1
            s, n = batches[b]
            with torch.cuda.stream(h2d):
                if b >= 2:
                    h2d.wait_event(ev_done[slot])  # the search of batch b-2 has read this slot
                qbuf[slot][:n].copy_(qh[s:s + n], non_blocking=True)
                ev_in[slot].record(h2d)

        load(0)
        for b, (s, n) in enumerate(batches):
            if b + 1 < len(batches):
                load(b + 1)
            slot = b & 1
            comp.wait_event(ev_in[slot])
            if b >= 2:
                comp.wait_event(ev_out[slot])  # batch b-2's results have left this slot
            dd, ii = run(qbuf[slot][:n], k, dbuf[slot][:n], ibuf[slot][:n])
            ev_done[slot].record(comp)
            with torch.cuda.stream(d2h):
                d2h.wait_event(ev_done[slot])
                out_d[s:s + n].copy_(dd, non_blocking=True)
                out_i[s:s + n].copy_(ii, non_blocking=True)
                ev_out[slot].record(d2h)
        d2h.synchronize()
        comp.wait_stream(d2h)
        comp.wait_stream(h2d)
    return out_d, out_i


__all__ = ["search_host"]
