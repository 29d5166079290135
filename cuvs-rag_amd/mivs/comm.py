"""Single-process cross-shard exchange over RCCL (xGMI): one communicator per local GPU.

The reference's drivers run one Python thread per GPU in ONE process
(index_building_coordinator.py:233, improved_multi_gpu_rag.py:105,206) and merge the per-GPU
results on the host with numpy (improved_multi_gpu_rag.py:239-277, cuvs-2gpu-main.ipynb:1820-1834).
``LocalComm`` keeps every shard's [Q, k] tile on its device: ``mivs_merge_topk_allgather`` runs one
grouped ncclAllGather per array over ncclCommInitAll communicators and the K7 merge reads the
rank-major receive buffer in place. Multi-process deployments (one rank per GPU, torchrun) use
``mivs.distributed.merge_across_ranks`` instead.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _native
from ._tensors import stream_ptr


class LocalComm:
    """RCCL communicators over ``devices`` (rank r = devices[r]) of this process."""

    def __init__(self, devices: Sequence[int]):
        self.devices = [int(d) for d in devices]
        if not self.devices:
            raise ValueError("LocalComm needs at least one device")
        arr = (ctypes.c_int32 * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _native.check(_native.lib().mivs_comm_init_all(len(self.devices), arr, ctypes.byref(h)))
        self._h = h
        self._lock = threading.Lock()

    @property
    def size(self) -> int:
        return len(self.devices)

    def rank_of(self, device: int) -> int:
        return self.devices.index(int(device))

    def merge_topk_allgather(self, dists: Dict[int, torch.Tensor], ids: Dict[int, torch.Tensor], k: int,
                             metric: str = "sqeuclidean", out_devices: Optional[Sequence[int]] = None
                             ) -> Dict[int, Tuple[torch.Tensor, torch.Tensor]]:
        """Global top-k of every shard's [nq, k_in] (dist, global id) tile, each on its own device.

        Returns {device: (dist [nq, k], ids [nq, k])} for each device in ``out_devices``
        (default: the first one). Ordering and padding follow ``mivs_merge_topk``."""
        from .ops import _merge_order

        if set(dists) != set(self.devices) or set(ids) != set(self.devices):
            raise ValueError(f"need one tile per communicator device {self.devices}, got {sorted(dists)}")
        shape = tuple(dists[self.devices[0]].shape)
        if len(shape) != 2:
            raise ValueError("per-shard tiles must be [nq, k_in]")
        nq, k_in = shape
        outs = [self.devices[0]] if out_devices is None else [int(d) for d in out_devices]
        P = self.size
        dd: List[torch.Tensor] = []
        ii: List[torch.Tensor] = []
        for dev in self.devices:
            d, i = dists[dev], ids[dev]
            if tuple(d.shape) != shape or tuple(i.shape) != shape:
                raise ValueError(f"cuda:{dev}: tile shape {tuple(d.shape)} != {shape}")
            if not d.is_cuda or d.device.index != dev or not i.is_cuda or i.device.index != dev:
                raise ValueError(f"the tile for cuda:{dev} must live on cuda:{dev}")
            dd.append(d.contiguous().float())
            ii.append(i.contiguous().to(torch.int64))
        res: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
        od = (ctypes.c_void_p * P)()
        oi = (ctypes.c_void_p * P)()
        for dev in outs:
            r = self.rank_of(dev)
            res[dev] = (torch.empty((nq, k), dtype=torch.float32, device=f"cuda:{dev}"),
                        torch.empty((nq, k), dtype=torch.int64, device=f"cuda:{dev}"))
            od[r], oi[r] = res[dev][0].data_ptr(), res[dev][1].data_ptr()
        streams = (ctypes.c_void_p * P)(*[stream_ptr(dev) for dev in self.devices])
        pd = (ctypes.c_void_p * P)(*[t.data_ptr() for t in dd])
        pi = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ii])
        with self._lock:
            _native.check(_native.lib().mivs_merge_topk_allgather(self._h, streams, pd, pi, nq, k_in, k,
                                                                  _merge_order(metric), od, oi))
        return res

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            _native.lib().mivs_comm_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self) -> str:
        return f"LocalComm(devices={self.devices})"


_cache: Dict[Tuple[int, ...], LocalComm] = {}
_cache_lock = threading.Lock()


def local_comm(devices: Sequence[int]) -> LocalComm:
    """One communicator set per device tuple, created on first use and kept for the process."""
    key = tuple(int(d) for d in devices)
    with _cache_lock:
        c = _cache.get(key)
        if c is None:
            c = _cache[key] = LocalComm(key)
        return c
