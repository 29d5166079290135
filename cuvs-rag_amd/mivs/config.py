"""Output conversion hook — the mivs counterpart of ``pylibraft.config.set_output_as``.

The reference makes every cuVS result host numpy with
``pylibraft.config.set_output_as(lambda device_ndarray: device_ndarray.copy_to_host())``
(improved_multi_gpu_rag.py:114, cuvs-2gpu-main.ipynb:290). The same call works
here: results are handed to the hook as a :class:`DeviceArray` (which has
``copy_to_host()``), or returned as torch tensors by default.
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Union

import torch


class DeviceArray:
    """Minimal pylibraft ``device_ndarray`` look-alike over a torch CUDA tensor."""

    def __init__(self, tensor: torch.Tensor):
        self.tensor = tensor

    @property
    def shape(self):
        return tuple(self.tensor.shape)

    @property
    def dtype(self):
        return self.tensor.dtype

    def copy_to_host(self):
        return self.tensor.detach().cpu().numpy()

    @property
    def __cuda_array_interface__(self):
        return self.tensor.__cuda_array_interface__

    def __repr__(self):
        return f"DeviceArray(shape={self.shape}, dtype={self.dtype}, device={self.tensor.device})"


_state = threading.local()
_global: Union[str, Callable[[DeviceArray], Any]] = "torch"


def set_output_as(output: Union[str, Callable[[DeviceArray], Any]]) -> None:
    """'torch' (default), 'raft'/'mivs' (DeviceArray), 'numpy', or a callable taking a DeviceArray."""
    global _global
    if isinstance(output, str) and output not in ("torch", "raft", "mivs", "numpy", "cupy"):
        raise ValueError(f"unknown output type {output!r}")
    _global = output


def get_output_as():
    return _global


def convert_output(t: torch.Tensor):
    out = _global
    if callable(out):
        return out(DeviceArray(t))
    if out == "torch":
        return t
    if out in ("raft", "mivs", "cupy"):
        return DeviceArray(t)
    if out == "numpy":
        return t.detach().cpu().numpy()
    raise ValueError(f"unknown output type {out!r}")
