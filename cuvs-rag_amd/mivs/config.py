"""Output conversion hook — the mivs counterpart of ``pylibraft.config.set_output_as``.

The reference makes every cuVS result host numpy with
``pylibraft.config.set_output_as(lambda device_ndarray: device_ndarray.copy_to_host())``
(improved_multi_gpu_rag.py:114, cuvs-2gpu-main.ipynb:290). The same call works
here: results are handed to the hook as a :class:`DeviceArray` (which has
``copy_to_host()``), or returned as torch tensors by default.
"""
from __future__ import annotations

import threading
from contextlib import contextmanager
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


# The process-wide hook (what pylibraft.config.set_output_as sets), and a per-thread override used by
# the engine's own worker threads: a driver thread that set the hook to copy_to_host must not change
# what a search running on another thread returns, and a worker that needs device tensors must not
# flip the hook under the driver's feet.
_state = threading.local()
_global: Union[str, Callable[[DeviceArray], Any]] = "torch"
_KINDS = ("torch", "raft", "mivs", "numpy", "cupy")


def _check(output) -> None:
    if isinstance(output, str) and output not in _KINDS:
        raise ValueError(f"unknown output type {output!r}")
    if not isinstance(output, str) and not callable(output):
        raise ValueError(f"output must be one of {_KINDS} or a callable, got {output!r}")


def set_output_as(output: Union[str, Callable[[DeviceArray], Any]]) -> None:
    """'torch' (default), 'raft'/'mivs' (DeviceArray), 'numpy', or a callable taking a DeviceArray.
    Process-wide, like pylibraft's; threads inside an ``output_as`` block keep their own setting."""
    global _global
    _check(output)
    _global = output


def get_output_as():
    """The setting in force on this thread (its ``output_as`` override, else the process-wide hook)."""
    return getattr(_state, "override", None) or _global


@contextmanager
def output_as(output: Union[str, Callable[[DeviceArray], Any]]):
    """Thread-local override of the output hook for the duration of the block (nests)."""
    _check(output)
    prev = getattr(_state, "override", None)
    _state.override = output
    try:
        yield
    finally:
        _state.override = prev


def convert_output(t: torch.Tensor):
    out = get_output_as()
    if callable(out):
        return out(DeviceArray(t))
    if out == "torch":
        return t
    if out in ("raft", "mivs", "cupy"):
        return DeviceArray(t)
    if out == "numpy":
        return t.detach().cpu().numpy()
    raise ValueError(f"unknown output type {out!r}")
