"""Tensor plumbing between PyTorch-ROCm and the C-ABI (device pointers, streams, outputs)."""
from __future__ import annotations

import numpy as np
import torch

from . import config


def as_device_f32(x, device: int | None = None, name: str = "array") -> torch.Tensor:
    """Return a contiguous float32 CUDA (ROCm) tensor holding `x` (copied to `device` if needed)."""
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    elif hasattr(x, "tensor") and isinstance(getattr(x, "tensor"), torch.Tensor):  # DeviceArray
        x = x.tensor
    elif not isinstance(x, torch.Tensor):
        x = torch.as_tensor(x)
    if x.dim() != 2:
        raise ValueError(f"{name} must be a 2-D array, got shape {tuple(x.shape)}")
    if not torch.cuda.is_available():
        raise RuntimeError("mivs needs a ROCm GPU: torch.cuda.is_available() is False")
    if x.is_cuda:
        if device is not None and x.device.index != device:
            x = x.to(f"cuda:{device}")
    else:
        x = x.to(f"cuda:{device if device is not None else torch.cuda.current_device()}")
    if x.dtype != torch.float32:
        x = x.float()
    return x.contiguous()


def stream_ptr(device: int) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def out_tensor(out, shape, dtype, device: int, name: str) -> torch.Tensor:
    if out is None:
        return torch.empty(shape, dtype=dtype, device=f"cuda:{device}")
    t = out.tensor if hasattr(out, "tensor") else out
    if not isinstance(t, torch.Tensor) or tuple(t.shape) != tuple(shape) or t.dtype != dtype or not t.is_cuda \
            or t.device.index != device or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous {dtype} tensor of shape {tuple(shape)} on cuda:{device}")
    return t


def emit(t: torch.Tensor):
    return config.convert_output(t)
