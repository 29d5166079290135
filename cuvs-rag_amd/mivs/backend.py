"""Backend availability shared by the drop-in managers.

The reference flips its managers between real cuVS calls and a simulation
(``CUVS_AVAILABLE``, index_building_coordinator.py:25-30) that its mock tests rely on.
Here the flag means "the mivs HIP engine is usable": libmivs.so loads AND a ROCm GPU is
visible. On a machine WITH a GPU a missing/unloadable libmivs.so is an import error —
never a silent simulation or CPU fallback.
"""
from __future__ import annotations

import torch

from . import _native


def engine_available() -> bool:
    try:
        gpu = torch.cuda.is_available()
    except Exception:
        gpu = False
    if not gpu:
        return False
    _native.load()  # raises NativeLibraryMissing on a GPU machine without the built engine
    return True
