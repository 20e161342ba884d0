"""Device ops.

``cuda`` tensors run the hand-written gfx950 HIP kernels compiled into the
in-tree extension ``hfens/ops/_hfens_hip*.so`` (see :mod:`hfens.ops.build`);
host tensors run the plain-PyTorch references in :mod:`hfens.ops.reference`
(the same references the kernel numerics tests compare against).  There is no
silent fallback: a ``cuda`` tensor with the extension missing raises.
"""
from __future__ import annotations

import importlib
import os
import sys

import torch

_EXT = None
_EXT_ERR = None


def ext():
    """Load (never build) the compiled HIP extension; raise loudly if absent."""
    global _EXT, _EXT_ERR
    if _EXT is not None:
        return _EXT
    if _EXT_ERR is not None:
        raise _EXT_ERR
    here = os.path.dirname(os.path.abspath(__file__))
    if here not in sys.path:
        sys.path.insert(0, here)
    try:
        _EXT = importlib.import_module("_hfens_hip")
    except ImportError as e:  # pragma: no cover - exercised on misconfigured boxes
        _EXT_ERR = RuntimeError(
            "hfens HIP extension _hfens_hip is not built/loadable "
            f"({e}); run `python -m hfens.ops.build` (gfx950) first")
        raise _EXT_ERR
    return _EXT


def has_ext() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


from .api import *  # noqa: E402,F401,F403
