"""Device plumbing: torch (ROCm) owns HBM allocations and streams; the HIP kernels receive raw pointers.

Every geometry array that feeds a kernel lives as a torch tensor on the current HIP device.  The stream
handed to the C ABI is torch's current stream, so facade calls order correctly with any torch work the
caller does on the same stream.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

try:
    import torch
except Exception:  # pragma: no cover - torch is part of the image
    torch = None


def require_gpu():
    if torch is None or not torch.cuda.is_available():
        raise RuntimeError("otslam-mi355x: a HIP device (MI355X, gfx950) is required for this operation; "
                           "there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    """Raw device pointer of a contiguous tensor (or None)."""
    if t is None:
        return None
    assert t.is_contiguous(), "kernel arguments must be contiguous"
    return C.c_void_p(t.data_ptr())


_TORCH_DT = {np.dtype(np.float64): "float64", np.dtype(np.float32): "float32", np.dtype(np.uint8): "uint8",
             np.dtype(np.uint16): "uint16", np.dtype(np.int32): "int32", np.dtype(np.int64): "int64"}


def to_device(a, dtype=None):
    """numpy array / tensor -> contiguous tensor on the current HIP device."""
    dev = require_gpu()
    if isinstance(a, torch.Tensor):
        t = a
        if dtype is not None:
            t = t.to(getattr(torch, dtype))
        return t.to(dev).contiguous()
    arr = np.ascontiguousarray(a if dtype is None else np.asarray(a, dtype=dtype))
    if arr.dtype == np.uint16:  # torch.from_numpy lacks uint16 on some builds: move the raw bits
        t = torch.from_numpy(arr.view(np.int16)).to(dev).view(torch.uint16)
        return t.contiguous()
    return torch.from_numpy(arr).to(dev).contiguous()


def to_host(t) -> np.ndarray:
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t
    if t.dtype == torch.uint16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    return t.detach().cpu().numpy()


def empty(shape, dtype):
    dev = require_gpu()
    return torch.empty(shape, dtype=getattr(torch, dtype), device=dev)


def is_tensor(a):
    return torch is not None and isinstance(a, torch.Tensor)
