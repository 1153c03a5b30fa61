"""Mirror of realtime_style_transfer/dataloaders/common.py — the preprocessing on the hot path.

``preprocess_numpy_image(image, shape)`` (common.py:44-57) runs on the device through
``rst_gbuffer_preprocess`` (ingest.hip): TF bilinear half-pixel resize to the aspect-preserving size,
then the center crop of ``resize_with_crop_or_pad``, in one pass, bit-identical to TF's f32 kernel
arithmetic. It returns a device ``torch.Tensor`` (the reference returns a ``tf.Tensor``).
``preprocess_planes`` takes the per-channel planes directly, so the channel concatenation of
hdrScreenshots.py:27 never happens on the host.
"""
from __future__ import annotations

import ctypes
import math
from typing import Sequence

import numpy as np
import torch

from .. import _lib


def resized_size(src_hw, shape):
    """The intermediate size of common.py:46-51 (as computed by librst)."""
    out = (ctypes.c_int * 2)()
    _lib.check(_lib.load().rst_gbuffer_resized_size(int(src_hw[0]), int(src_hw[1]), int(shape[0]), int(shape[1]), out))
    return (out[0], out[1])


def preprocess_planes(planes: Sequence[torch.Tensor], shape, out: torch.Tensor = None) -> torch.Tensor:
    """Channel planes (each (h, w) float32 on the device, or views with a pixel stride) -> (H, W, C)."""
    if len(planes) == 0:
        raise ValueError("preprocess_planes: no channel planes")
    h, w = planes[0].shape[:2]
    for p in planes:
        if p.shape[:2] != (h, w):
            raise ValueError(f"preprocess_planes: plane shapes differ: {tuple(p.shape)} vs {(h, w)}")
        if p.dtype != torch.float32 or not p.is_cuda:
            raise ValueError("preprocess_planes: planes must be float32 device tensors")
    rs, ps = planes[0].stride(0), planes[0].stride(1)
    if any(p.stride(0) != rs or p.stride(1) != ps for p in planes):
        raise ValueError("preprocess_planes: planes must share one (row, pixel) stride")
    H, W = int(shape[0]), int(shape[1])
    if out is None:
        out = torch.empty((H, W, len(planes)), dtype=torch.float32, device=planes[0].device)
    elif tuple(out.shape) != (H, W, len(planes)) or not out.is_contiguous():
        raise ValueError(f"preprocess_planes: out must be a contiguous {(H, W, len(planes))} tensor")
    ptrs = (ctypes.c_void_p * len(planes))(*[p.data_ptr() for p in planes])
    _lib.check(_lib.load().rst_gbuffer_preprocess(ptrs, len(planes), h, w, rs, ps, _lib.dev_ptr(out), H, W,
                                                  _lib.stream_ptr()))
    return out


def preprocess_numpy_image(image, shape, device=None, out: torch.Tensor = None) -> torch.Tensor:
    """common.py:44-57: (h, w, C) image (numpy or tensor) -> device (shape[0], shape[1], C)."""
    t = torch.as_tensor(np.ascontiguousarray(image, dtype=np.float32)) if isinstance(image, np.ndarray) else image
    if t.dim() != 3:
        raise ValueError(f"preprocess_numpy_image: expected an (h, w, C) image, got {tuple(t.shape)}")
    t = t.to(device=device or torch.device('cuda'), dtype=torch.float32).contiguous()
    return preprocess_planes([t[:, :, k] for k in range(t.shape[2])], shape, out=out)
