"""Mirror of realtime_style_transfer/dataloaders/tensorbuffer.py — the raw float32 tensor-buffer
format Unreal dumps (show_unreal_tensor_buffer.py, predict_style_params.py:38-40): the first
prod(shape) little-endian float32 values of the file, row-major in ``shape``."""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np
import torch


def load_tensor_from_buffer(buffer_filepath: Path, shape, device=None) -> torch.Tensor:
    """tensorbuffer.py:8-16; returns a float32 tensor (on ``device`` if given)."""
    num_elements = math.prod(shape)
    with Path(buffer_filepath).open(mode='rb') as f:
        raw = f.read(num_elements * 4)
    if len(raw) != num_elements * 4:   # the reference's struct.unpack raises on a short file
        raise ValueError(f"{buffer_filepath}: {len(raw)} bytes, need {num_elements * 4} for shape {tuple(shape)}")
    t = torch.from_numpy(np.frombuffer(raw, dtype='<f4').astype(np.float32).reshape(shape))
    return t.to(device) if device is not None else t


def save_tensor_to_buffer(buffer_filepath: Path, tensor) -> None:
    """Write ``tensor`` in the same format (little-endian float32, row-major)."""
    a = tensor.detach().cpu().numpy() if isinstance(tensor, torch.Tensor) else np.asarray(tensor)
    Path(buffer_filepath).write_bytes(np.ascontiguousarray(a, dtype='<f4').tobytes())
