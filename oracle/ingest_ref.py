"""CPU oracle (numpy, float32) of the G-buffer ingest.

TEST INFRASTRUCTURE ONLY. Only ``tests/`` and ``bench.py``'s baseline leg may import this module, as
the checker; the product path (``realtime_style_transfer_amd.dataloaders``) runs rst_gbuffer_preprocess
on the device and never imports it.

Restates, in float32 numpy (no FMA: every product and sum rounds separately, as TF's C++ kernel does):

* ``load_unreal_hdr_screenshot`` channel assembly    dataloaders/hdrScreenshots.py:14-30
  (3-channel entries stack R, G, B; 1-channel entries take R; concatenated in list order)
* ``preprocess_numpy_image``                         dataloaders/common.py:44-57
  - target size: ``(ceil(W * h/w), W)`` if ``h/w > H/W`` else ``(H, ceil(H / (h/w)))`` (Python floats)
  - ``tf.image.resize(image, size)`` = TF 2.9 ResizeBilinear(half_pixel_centers=True, align_corners=False),
    third-party (tensorflow/core/kernels/image/resize_bilinear_op.cc, not vendored in the reference):
      scale = float32(in) / out
      in    = (float32(o) + 0.5) * scale - 0.5                         (HalfPixelScaler)
      lower = max(floor(in), 0); upper = min(ceil(in), in_size - 1); lerp = in - floor(in)
      top = tl + (tr - tl) * xl; bottom = bl + (br - bl) * xl; out = top + (bottom - top) * yl
  - ``tf.image.resize_with_crop_or_pad(image, H, W)``: crop offset ``max((in - H) // 2, 0)``, pad offset
    ``max((H - in) // 2, 0)`` with zeros
* ``load_tensor_from_buffer``                        dataloaders/tensorbuffer.py:8-16
  (the first prod(shape) little-endian float32 values of the file, reshaped)

Parity status: the reference holds no EXR screenshots, tensor buffers or expected outputs, and
TensorFlow is not installed here, so the resize arithmetic is **parity unpinned** against TF itself:
it follows the TF kernel's published algorithm above and is pinned by known-answer cases that hold
for that algorithm (identity size, exact 2x box average, constant images, edge clamping) in
tests/test_ingest.py.
"""
from __future__ import annotations

import math

import numpy as np


def resized_size(src_hw, shape):
    """common.py:46-51 — the aspect-preserving intermediate size (Python float arithmetic)."""
    h, w = src_hw
    aspect_ratio_image = h / w
    aspect_ratio_target = shape[0] / shape[1]
    if aspect_ratio_image > aspect_ratio_target:
        return (math.ceil(shape[1] * aspect_ratio_image), shape[1])
    return (shape[0], math.ceil(shape[0] / aspect_ratio_image))


def _interp(out_size: int, in_size: int):
    scale = np.float32(np.float32(in_size) / np.float32(out_size))
    o = np.arange(out_size, dtype=np.float32)
    pos = (o + np.float32(0.5)) * scale - np.float32(0.5)          # float32 ops, one rounding each
    f = np.floor(pos)
    lower = np.maximum(f.astype(np.int64), 0)
    upper = np.minimum(np.ceil(pos).astype(np.int64), in_size - 1)
    lerp = (pos - f).astype(np.float32)
    return lower, upper, lerp


def resize_bilinear_half_pixel(image: np.ndarray, size) -> np.ndarray:
    """tf.image.resize(image (h, w, C), size) with the default bilinear method, float32."""
    image = np.asarray(image, dtype=np.float32)
    y0, y1, yl = _interp(size[0], image.shape[0])
    x0, x1, xl = _interp(size[1], image.shape[1])
    xl = xl[None, :, None]
    yl = yl[:, None, None]
    tl = image[y0][:, x0]
    tr = image[y0][:, x1]
    bl = image[y1][:, x0]
    br = image[y1][:, x1]
    top = tl + (tr - tl) * xl
    bottom = bl + (br - bl) * xl
    return (top + (bottom - top) * yl).astype(np.float32)


def resize_with_crop_or_pad(image: np.ndarray, target_h: int, target_w: int) -> np.ndarray:
    h, w = image.shape[:2]
    cy, py = max((h - target_h) // 2, 0), max((target_h - h) // 2, 0)
    cx, px = max((w - target_w) // 2, 0), max((target_w - w) // 2, 0)
    out = np.zeros((target_h, target_w) + image.shape[2:], dtype=image.dtype)
    hh, ww = min(h, target_h), min(w, target_w)
    out[py:py + hh, px:px + ww] = image[cy:cy + hh, cx:cx + ww]
    return out


def preprocess_numpy_image(image: np.ndarray, shape) -> np.ndarray:
    """common.py:44-57."""
    resized = resize_bilinear_half_pixel(image, resized_size(image.shape[:2], shape))
    return resize_with_crop_or_pad(resized, shape[0], shape[1])


def assemble_channels(channel_images, expected_channels) -> np.ndarray:
    """hdrScreenshots.py:16-27 — ``channel_images[name]`` is a dict {'R': plane, 'G': ..., 'B': ...}."""
    out = []
    for name, n in expected_channels:
        ch = channel_images[name]
        if n == 3:
            out.append(np.stack([ch['R'], ch['G'], ch['B']], axis=-1))
        elif n == 1:
            out.append(np.expand_dims(ch['R'], axis=-1))
        else:
            out.append(np.stack([v for _, v in ch.items()]))
    return np.concatenate(out, axis=-1)


def load_tensor_from_buffer(path, shape) -> np.ndarray:
    """tensorbuffer.py:8-16 (struct.unpack of little-endian-native float32 values)."""
    n = math.prod(shape)
    raw = open(path, 'rb').read(n * 4)
    return np.frombuffer(raw, dtype='<f4', count=n).astype(np.float32).reshape(shape)
