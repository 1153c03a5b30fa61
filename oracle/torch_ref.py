"""Second, independent CPU restatement (torch-CPU, float32) of the transfer network.

TEST INFRASTRUCTURE ONLY (checker + ``bench.py`` ``cpu_baseline`` leg). It never runs
on the GPU and the product path never imports it.

Role: (1) cross-check of oracle/numpy_ref.py — two restatements written against the same
TF semantics must agree to float32 rounding; (2) the CPU baseline: TensorFlow is not
installed here, so the reference's TF-CPU path cannot run; this is the same graph on
torch-CPU (oneDNN) — ``cpu_baseline.kind = "port"``; (3) full-size (480x960x17) parity
on the GPU box, where the float64 numpy oracle would be slow.

Reference anchors are those listed in oracle/numpy_ref.py (styleTransfer.py:12-345).
TF SAME padding is applied with an explicit asymmetric ``F.pad``; a SAME transposed
conv is ``F.conv_transpose2d(padding=0)`` cropped at ``[pad_before : pad_before + in*s]``.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .numpy_ref import transfer_structure


def _same_pads(n_in, k, s):
    n_out = -(-n_in // s)
    total = max((n_out - 1) * s + k - n_in, 0)
    return total // 2, total - total // 2


def conv2d_same(x, w_hwio, b, stride):
    """x NCHW (channels_last ok), w_hwio (kh,kw,cin,cout)."""
    kh, kw = w_hwio.shape[:2]
    pt, pb = _same_pads(x.shape[2], kh, stride)
    pl, pr = _same_pads(x.shape[3], kw, stride)
    x = F.pad(x, (pl, pr, pt, pb))
    w = w_hwio.permute(3, 2, 0, 1).contiguous()
    return F.conv2d(x, w, b, stride=stride)


def conv2d_transpose_same(x, w_hwoi, b, stride):
    """w_hwoi: Keras Conv2DTranspose kernel (kh, kw, out, in)."""
    kh, kw = w_hwoi.shape[:2]
    H, W = x.shape[2], x.shape[3]
    pt = max(kh - stride, 0) // 2
    pl = max(kw - stride, 0) // 2
    w = w_hwoi.permute(3, 2, 0, 1).contiguous()      # (in, out, kh, kw)
    y = F.conv_transpose2d(x, w, None, stride=stride)
    y = y[:, :, pt:pt + H * stride, pl:pl + W * stride]
    return y + b.view(1, -1, 1, 1)


def cin(x, scale, bias, eps=1e-5):
    mean = x.mean(dim=(2, 3), keepdim=True)
    var = ((x - mean) ** 2).mean(dim=(2, 3), keepdim=True)
    inv = torch.rsqrt(var + eps)
    return bias + (x * inv - mean * inv) * scale


class TorchTransfer:
    """Prepared torch-CPU fp32 transfer net (weights converted once)."""

    def __init__(self, weights: Sequence[np.ndarray], input_shape, output_shape, bottleneck_res_y,
                 bottleneck_num_filters, threads=None):
        self.blocks, self.P = transfer_structure(input_shape, output_shape, bottleneck_res_y,
                                                 bottleneck_num_filters)
        self.w = [torch.from_numpy(np.asarray(a, np.float32)) for a in weights]
        if threads:
            torch.set_num_threads(threads)

    @torch.no_grad()
    def __call__(self, content_nhwc: np.ndarray, style_params: np.ndarray) -> np.ndarray:
        x = torch.from_numpy(np.ascontiguousarray(content_nhwc, np.float32)).permute(0, 3, 1, 2)
        x = x.contiguous(memory_format=torch.channels_last)
        sp = torch.from_numpy(np.asarray(style_params, np.float32))
        if sp.shape[1] != 1:
            raise NotImplementedError("torch restatement covers num_styles == 1")
        sp = sp[:, 0, :]
        off = 0
        wi = iter(self.w)
        for kind, k, s, f in self.blocks:
            if kind == 'contract':
                w, b, g, be, mm, mv = (next(wi) for _ in range(6))
                x = F.relu(conv2d_same(x, w, b, s))
                inv = g / torch.sqrt(mv + 1e-3)
                x = F.relu(x * inv.view(1, -1, 1, 1) + (be - mm * inv).view(1, -1, 1, 1))
            elif kind.startswith('residual'):
                inp = x
                for j in range(2):
                    w, b = next(wi), next(wi)
                    x = F.relu(conv2d_same(x, w, b, 1))
                    scale = sp[:, off:off + f].view(-1, f, 1, 1)
                    bias = sp[:, off + f:off + 2 * f].view(-1, f, 1, 1)
                    off += 2 * f
                    x = cin(x, scale, bias)
                    if j == 0:
                        x = F.relu(x)
                if kind != 'residual_first':
                    x = inp + x
            else:
                w, b = next(wi), next(wi)
                x = conv2d_transpose_same(x, w, b, s)
                scale = sp[:, off:off + f].view(-1, f, 1, 1)
                bias = sp[:, off + f:off + 2 * f].view(-1, f, 1, 1)
                off += 2 * f
                x = cin(x, scale, bias)
                x = torch.sigmoid(x) if kind == 'expand_last' else F.relu(x)
        assert off == self.P
        return x.permute(0, 2, 3, 1).contiguous().numpy()


def gram_matrix(features_nhwc: torch.Tensor) -> torch.Tensor:
    B, H, W, C = features_nhwc.shape
    f = features_nhwc.reshape(B, H * W, C)
    return torch.bmm(f.transpose(1, 2), f) / (H * W)
