"""CPU oracle of one training step (torch-CPU float64 autograd) — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this (it is the checker for ``rst_trainer_*``); the product path
never does. It restates, in float64 with torch autograd as the differentiator:

* the transfer network in Keras training mode (styleTransfer.py:95-276): BatchNormalization
  uses the batch's biased moments over (B, H, W) for normalisation and updates the moving
  statistics with momentum 0.99 and the Bessel-corrected variance (Keras fused batch norm);
  conditional instance norm uses per-image moments (styleTransfer.py:57-71);
* the VGG16 / Gram loss without the depth term (styleLoss.py:69-109, 290-369): x*255,
  RGB->BGR, minus the caffe mean, 13 convs + 4 max-pools, feature loss on block5_conv3,
  style loss = mean over four Gram layers, total variation (tf.image.total_variation);
* the gradient of the batch-summed loss (Keras minimises the (B,) loss vector), w.r.t. every
  trainable transfer weight and the style parameters;
* RMSprop as Keras OptimizerV2 with momentum 0 (train_network.py:102):
  ms = rho*ms + (1-rho)*g^2; w -= lr*g/(sqrt(ms)+eps); slots start at zero.

Parity status: the forward pieces are the same restatement as oracle/numpy_ref.py and
oracle/torch_ref.py (pinned by the golden fixtures and the apply_style_weights KAT);
the gradients are torch autograd of that restatement, checked against central finite
differences in tests/test_oracle.py. The reference's own tests pin no training numbers
("parity unpinned" for the TF training step itself).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .numpy_ref import CONTENT_LAYERS, STYLE_LAYERS, VGG16_LAYERS, VGG_MEAN_BGR, bf16_round, transfer_structure
from .torch_ref import cin, conv2d_same, conv2d_transpose_same

BN_MOMENTUM = 0.99
BN_EPS = 1e-3


def transfer_forward_train(content, style_params, w: Sequence[torch.Tensor], blocks, bn_mode="train", taps=None):
    """content NCHW float64; style_params (B, P); w in Keras get_weights() order.

    Returns (prediction NCHW, list of (mean, unbiased var) per BatchNorm layer). With ``taps``
    (a list), every conv layer's activated output (before a skip add) is appended with
    ``retain_grad`` so its gradient can be read after backward."""
    x = content
    off = 0
    wi = iter(w)
    bn_stats = []

    def tap(t):
        if taps is not None and t.requires_grad:
            t.retain_grad()
            taps.append(t)
        return t

    for kind, k, s, f in blocks:
        if kind == 'contract':
            kw, b, g, be, mm, mv = (next(wi) for _ in range(6))
            x = F.relu(conv2d_same(x, kw, b, s))
            if bn_mode == "train":
                mean = x.mean(dim=(0, 2, 3))
                var = ((x - mean.view(1, -1, 1, 1)) ** 2).mean(dim=(0, 2, 3))
                n = x.shape[0] * x.shape[2] * x.shape[3]
                bn_stats.append((mean.detach(), var.detach() * n / max(n - 1, 1)))
            else:
                mean, var = mm, mv
            inv = torch.rsqrt(var + BN_EPS)
            x = (x - mean.view(1, -1, 1, 1)) * inv.view(1, -1, 1, 1) * g.view(1, -1, 1, 1) + be.view(1, -1, 1, 1)
            x = tap(F.relu(x))
        elif kind.startswith('residual'):
            inp = x
            for j in range(2):
                kw, b = next(wi), next(wi)
                x = F.relu(conv2d_same(x, kw, b, 1))
                scale = style_params[:, off:off + f].reshape(-1, f, 1, 1)
                bias = style_params[:, off + f:off + 2 * f].reshape(-1, f, 1, 1)
                off += 2 * f
                x = cin(x, scale, bias)
                if j == 0:
                    x = F.relu(x)
                x = tap(x)
            if kind != 'residual_first':
                x = inp + x
        else:
            kw, b = next(wi), next(wi)
            x = conv2d_transpose_same(x, kw, b, s)
            scale = style_params[:, off:off + f].reshape(-1, f, 1, 1)
            bias = style_params[:, off + f:off + 2 * f].reshape(-1, f, 1, 1)
            off += 2 * f
            x = cin(x, scale, bias)
            x = tap(torch.sigmoid(x) if kind == 'expand_last' else F.relu(x))
    return x, bn_stats


class _RoutedMaxPool2(torch.autograd.Function):
    """2x2 max-pool whose backward sends each window's gradient to the first maximum of a
    supplied routing tensor (the implementation-under-test's float32 activations) instead of
    this float64 tensor. Forward values are the float64 maxima. Only the measure-zero choice
    between near-equal window values is aligned; see tests/test_gpu_train.py."""

    @staticmethod
    def forward(ctx, x, route):
        B, C, H, W = x.shape
        win = route.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
        m = win.max(dim=-1, keepdim=True).values
        first = (win == m).to(torch.int64).argmax(dim=-1)            # first maximum in scan order
        ctx.save_for_backward(first)
        ctx.shape = x.shape
        return F.max_pool2d(x, 2)

    @staticmethod
    def backward(ctx, gy):
        (first,) = ctx.saved_tensors
        B, C, H, W = ctx.shape
        onehot = F.one_hot(first, 4).to(gy.dtype) * gy.unsqueeze(-1)
        gx = onehot.reshape(B, C, H // 2, W // 2, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H, W)
        return gx, None


class _RoutedRelu(torch.autograd.Function):
    """ReLU whose backward mask (which units pass the gradient) comes from a supplied routing tensor
    (the implementation-under-test's float32 post-ReLU activations: unit active iff > 0) instead of
    this float64 tensor's sign. Forward values are the float64 ReLU. Only the measure-zero decision at
    pre-activations within rounding distance of 0 is aligned (same idea as _RoutedMaxPool2)."""

    @staticmethod
    def forward(ctx, x, route):
        mask = (route > 0).to(x.dtype)
        ctx.save_for_backward(mask)
        return F.relu(x)

    @staticmethod
    def backward(ctx, gy):
        (mask,) = ctx.saved_tensors
        return gy * mask, None


def _bf16(t: torch.Tensor) -> torch.Tensor:
    return torch.from_numpy(bf16_round(t.detach().numpy())).to(t.dtype)


class _Bf16Conv(torch.autograd.Function):
    """A VGG16 conv in the device's RST_PRECISION_BF16 arithmetic: forward on bf16-rounded input and
    kernel, input gradient from the bf16-rounded output gradient and kernel (products exact in
    float64, as they are in the fp32 accumulators), rounded to bf16 as the device stores it. The kernel is frozen
    (no weight gradient)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(w)
        ctx.xshape = x.shape
        return conv2d_same(_bf16(x), _bf16(w), b, 1)

    @staticmethod
    def backward(ctx, gy):
        (w,) = ctx.saved_tensors
        xd = torch.zeros(ctx.xshape, dtype=gy.dtype, requires_grad=True)
        with torch.enable_grad():
            y = conv2d_same(xd, _bf16(w), None, 1)
            (gx,) = torch.autograd.grad(y, xd, _bf16(gy))
        return _bf16(gx), None, None   # the input gradient is stored as bf16 (a pool's input gradient routes it as is)


class _Bf16FwdConv(torch.autograd.Function):
    """block1_conv1 in the device's plain-bf16 loss: forward on the bf16-rounded preprocessed image and
    kernel (vgg_conv0_bf16); its input gradient (the gradient reaching the prediction) is the f32 path
    (train_api vgg_backward: 1x1 conv + tap sum on unrounded weights), so the backward is the exact one."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(w)
        ctx.xshape = x.shape
        return conv2d_same(_bf16(x), _bf16(w), b, 1)

    @staticmethod
    def backward(ctx, gy):
        (w,) = ctx.saved_tensors
        xd = torch.zeros(ctx.xshape, dtype=gy.dtype, requires_grad=True)
        with torch.enable_grad():
            y = conv2d_same(xd, w, None, 1)
            (gx,) = torch.autograd.grad(y, xd, gy)
        return gx, None, None


class _Bf16Store(torch.autograd.Function):
    """A mixed_bfloat16 layer output: the value rounded to bf16 (the device stores every VGG16 layer output as bf16
    bits in the plain-bf16 loss), and so is its gradient — the sum of what flows back into it (the next conv's or pool's
    input gradient, the Gram's and the content term's), each contribution already bf16, rounded once."""

    @staticmethod
    def forward(ctx, x):
        return _bf16(x)

    @staticmethod
    def backward(ctx, gy):
        return _bf16(gy)


def vgg_features(images01, vgg: Sequence[torch.Tensor], taps=None, route=None,
                 bf16: bool = False, relu_route=None) -> Dict[str, torch.Tensor]:
    """StyleLossModelVGG.call (styleLoss.py:106-109) on NCHW float64 images in [0, 1].
    ``taps``: list receiving every conv output (retain_grad) when the input requires grad.
    ``route``: {conv index: NCHW activations} whose window maxima route the max-pool backward.
    ``bf16``: every conv in bf16 arithmetic (_Bf16Conv; the first, whose input gradient stays f32 on the
    device, _Bf16FwdConv) and every layer output stored in bf16 (_Bf16Store).
    ``relu_route``: {conv index: NCHW post-ReLU activations} whose positive units set the ReLU backward mask."""
    x = images01 * 255.0
    mean = torch.tensor(VGG_MEAN_BGR, dtype=x.dtype).view(1, 3, 1, 1)
    x = x.flip(1) - mean
    feats = {}
    i = 0
    for entry in VGG16_LAYERS:
        if entry[0] == 'pool':
            if route is not None and (i - 1) in route:
                x = _RoutedMaxPool2.apply(x, route[i - 1])
            else:
                x = F.max_pool2d(x, 2)
            continue
        name = entry[0]
        if bf16 and i > 0:
            x = _Bf16Conv.apply(x, vgg[2 * i], vgg[2 * i + 1])
        elif bf16:
            x = _Bf16FwdConv.apply(x, vgg[2 * i], vgg[2 * i + 1])
        else:
            x = conv2d_same(x, vgg[2 * i], vgg[2 * i + 1], 1)
        x = _RoutedRelu.apply(x, relu_route[i]) if relu_route is not None and i in relu_route else F.relu(x)
        if bf16:
            x = _Bf16Store.apply(x)
        i += 1
        if taps is not None and x.requires_grad:
            x.retain_grad()
            taps.append(x)
        if name in STYLE_LAYERS or name in CONTENT_LAYERS:
            feats[name] = x
        if name == CONTENT_LAYERS[0]:
            break
    return feats


def _gram(f):
    B, C, H, W = f.shape
    f2 = f.reshape(B, C, H * W)
    return torch.bmm(f2, f2.transpose(1, 2)) / (H * W)


class _Bf16Gram(torch.autograd.Function):
    """The device's RST_PRECISION_BF16 Gram (gram.hip gram_partial_bf16_kernel): forward on bf16-rounded
    features (products exact, float64 sums); backward as the device's Gram backward (train_api vgg_backward:
    a conv_bf3 1x1 conv), dF = W F with W = (dG + dG^T) / HW rounded to bf16 when packed and F rounded to
    bf16 as the conv stages it."""

    @staticmethod
    def forward(ctx, f):
        ctx.save_for_backward(f)
        return _gram(_bf16(f))

    @staticmethod
    def backward(ctx, gg):
        (f,) = ctx.saved_tensors
        B, C, H, W = f.shape
        f2 = _bf16(f.reshape(B, C, H * W))
        w = _bf16((gg + gg.transpose(1, 2)) / (H * W))
        return torch.bmm(w, f2).reshape(B, C, H, W)   # f32 on the device; the sum with the pool's gradient is rounded once


def _mean_l2(t):
    return (0.5 * t ** 2).reshape(t.shape[0], -1).mean(dim=1)


def style_losses(pred, content, style, vgg, content_factor=1e4, style_factor=1e-3, tv_factor=1e-1, taps=None,
                 route=None, bf16=False, relu_route=None):
    """make_style_loss_function without depth (styleLoss.py:295-369) -> (B, 4) [loss, feature, style, tv]."""
    fp = vgg_features(pred, vgg, taps, route, bf16, relu_route)
    fc, fs = vgg_features(content, vgg, bf16=bf16), vgg_features(style, vgg, bf16=bf16)
    feature = torch.stack([_mean_l2(fp[n] - fc[n]) for n in CONTENT_LAYERS]).mean(0) * content_factor
    gram = _Bf16Gram.apply if bf16 else _gram   # plain-bf16 loss: Grams on bf16-rounded features too
    style_l = torch.stack([_mean_l2(gram(fp[n]) - gram(fs[n])) for n in STYLE_LAYERS]).mean(0) * style_factor
    tv = ((pred[:, :, 1:, :] - pred[:, :, :-1, :]).abs().sum(dim=(1, 2, 3)) +
          (pred[:, :, :, 1:] - pred[:, :, :, :-1]).abs().sum(dim=(1, 2, 3))) * tv_factor
    return torch.stack([feature + style_l + tv, feature, style_l, tv], dim=1)


def _nchw(a, dtype=torch.float64):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype).permute(0, 3, 1, 2)


def training_step(weights: Sequence[np.ndarray], vgg_weights: Sequence[np.ndarray], content, style_params,
                  gt_content, gt_style, input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters,
                  factors=(1e4, 1e-3, 1e-1), ms: Optional[Sequence[np.ndarray]] = None,
                  lr=1e-3, rho=0.9, eps=1e-7, pool_route: Optional[Dict[int, np.ndarray]] = None,
                  vgg_bf16: bool = False, relu_route: Optional[Dict[int, np.ndarray]] = None,
                  dtype=torch.float64) -> Dict[str, object]:
    """One Keras train_step: forward (BN training mode), loss, gradients, RMSprop.

    Inputs are NHWC numpy; returns numpy: prediction (B,H,W,3), losses (B,4), grads (Keras order;
    zeros for the BN moving statistics), grad_style_params (B,P), weights after the update
    (moving statistics updated by the forward), ms (RMSprop slots after the update).
    ``pool_route``: {VGG conv index before a pool: NHWC activations of the prediction} to align
    the max-pool backward's choice among near-equal maxima with an implementation under test;
    ``relu_route``: {VGG conv index: NHWC post-ReLU activations of the prediction} aligning the ReLU
    backward masks the same way (pre-activations within rounding distance of 0).
    ``dtype``: torch.float64 (the checker) or torch.float32 (bench.py's CPU baseline of the step: the same
    graph in the reference's own fp32 arithmetic)."""
    blocks, P = transfer_structure(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters)
    w = [torch.tensor(np.asarray(a, np.float64), dtype=dtype, requires_grad=True) for a in weights]
    vgg = [torch.tensor(np.asarray(a, np.float64), dtype=dtype) for a in vgg_weights]
    sp = torch.tensor(np.asarray(style_params, np.float64).reshape(len(content), P), dtype=dtype, requires_grad=True)
    gts = np.asarray(gt_style)
    if gts.ndim == 5:
        gts = gts[:, 0]
    taps = []
    pred, bn_stats = transfer_forward_train(_nchw(content, dtype), sp, w, blocks, taps=taps)
    vtaps = []
    route = None if pool_route is None else {k: _nchw(v, dtype) for k, v in pool_route.items()}
    rroute = None if relu_route is None else {k: _nchw(v, dtype) for k, v in relu_route.items()}
    losses = style_losses(pred, _nchw(gt_content, dtype), _nchw(gts, dtype), vgg, *factors, taps=vtaps, route=route,
                          bf16=vgg_bf16, relu_route=rroute)
    losses[:, 0].sum().backward()
    # Keras trainable set: conv kernels/biases, BN gamma/beta (moving statistics are not trained)
    grads, new_w, new_ms = [], [], []
    trainable = []
    for kind, k, s, f in blocks:
        n = 6 if kind == 'contract' else (4 if kind.startswith('residual') else 2)
        trainable += [not (kind == 'contract' and j >= 4) for j in range(n)]
    bn_i = 0
    ms = [np.zeros_like(np.asarray(a, np.float64)) for a in weights] if ms is None else \
        [np.asarray(m, np.float64) for m in ms]
    for i, (t, tr) in enumerate(zip(w, trainable)):
        g = t.grad.detach().numpy() if (tr and t.grad is not None) else np.zeros(t.shape)
        grads.append(g)
        m = rho * ms[i] + (1.0 - rho) * g * g
        new_ms.append(m)
        new_w.append(t.detach().numpy() - lr * g / (np.sqrt(m) + eps))
    # moving statistics (contract blocks: weights 4 and 5 of each 6-group)
    i = 0
    for kind, k, s, f in blocks:
        if kind == 'contract':
            mean, var = bn_stats[bn_i]
            bn_i += 1
            new_w[i + 4] = BN_MOMENTUM * np.asarray(weights[i + 4], np.float64) + (1 - BN_MOMENTUM) * mean.numpy()
            new_w[i + 5] = BN_MOMENTUM * np.asarray(weights[i + 5], np.float64) + (1 - BN_MOMENTUM) * var.numpy()
            i += 6
        else:
            i += 4 if kind.startswith('residual') else 2
    return {
        'prediction': pred.detach().permute(0, 2, 3, 1).numpy(),
        'losses': losses.detach().numpy(),
        'grads': grads,
        'grad_style_params': sp.grad.detach().numpy(),
        'weights': new_w,
        'ms': new_ms,
        'output_grads': [t.grad.detach().permute(0, 2, 3, 1).numpy() for t in taps],
        'vgg_grads': [t.grad.detach().permute(0, 2, 3, 1).numpy() for t in vtaps],
    }


def loss_of(weights, vgg_weights, content, style_params, gt_content, gt_style, input_shape, output_shape,
            bottleneck_res_y, bottleneck_num_filters, factors=(1e4, 1e-3, 1e-1)) -> float:
    """Batch-summed training-mode loss (finite-difference checks of the oracle's gradients)."""
    blocks, P = transfer_structure(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters)
    with torch.no_grad():
        w = [torch.tensor(np.asarray(a, np.float64)) for a in weights]
        vgg = [torch.tensor(np.asarray(a, np.float64)) for a in vgg_weights]
        sp = torch.tensor(np.asarray(style_params, np.float64).reshape(len(content), P))
        gts = np.asarray(gt_style)
        if gts.ndim == 5:
            gts = gts[:, 0]
        pred, _ = transfer_forward_train(_nchw(content), sp, w, blocks)
        return float(style_losses(pred, _nchw(gt_content), _nchw(gts), vgg, *factors)[:, 0].sum())
