"""CPU oracle (numpy float64 + an independent torch-CPU float32 restatement) of the style predictor.

TEST INFRASTRUCTURE ONLY: imported by tests/ and tests/golden/make_golden.py as the checker.
The product path (realtime_style_transfer_amd) never imports it.

Restates ``create_style_prediction_model`` (realtime_style_transfer/models/stylePrediction.py:25-75):

* ``StyleFeatureExtractor.DUMMY``: ``Conv2D(1, 9, strides=5, padding='same')`` (with bias, no
  activation) on the raw image (stylePrediction.py:31-32).
* ``StyleFeatureExtractor.MOBILE_NET``: ``Rescaling(2.0, -1.0)`` (:38) then
  ``tf.keras.applications.MobileNetV3Small(include_top=False, include_preprocessing=False)``
  (:33-37; alpha 1.0, minimalistic False). The MobileNetV3 graph lives in Keras 2.9
  (``keras/applications/mobilenet_v3.py``, pinned by the reference's environment.yml:6,8-9 —
  TensorFlow/Keras 2.9.*), which is not vendored under /root/reference nor installed here; its
  published structure is restated below:
    - stem: Conv2D(16, 3, s2, same, no bias) -> BN(eps 1e-3) -> hard_swish
    - 11 inverted-residual blocks (expansion, filters, kernel, stride, SE, activation):
      (1,16,3,2,SE,relu) (72/16,24,3,2,-,relu) (88/24,24,3,1,-,relu) (4,40,5,2,SE,hs)
      (6,40,5,1,SE,hs) (6,40,5,1,SE,hs) (3,48,5,1,SE,hs) (3,48,5,1,SE,hs) (6,96,5,2,SE,hs)
      (6,96,5,1,SE,hs) (6,96,5,1,SE,hs); each block: [1x1 expand to _depth(cin*e) -> BN -> act]
      (not block 0) -> [ZeroPadding2D(correct_pad) if s2] DepthwiseConv2D(k, s, 'same'|'valid', no
      bias) -> BN -> act -> [SE: GAP -> Conv2D(_depth(C/4), 1) -> ReLU -> Conv2D(C, 1) ->
      hard_sigmoid -> x * s] -> 1x1 project (no bias) -> BN -> [+ shortcut if s1 and cin == cout]
    - head: Conv2D(_depth(96*6) = 576, 1, no bias) -> BN -> hard_swish
    - hard_sigmoid(x) = ReLU(6)(x + 3) * (1/6); hard_swish(x) = x * hard_sigmoid(x)
* ``GlobalAveragePooling2D(keepdims=True)`` (:55) -> ``Conv2D(num_style_parameters=100, 1)``
  (:60-64) -> ``Conv2D(num_top_parameters, 1)`` (:67-71) -> squeeze -> float32 (:73-74). No
  activation between the two heads.

Weights are consumed in Keras ``get_weights()`` order: per layer kernel[, bias]; BatchNormalization
gamma, beta, moving_mean, moving_variance (inference: moving statistics).

Parity status: the reference pins no numerics of the predictor (its tests only run the DUMMY
extractor on zeros for shapes, styleTransferInferenceModelTest.py:47-53); ImageNet weights are not
available offline. The two restatements here (float64 loops / torch float32 with grouped convs)
must agree, and the committed golden fixture (tests/golden/predictor_*.npz) freezes them:
**parity unpinned** against Keras itself.
"""
from __future__ import annotations

from typing import Iterator, List, Sequence, Tuple

import numpy as np

BN_EPS = 1e-3

# (expansion, filters, kernel, stride, se, activation) — MobileNetV3Small stack_fn
MOBILENET_V3_SMALL_BLOCKS = [
    (1.0, 16, 3, 2, True, 'relu'),
    (72.0 / 16, 24, 3, 2, False, 'relu'),
    (88.0 / 24, 24, 3, 1, False, 'relu'),
    (4.0, 40, 5, 2, True, 'hard_swish'),
    (6.0, 40, 5, 1, True, 'hard_swish'),
    (6.0, 40, 5, 1, True, 'hard_swish'),
    (3.0, 48, 5, 1, True, 'hard_swish'),
    (3.0, 48, 5, 1, True, 'hard_swish'),
    (6.0, 96, 5, 2, True, 'hard_swish'),
    (6.0, 96, 5, 1, True, 'hard_swish'),
    (6.0, 96, 5, 1, True, 'hard_swish'),
]
SE_RATIO = 0.25


def make_divisible(v: float, divisor: int = 8) -> int:
    """keras mobilenet_v3._depth."""
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def hard_sigmoid(x):
    return np.minimum(np.maximum(x + 3.0, 0.0), 6.0) * (1.0 / 6.0)


def hard_swish(x):
    return x * hard_sigmoid(x)


def relu(x):
    return np.maximum(x, 0.0)


ACT = {'relu': relu, 'hard_swish': hard_swish}


def _same(n, k, s):
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2, total - total // 2


def correct_pad(hw, k):
    """keras imagenet_utils.correct_pad for a known input size -> ((top, bottom), (left, right))."""
    adjust = (1 - hw[0] % 2, 1 - hw[1] % 2)
    c = k // 2
    return (c - adjust[0], c), (c - adjust[1], c)


def conv2d(x, w, b, stride, pads):
    """x (B,H,W,Cin) float64, w (kh,kw,Cin,Cout), pads ((t,b),(l,r)) -> valid conv on the padded map."""
    B, H, W, _ = x.shape
    kh, kw, _, cout = w.shape
    xp = np.pad(x, ((0, 0), pads[0], pads[1], (0, 0)))
    Ho = (H + sum(pads[0]) - kh) // stride + 1
    Wo = (W + sum(pads[1]) - kw) // stride + 1
    out = np.zeros((B, Ho, Wo, cout))
    for ky in range(kh):
        for kx in range(kw):
            patch = xp[:, ky:ky + stride * (Ho - 1) + 1:stride, kx:kx + stride * (Wo - 1) + 1:stride, :]
            out += patch @ np.asarray(w[ky, kx], np.float64)
    if b is not None:
        out += np.asarray(b, np.float64)
    return out


def conv2d_same(x, w, b, stride):
    _, pt, pb = _same(x.shape[1], w.shape[0], stride)
    _, pl, pr = _same(x.shape[2], w.shape[1], stride)
    return conv2d(x, w, b, stride, ((pt, pb), (pl, pr)))


def depthwise(x, w, stride, pads):
    """DepthwiseConv2D (depth multiplier 1): w (kh,kw,C,1)."""
    B, H, W, C = x.shape
    kh, kw = w.shape[:2]
    xp = np.pad(x, ((0, 0), pads[0], pads[1], (0, 0)))
    Ho = (H + sum(pads[0]) - kh) // stride + 1
    Wo = (W + sum(pads[1]) - kw) // stride + 1
    out = np.zeros((B, Ho, Wo, C))
    for ky in range(kh):
        for kx in range(kw):
            patch = xp[:, ky:ky + stride * (Ho - 1) + 1:stride, kx:kx + stride * (Wo - 1) + 1:stride, :]
            out += patch * np.asarray(w[ky, kx, :, 0], np.float64)
    return out


def batch_norm(x, gamma, beta, mean, var, eps=BN_EPS):
    g, b, m, v = (np.asarray(a, np.float64) for a in (gamma, beta, mean, var))
    return (x - m) / np.sqrt(v + eps) * g + b


def mobilenet_v3_small_structure(input_hw: Tuple[int, int]):
    """Layer list [(kind, params...)] with weight shapes in Keras get_weights() order."""
    shapes: List[Tuple[int, ...]] = [(3, 3, 3, 16)] + [(16,)] * 4
    cin = 16
    for bi, (e, f, k, s, se, act) in enumerate(MOBILENET_V3_SMALL_BLOCKS):
        ce = make_divisible(cin * e)
        if bi:
            shapes += [(1, 1, cin, ce)] + [(ce,)] * 4
        shapes += [(k, k, ce, 1)] + [(ce,)] * 4
        if se:
            r = make_divisible(ce * SE_RATIO)
            shapes += [(1, 1, ce, r), (r,), (1, 1, r, ce), (ce,)]
        shapes += [(1, 1, ce, f)] + [(f,)] * 4
        cin = f
    last = make_divisible(cin * 6)
    shapes += [(1, 1, cin, last)] + [(last,)] * 4
    return shapes, last


def mobilenet_v3_small(x, wi: Iterator[np.ndarray], return_blocks=False):
    """MobileNetV3Small(include_top=False, include_preprocessing=False) on x (B,H,W,3) float64."""
    blocks = []
    x = conv2d_same(x, next(wi), None, 2)
    x = hard_swish(batch_norm(x, next(wi), next(wi), next(wi), next(wi)))
    cin = 16
    for bi, (e, f, k, s, se, act_name) in enumerate(MOBILENET_V3_SMALL_BLOCKS):
        act = ACT[act_name]
        shortcut = x
        ce = make_divisible(cin * e)
        if bi:
            x = conv2d(x, next(wi), None, 1, ((0, 0), (0, 0)))
            x = act(batch_norm(x, next(wi), next(wi), next(wi), next(wi)))
        if s == 2:
            pads = correct_pad(x.shape[1:3], k)
        else:
            _, pt, pb = _same(x.shape[1], k, 1)
            _, pl, pr = _same(x.shape[2], k, 1)
            pads = ((pt, pb), (pl, pr))
        x = depthwise(x, next(wi), s, pads)
        x = act(batch_norm(x, next(wi), next(wi), next(wi), next(wi)))
        if se:
            g = x.mean(axis=(1, 2), keepdims=True)
            w1, b1, w2, b2 = next(wi), next(wi), next(wi), next(wi)
            g = relu(conv2d(g, w1, b1, 1, ((0, 0), (0, 0))))
            g = hard_sigmoid(conv2d(g, w2, b2, 1, ((0, 0), (0, 0))))
            x = x * g
        x = conv2d(x, next(wi), None, 1, ((0, 0), (0, 0)))
        x = batch_norm(x, next(wi), next(wi), next(wi), next(wi))
        if s == 1 and cin == f:
            x = shortcut + x
        cin = f
        blocks.append(x)
    x = conv2d(x, next(wi), None, 1, ((0, 0), (0, 0)))
    x = hard_swish(batch_norm(x, next(wi), next(wi), next(wi), next(wi)))
    return (x, blocks) if return_blocks else x


def predictor_weight_shapes(input_shape, extractor: str, num_top_parameters: int, num_style_parameters: int = 100):
    if extractor == 'DUMMY':
        shapes, c = [(9, 9, input_shape[2], 1), (1,)], 1
    elif extractor == 'MOBILE_NET':
        shapes, c = mobilenet_v3_small_structure(input_shape[:2])
    else:
        raise ValueError(extractor)
    shapes += [(1, 1, c, num_style_parameters), (num_style_parameters,),
               (1, 1, num_style_parameters, num_top_parameters), (num_top_parameters,)]
    return shapes


def style_predictor_forward(style, weights: Sequence[np.ndarray], extractor: str, return_features=False):
    """create_style_prediction_model(...)(style) in float64: style (B,H,W,3) -> (B, num_top_parameters)."""
    x = np.asarray(style, np.float64)
    wi = iter(weights)
    if extractor == 'DUMMY':
        x = conv2d_same(x, next(wi), next(wi), 5)                       # stylePrediction.py:31-32
    elif extractor == 'MOBILE_NET':
        x = x * 2.0 - 1.0                                                # Rescaling(2.0, -1.0) :38
        x = mobilenet_v3_small(x, wi)
    else:
        raise ValueError(extractor)
    feat = x
    g = x.mean(axis=(1, 2))                                              # GAP :55
    w1, b1, w2, b2 = next(wi), next(wi), next(wi), next(wi)
    h = g @ np.asarray(w1[0, 0], np.float64) + np.asarray(b1, np.float64)       # :60-64
    y = h @ np.asarray(w2[0, 0], np.float64) + np.asarray(b2, np.float64)       # :67-71
    assert next(wi, None) is None, "unused weights"
    return (y, feat) if return_features else y


# ----------------------------------------------------------------------------- torch float32 restatement

def torch_style_predictor_forward(style, weights: Sequence[np.ndarray], extractor: str):
    """Independent restatement on torch-CPU float32 (grouped conv for the depthwise layers)."""
    import torch
    import torch.nn.functional as F

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a, np.float32))

    def conv(x, w, b, stride, pads, groups=1):
        (pt, pb), (pl, pr) = pads
        x = F.pad(x, (pl, pr, pt, pb))
        wt = t(w).permute(3, 2, 0, 1) if groups == 1 else t(w).permute(2, 3, 0, 1)
        return F.conv2d(x, wt.contiguous(), None if b is None else t(b), stride=stride, groups=groups)

    def same(x, k, s):
        _, pt, pb = _same(x.shape[2], k, s)
        _, pl, pr = _same(x.shape[3], k, s)
        return (pt, pb), (pl, pr)

    def bn(x, g, b, m, v):
        scale = t(g) / torch.sqrt(t(v) + BN_EPS)
        return x * scale[None, :, None, None] + (t(b) - t(m) * scale)[None, :, None, None]

    def hsig(x):
        return F.relu6(x + 3.0) * (1.0 / 6.0)

    def hsw(x):
        return x * hsig(x)

    acts = {'relu': F.relu, 'hard_swish': hsw}
    wi = iter(weights)
    x = t(style).permute(0, 3, 1, 2)
    with torch.no_grad():
        if extractor == 'DUMMY':
            w = next(wi)
            x = conv(x, w, next(wi), 5, same(x, 9, 5))
        else:
            x = x * 2.0 - 1.0
            w = next(wi)
            x = hsw(bn(conv(x, w, None, 2, same(x, 3, 2)), next(wi), next(wi), next(wi), next(wi)))
            cin = 16
            for bi, (e, f, k, s, se, an) in enumerate(MOBILENET_V3_SMALL_BLOCKS):
                act = acts[an]
                sc = x
                ce = make_divisible(cin * e)
                if bi:
                    x = act(bn(conv(x, next(wi), None, 1, ((0, 0), (0, 0))), next(wi), next(wi), next(wi), next(wi)))
                pads = correct_pad((x.shape[2], x.shape[3]), k) if s == 2 else same(x, k, 1)
                x = act(bn(conv(x, next(wi), None, s, pads, groups=ce), next(wi), next(wi), next(wi), next(wi)))
                if se:
                    g = x.mean(dim=(2, 3), keepdim=True)
                    w1, b1, w2, b2 = next(wi), next(wi), next(wi), next(wi)
                    g = F.relu(conv(g, w1, b1, 1, ((0, 0), (0, 0))))
                    x = x * hsig(conv(g, w2, b2, 1, ((0, 0), (0, 0))))
                x = bn(conv(x, next(wi), None, 1, ((0, 0), (0, 0))), next(wi), next(wi), next(wi), next(wi))
                if s == 1 and cin == f:
                    x = sc + x
                cin = f
            x = hsw(bn(conv(x, next(wi), None, 1, ((0, 0), (0, 0))), next(wi), next(wi), next(wi), next(wi)))
        g = x.mean(dim=(2, 3))
        w1, b1, w2, b2 = next(wi), next(wi), next(wi), next(wi)
        y = (g @ t(w1[0, 0]) + t(b1)) @ t(w2[0, 0]) + t(b2)
    return y.numpy()


# ----------------------------------------------------------------------------- training mode (float64 autograd)

BN_MOMENTUM = 0.999   # keras mobilenet_v3 BatchNormalization(momentum=0.999)


def predictor_train_reference(style, weights: Sequence[np.ndarray], extractor: str, d_style_params):
    """One training-mode forward + backward of the predictor in float64 (torch autograd).

    Keras training=True: every BatchNormalization normalises with the batch's biased moments over
    (B, H, W) and updates moving_mean / moving_variance with momentum 0.999 and the Bessel-corrected
    batch variance. The backward is the gradient of sum(style_params * d_style_params).
    Returns {'output', 'grads' (Keras order, zeros for moving statistics), 'weights' (moving
    statistics updated)}."""
    import torch
    import torch.nn.functional as F

    ws = [torch.tensor(np.asarray(w, np.float64), requires_grad=True) for w in weights]
    new_w = [np.asarray(w, np.float64).copy() for w in weights]
    moving = set()
    idx = [0]

    def nxt():
        i = idx[0]
        idx[0] += 1
        return i

    def conv(x, w, b, stride, pads, groups=1):
        (pt, pb), (pl, pr) = pads
        x = F.pad(x, (pl, pr, pt, pb))
        wt = (w.permute(3, 2, 0, 1) if groups == 1 else w.permute(2, 3, 0, 1)).contiguous()
        return F.conv2d(x, wt, b, stride=stride, groups=groups)

    def same(x, k, s):
        _, pt, pb = _same(x.shape[2], k, s)
        _, pl, pr = _same(x.shape[3], k, s)
        return (pt, pb), (pl, pr)

    def bn(x):
        gi, bi, mi, vi = nxt(), nxt(), nxt(), nxt()
        moving.update((mi, vi))
        mean = x.mean(dim=(0, 2, 3))
        var = ((x - mean.view(1, -1, 1, 1)) ** 2).mean(dim=(0, 2, 3))
        n = x.shape[0] * x.shape[2] * x.shape[3]
        new_w[mi] = new_w[mi] * BN_MOMENTUM + mean.detach().numpy() * (1 - BN_MOMENTUM)
        new_w[vi] = new_w[vi] * BN_MOMENTUM + var.detach().numpy() * n / max(n - 1, 1) * (1 - BN_MOMENTUM)
        inv = torch.rsqrt(var + BN_EPS)
        return (x - mean.view(1, -1, 1, 1)) * (inv * ws[gi]).view(1, -1, 1, 1) + ws[bi].view(1, -1, 1, 1)

    def hsig(x):
        return F.relu6(x + 3.0) * (1.0 / 6.0)

    def hsw(x):
        return x * hsig(x)

    acts = {'relu': F.relu, 'hard_swish': hsw}
    x = torch.tensor(np.asarray(style, np.float64)).permute(0, 3, 1, 2)
    if extractor == 'DUMMY':
        w, b = ws[nxt()], ws[nxt()]
        x = conv(x, w, b, 5, same(x, 9, 5))
    else:
        x = x * 2.0 - 1.0
        w = ws[nxt()]
        x = hsw(bn(conv(x, w, None, 2, same(x, 3, 2))))
        cin = 16
        for bi, (e, f, k, s, se, an) in enumerate(MOBILENET_V3_SMALL_BLOCKS):
            act = acts[an]
            sc = x
            ce = make_divisible(cin * e)
            if bi:
                w = ws[nxt()]
                x = act(bn(conv(x, w, None, 1, ((0, 0), (0, 0)))))
            pads = correct_pad((x.shape[2], x.shape[3]), k) if s == 2 else same(x, k, 1)
            w = ws[nxt()]
            x = act(bn(conv(x, w, None, s, pads, groups=ce)))
            if se:
                g = x.mean(dim=(2, 3), keepdim=True)
                w1, b1, w2, b2 = ws[nxt()], ws[nxt()], ws[nxt()], ws[nxt()]
                g = F.relu(conv(g, w1, b1, 1, ((0, 0), (0, 0))))
                x = x * hsig(conv(g, w2, b2, 1, ((0, 0), (0, 0))))
            w = ws[nxt()]
            x = bn(conv(x, w, None, 1, ((0, 0), (0, 0))))
            if s == 1 and cin == f:
                x = sc + x
            cin = f
        w = ws[nxt()]
        x = hsw(bn(conv(x, w, None, 1, ((0, 0), (0, 0)))))
    g = x.mean(dim=(2, 3))
    w1, b1, w2, b2 = ws[nxt()], ws[nxt()], ws[nxt()], ws[nxt()]
    y = (g @ w1[0, 0] + b1) @ w2[0, 0] + b2
    assert idx[0] == len(ws)
    (y * torch.tensor(np.asarray(d_style_params, np.float64))).sum().backward()
    grads = []
    for i, w in enumerate(ws):
        if i in moving or w.grad is None:
            grads.append(np.zeros(w.shape))
        else:
            grads.append(w.grad.numpy().copy())
    return {'output': y.detach().numpy(), 'grads': grads, 'weights': new_w}
