"""CPU oracle (numpy, float64) for the realtime style-transfer hot path.

TEST INFRASTRUCTURE ONLY. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker.
The product path (``realtime_style_transfer_amd``) never imports it.

This is a restatement of the reference's TensorFlow/Keras graph with the TF
semantics written out explicitly:

* ``create_style_transfer_model``      realtime_style_transfer/models/styleTransfer.py:213-332
* ``contract`` (Conv2D relu -> BN -> ReLU)                    styleTransfer.py:188-205
* ``residual_block`` (conv relu -> CIN -> relu -> conv relu -> CIN [+ x])   :144-185
* ``expand`` (Conv2DTranspose -> CIN -> act)                  styleTransfer.py:95-141
* ``ConditionalInstanceNormalization.call``                   styleTransfer.py:57-71
* ``StyleParamStack`` sequential slicing                      styleTransfer.py:12-33
* ``_apply_style_weights``                                    styleTransfer.py:36-44
* ``gram_matrix``                                             models/styleLoss.py:21-37
* ``mean_l2_loss_on_batch``                                   models/styleLoss.py:290-292
* ``make_style_loss_function`` (feature/style/TV terms)       models/styleLoss.py:295-369
* ``tf.image.total_variation`` (sum |dy| + sum |dx| per image)

Parity status: the reference's only numeric known-answer test is
``models/styleTransferTest.py:28-49`` (``_apply_style_weights``); this oracle reproduces it
(tests/test_oracle.py). TensorFlow is not installed in this container, so conv / CIN /
BN / Gram numerics are **parity unpinned** against TF itself: they follow the documented
TF semantics below and are cross-checked by an independent torch-CPU restatement
(oracle/torch_ref.py) and by committed golden fixtures (tests/golden/).

TF semantics restated:
* SAME padding: ``out = ceil(in/s)``, ``pad_total = max((out-1)*s + k - in, 0)``,
  ``pad_before = pad_total // 2`` (asymmetric for stride 2: top/left 0, bottom/right 1).
* Conv2D kernel (kh, kw, in, out); Conv2DTranspose kernel (kh, kw, out, in); output of a
  SAME transposed conv is ``in*s`` and equals the adjoint of the SAME forward conv.
* ``tf.nn.moments`` -> biased variance; CIN: ``x*rsqrt(var+eps) + (-mean*rsqrt)``, then
  ``bias + x*scale`` with ``eps=1e-5``.
* Keras BatchNormalization (inference): ``gamma*(x-mm)/sqrt(mv+1e-3) + beta``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import numpy as np

_CONTRACT = [(16, 3, 2), (32, 3, 2), (32, 3, 2), (32, 3, 2)]
_EXPAND = [(32, 3, 2), (16, 3, 2), (8, 3, 2), (4, 3, 2), (3, 3, 2), (3, 3, 2), (3, 3, 2), (3, 3, 2)]


def _same_pads(n_in: int, k: int, s: int) -> Tuple[int, int, int]:
    n_out = -(-n_in // s)
    total = max((n_out - 1) * s + k - n_in, 0)
    return n_out, total // 2, total - total // 2


def conv2d_same(x: np.ndarray, w: np.ndarray, b: np.ndarray, stride: int) -> np.ndarray:
    """tf.keras.layers.Conv2D(padding='same') forward. x (B,H,W,Cin), w (kh,kw,Cin,Cout)."""
    x = np.asarray(x, np.float64)
    w = np.asarray(w, np.float64)
    B, H, W, _ = x.shape
    kh, kw, _, cout = w.shape
    Ho, pt, pb = _same_pads(H, kh, stride)
    Wo, pl, pr = _same_pads(W, kw, stride)
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    out = np.zeros((B, Ho, Wo, cout), np.float64)
    for ky in range(kh):
        for kx in range(kw):
            patch = xp[:, ky:ky + stride * (Ho - 1) + 1:stride, kx:kx + stride * (Wo - 1) + 1:stride, :]
            out += patch @ w[ky, kx]
    return out + np.asarray(b, np.float64)


def conv2d_transpose_same(x: np.ndarray, w: np.ndarray, b: np.ndarray, stride: int) -> np.ndarray:
    """tf.keras.layers.Conv2DTranspose(padding='same'). x (B,H,W,Cin), w (kh,kw,Cout,Cin).

    Adjoint of the SAME forward conv on an ``in*s`` sized map:
    ``full[i*s + k] += x[i] w[k]``, then crop ``[pad_before : pad_before + in*s]``
    with ``pad_before = max(k - s, 0) // 2``.
    """
    x = np.asarray(x, np.float64)
    w = np.asarray(w, np.float64)
    B, H, W, _ = x.shape
    kh, kw, cout, _ = w.shape
    Ho, Wo = H * stride, W * stride
    pt = max(kh - stride, 0) // 2
    pl = max(kw - stride, 0) // 2
    full = np.zeros((B, (H - 1) * stride + kh, (W - 1) * stride + kw, cout), np.float64)
    for ky in range(kh):
        for kx in range(kw):
            full[:, ky:ky + stride * (H - 1) + 1:stride, kx:kx + stride * (W - 1) + 1:stride, :] += x @ w[ky, kx].T
    return full[:, pt:pt + Ho, pl:pl + Wo, :] + np.asarray(b, np.float64)


def batch_norm_inference(x, gamma, beta, mean, var, eps=1e-3):
    inv = np.asarray(gamma, np.float64) / np.sqrt(np.asarray(var, np.float64) + eps)
    return x * inv + (np.asarray(beta, np.float64) - np.asarray(mean, np.float64) * inv)


def apply_style_weights(style_weights, style_params):
    """styleTransfer.py:36-44: per-pixel blend only when S == 2; else params unchanged."""
    style_params = np.asarray(style_params, np.float64)
    if style_params.shape[-2] == 2:
        sp = np.expand_dims(style_params, 1)                  # (B,1,1,2,F)
        sw = np.expand_dims(np.asarray(style_weights, np.float64), -1)  # (B,H,W,2,1)
        return np.sum(sp * sw, axis=-2)
    return style_params


def conditional_instance_norm(x, scale, bias, eps=1e-5):
    """styleTransfer.py:57-71. x (B,H,W,F); scale/bias broadcastable (B,1,1,F) or (B,H,W,F)."""
    mean = x.mean(axis=(1, 2), keepdims=True)
    var = ((x - mean) ** 2).mean(axis=(1, 2), keepdims=True)
    inv = 1.0 / np.sqrt(var + eps)
    x = x * inv + (-mean * inv)
    return bias + x * scale


def relu(x):
    return np.maximum(x, 0.0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def avg_pool2(x):
    """tf.keras.layers.AvgPool2D(2) (valid padding) on NHWC."""
    B, H, W, C = x.shape
    H2, W2 = H // 2, W // 2
    x = x[:, :H2 * 2, :W2 * 2, :]
    return x.reshape(B, H2, 2, W2, 2, C).mean(axis=(2, 4))


class _ParamStack:
    """StyleParamStack (styleTransfer.py:12-33)."""

    def __init__(self, params):
        self.params = params
        self.lower = 0

    def get(self, n):
        lo = self.lower
        self.lower += n
        return self.params[..., lo:lo + n]


def transfer_structure(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters):
    """Block list of create_style_transfer_model (styleTransfer.py:213-276)."""
    H = input_shape[0]
    n_c = math.ceil(math.log2(H) - math.log2(bottleneck_res_y))
    blocks = [('contract', 9, 1, 32)]
    blocks += [('contract', _CONTRACT[i][1], _CONTRACT[i][2], _CONTRACT[i][0]) for i in range(n_c)]
    res_h = int(H * 2 ** -n_c)
    blocks += [('residual_first', 3, 1, bottleneck_num_filters)]
    blocks += [('residual', 3, 1, bottleneck_num_filters)] * 4
    n_e = math.ceil(math.log2(output_shape[0]) - math.log2(res_h))
    blocks += [('expand', _EXPAND[i][1], _EXPAND[i][2], _EXPAND[i][0]) for i in range(n_e)]
    blocks += [('expand_last', 9, 1, 3)]
    P = 5 * 2 * 2 * bottleneck_num_filters + sum(2 * _EXPAND[i][0] for i in range(n_e)) + 6
    return blocks, P


def transfer_forward(content, style_params, weights: Sequence[np.ndarray], input_shape, output_shape,
                     bottleneck_res_y, bottleneck_num_filters, style_weights=None, return_intermediates=False,
                     operand_round=None):
    """Forward of the transfer net in float64.

    content (B,H,W,C); style_params (B,S,P); weights in Keras get_weights() order;
    style_weights (B,Ho,Wo,S-1) for S>1 (styleTransfer.py:290-303). ``operand_round`` (e.g. bf16_round)
    is applied to the input and kernel of the residual-block convs (the layers a bf16 precision mode
    runs on the bf16 pipe) to simulate that mode.
    """
    blocks, P = transfer_structure(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters)
    x = np.asarray(content, np.float64)
    sp = np.asarray(style_params, np.float64)
    if sp.shape[-1] != P:
        raise ValueError(f"style_params last dim {sp.shape[-1]} != P={P}")
    S = sp.shape[1]
    mips = None
    if S > 1:
        sw = np.asarray(style_weights, np.float64)
        sw = np.concatenate([1.0 - sw.sum(-1, keepdims=True), sw], -1)        # :297-302
        mips = {sw.shape[-2]: sw}
        last = sw
        n_mips = sum(1 for b in blocks if b[0] == 'expand') + 1
        for _ in range(n_mips):                                                # :335-345
            last = avg_pool2(last)
            mips[last.shape[-2]] = last
    sp = np.expand_dims(sp, 1)                                                 # (B,1,S,P) :305
    stack = _ParamStack(sp)
    wi = iter(weights)
    inter: Dict[str, np.ndarray] = {}
    for bi, (kind, k, s, f) in enumerate(blocks):
        if kind == 'contract':
            w, b = next(wi), next(wi)
            gamma, beta, mm, mv = next(wi), next(wi), next(wi), next(wi)
            x = relu(conv2d_same(x, w, b, s))
            x = relu(batch_norm_inference(x, gamma, beta, mm, mv))
        elif kind.startswith('residual'):
            block_params = _ParamStack(stack.get(4 * f))
            sw = mips[x.shape[-2]] if mips is not None else None
            inp = x
            fx = x
            for j in range(2):
                w, b = next(wi), next(wi)
                if operand_round is not None:
                    fx, w = operand_round(fx), operand_round(w)
                fx = relu(conv2d_same(fx, w, b, 1))
                cin_params = _ParamStack(block_params.get(2 * f))
                scale = apply_style_weights(sw, cin_params.get(f))
                bias = apply_style_weights(sw, cin_params.get(f))
                fx = conditional_instance_norm(fx, scale, bias)
                if j == 0:
                    fx = relu(fx)
            x = fx if kind == 'residual_first' else inp + fx
        else:
            w, b = next(wi), next(wi)
            params = _ParamStack(stack.get(2 * f))
            sw = mips[x.shape[-2] * s] if mips is not None else None
            x = conv2d_transpose_same(x, w, b, s)
            scale = apply_style_weights(sw, params.get(f))
            bias = apply_style_weights(sw, params.get(f))
            x = conditional_instance_norm(x, scale, bias)
            x = sigmoid(x) if kind == 'expand_last' else relu(x)
        if return_intermediates:
            inter[f'{bi}_{kind}'] = x
    return (x, inter) if return_intermediates else x


# ----------------------------------------------------------------------------- loss

def gram_matrix(features):
    """styleLoss.py:21-37: einsum('bijc,bijd->bcd') / (H*W)."""
    f = np.asarray(features, np.float64)
    B, H, W, C = f.shape
    f2 = f.reshape(B, H * W, C)
    return np.einsum('bpc,bpd->bcd', f2, f2) / (H * W)


def mean_l2_loss_on_batch(t):
    """styleLoss.py:290-292: mean(0.5 t^2) over all non-batch axes."""
    t = np.asarray(t, np.float64)
    return np.mean(0.5 * t ** 2, axis=tuple(range(1, t.ndim)))


def total_variation(images):
    """tf.image.total_variation for a 4-D batch: sum |dy| + sum |dx| per image."""
    x = np.asarray(images, np.float64)
    dy = np.abs(x[:, 1:, :, :] - x[:, :-1, :, :]).sum(axis=(1, 2, 3))
    dx = np.abs(x[:, :, 1:, :] - x[:, :, :-1, :]).sum(axis=(1, 2, 3))
    return dy + dx


VGG_MEAN_BGR = np.array([103.939, 116.779, 123.68])
VGG16_LAYERS = [  # keras.applications.VGG16 (include_top=False) trunk
    ('block1_conv1', 64), ('block1_conv2', 64), ('pool',),
    ('block2_conv1', 128), ('block2_conv2', 128), ('pool',),
    ('block3_conv1', 256), ('block3_conv2', 256), ('block3_conv3', 256), ('pool',),
    ('block4_conv1', 512), ('block4_conv2', 512), ('block4_conv3', 512), ('pool',),
    ('block5_conv1', 512), ('block5_conv2', 512), ('block5_conv3', 512),
]
STYLE_LAYERS = ['block1_conv2', 'block2_conv2', 'block3_conv3', 'block4_conv3']   # styleLoss.py:79
CONTENT_LAYERS = ['block5_conv3']                                                  # styleLoss.py:80


def max_pool2(x):
    B, H, W, C = x.shape
    H2, W2 = H // 2, W // 2
    return x[:, :H2 * 2, :W2 * 2, :].reshape(B, H2, 2, W2, 2, C).max(axis=(2, 4))


def bf16_round(x):
    """Round to bfloat16 (round-to-nearest-even) through float32, as the device does with its fp32
    values; returned as float64 (bf16 x bf16 products are exact in fp32 and float64)."""
    u = np.ascontiguousarray(np.asarray(x, np.float32)).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).astype(np.float64)


def vgg16_features(images01, vgg_weights: Dict[str, Tuple[np.ndarray, np.ndarray]], operand_round=None):
    """StyleLossModelVGG.call (styleLoss.py:106-109): x*255, RGB->BGR, -mean, VGG16 trunk.
    ``operand_round`` (bf16_round) is applied to the input and kernel of every conv — the device's plain-bf16
    loss runs all thirteen on bf16 operands (block1_conv1 on vgg_conv0_bf16, the preprocessed image rounded),
    as Keras mixed_bfloat16 does — and to every conv's output: the layer outputs are stored in bf16 (a
    mixed_bfloat16 layer emits its compute dtype), which the content loss and the feature maps see directly
    (the next conv's input rounding is then exact, and a max pool of rounded values is the rounded max)."""
    x = np.asarray(images01, np.float64) * 255.0
    x = x[..., ::-1] - VGG_MEAN_BGR                                   # vgg16.preprocess_input ('caffe')
    feats = {}
    for entry in VGG16_LAYERS:
        if entry[0] == 'pool':
            x = max_pool2(x)
            continue
        name = entry[0]
        w, b = vgg_weights[name]
        if operand_round is not None:
            x, w = operand_round(x), operand_round(w)
        x = relu(conv2d_same(x, w, b, 1))
        if operand_round is not None:
            x = operand_round(x)
        if name in STYLE_LAYERS or name in CONTENT_LAYERS:
            feats[name] = x
        if name == CONTENT_LAYERS[0]:
            break
    return feats


def style_loss_terms(prediction, gt_content, gt_style, vgg_weights,
                     content_factor=1e4, style_factor=1e-3, tv_factor=1e-1, operand_round=None):
    """make_style_loss_function without the MiDaS depth term (styleLoss.py:295-369)."""
    style = np.asarray(gt_style, np.float64)
    if style.ndim == 5:
        assert style.shape[1] == 1
        style = style[:, 0]
    fc = vgg16_features(gt_content, vgg_weights, operand_round)
    fs = vgg16_features(style, vgg_weights, operand_round)
    fp = vgg16_features(prediction, vgg_weights, operand_round)
    feature_loss = np.mean([mean_l2_loss_on_batch(fp[n] - fc[n]) for n in CONTENT_LAYERS], axis=0) * content_factor
    # operand_round (the device's plain-bf16 loss) also rounds the Gram operands: its Gram runs on bf16 features
    # (gram.hip gram_partial_bf16_kernel, the mixed_bfloat16 einsum)
    gram = (lambda f: gram_matrix(operand_round(f))) if operand_round is not None else gram_matrix
    style_loss = np.mean([mean_l2_loss_on_batch(gram(fp[n]) - gram(fs[n])) for n in STYLE_LAYERS],
                         axis=0) * style_factor
    tv = total_variation(prediction) * tv_factor
    return {'loss': feature_loss + style_loss + tv, 'feature_loss': feature_loss, 'style_loss': style_loss,
            'total_variation_loss': tv}
