"""ONNX export of the transfer network and the style predictor (f2: weights interop).

The reference exports both Keras models with tf2onnx (``save_using_checkpoint.py:90-103``):
the predictor as ``<out>.predictor.onnx`` with one input named ``style``, the transfer net as
``<out>.transfer.onnx`` with the inputs named after the Keras input dict, ``content`` and
``style_params`` (``styleTransfer.py:281-284``) — the names the Unreal plugin binds. tf2onnx and
onnx are not installed here, so this module writes the ModelProto itself with a small protobuf
encoder (onnx.proto field numbers, IR version 8, default-domain opset 17) and reads it back with a
matching decoder (``read_model``).

Graph layout: the inputs and the output stay NHWC like the Keras models; a Transpose moves to NCHW
for the ONNX Conv / ConvTranspose operators and back at the end (what tf2onnx emits for Keras
convs). Everything else restates the reference layers op by op:
  * contract: Conv (explicit SAME pads) + bias -> Relu -> BatchNormalization(eps 1e-3) -> Relu
    (``styleTransfer.py:188-205``);
  * CIN (``:57-71``): ReduceMean over H, W, the biased variance, ``x * rsqrt(var+eps) +
    (-mean * rsqrt(var+eps))`` then ``bias + x * scale``, with scale/bias Sliced out of
    ``style_params`` at the StyleParamStack offsets (``:12-33``);
  * residual blocks (``:144-185``), block 0 without the skip Add;
  * expand: ConvTranspose (pads = the SAME crop: begin (k-s)//2, end the rest) + CIN + Relu, the last
    one + Sigmoid (``:95-141,269-276``);
  * predictor: Rescaling(2, -1) as Mul/Add, MobileNetV3Small (Conv, depthwise Conv with group = C,
    BatchNormalization, Relu / HardSwish, squeeze-excite with HardSigmoid(1/6, 1/2)), the global
    average pool and the two 1x1 heads (``stylePrediction.py:25-75``).
Two styles (``num_styles == 2``) add the ``style_weights`` input (N, Ho, Wo, 1): the full weight map
``[1 - sum(w), w]`` (``styleTransfer.py:290-303``), its AvgPool2 mip chain keyed by width (``:335-345``,
``num_expand_blocks + 1`` levels, valid pooling) and, in every CIN, the per-pixel blend of the two styles'
scale and bias with the mip of the layer's output width (``_apply_style_weights``, ``:36-44``). For more
than two styles the reference returns the unblended (B, 1, S, F) parameters, which do not broadcast against
a (B, H, W, F) feature map; that graph is not exported.

Parity: the exported graph is checked by executing it with the repo's own reader and a numpy
evaluator of these operators (tests/onnx_runner.py) against the float64 oracle; loading it in
onnxruntime / TensorRT / the Unreal NNE plugin is *parity unpinned* (none is installed here).
"""
from __future__ import annotations

import struct
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .plan import BN_EPS, CIN_EPS, Plan

IR_VERSION = 8
OPSET = 17
FLOAT, INT64 = 1, 7                       # TensorProto.DataType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_FLOATS, A_INTS = 1, 2, 3, 4, 6, 7   # AttributeProto.AttributeType


# ----------------------------------------------------------------------------------------------------
# protobuf wire format
# ----------------------------------------------------------------------------------------------------
def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _f_varint(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(int(v))


def _f_bytes(field: int, b: bytes) -> bytes:
    return _key(field, 2) + _varint(len(b)) + b


def _f_str(field: int, s: str) -> bytes:
    return _f_bytes(field, s.encode())


def _f_float(field: int, v: float) -> bytes:
    return _key(field, 5) + struct.pack('<f', float(v))


def _parse(buf: bytes) -> List[Tuple[int, int, object]]:
    """Decode one message level into [(field, wire type, value)] (value: int or bytes)."""
    out, i, n = [], 0, len(buf)
    while i < n:
        key, i = _read_varint(buf, i)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            v, i = buf[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            v, i = bytes(buf[i:i + ln]), i + ln
        elif wt == 5:
            v, i = buf[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.append((field, wt, v))
    return out


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def _signed(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


# ----------------------------------------------------------------------------------------------------
# ONNX messages
# ----------------------------------------------------------------------------------------------------
def _tensor(name: str, arr: np.ndarray) -> bytes:
    arr = np.ascontiguousarray(arr)
    if arr.dtype == np.float32:
        dt = FLOAT
    elif arr.dtype == np.int64:
        dt = INT64
    else:
        raise TypeError(f"initializer {name}: unsupported dtype {arr.dtype}")
    b = b''.join(_f_varint(1, d) for d in arr.shape)
    b += _f_varint(2, dt) + _f_str(8, name) + _f_bytes(9, arr.astype(arr.dtype.newbyteorder('<')).tobytes())
    return b


def _value_info(name: str, shape: Sequence[Optional[int]]) -> bytes:
    dims = b''
    for d in shape:
        dims += _f_bytes(1, _f_varint(1, d) if isinstance(d, int) else _f_str(2, str(d)))
    tensor_type = _f_varint(1, FLOAT) + _f_bytes(2, dims)
    return _f_str(1, name) + _f_bytes(2, _f_bytes(1, tensor_type))


def _attribute(name: str, v) -> bytes:
    b = _f_str(1, name)
    if isinstance(v, float):
        return b + _f_float(2, v) + _f_varint(20, A_FLOAT)
    if isinstance(v, (int, np.integer)):
        return b + _f_varint(3, int(v)) + _f_varint(20, A_INT)
    if isinstance(v, str):
        return b + _f_bytes(4, v.encode()) + _f_varint(20, A_STRING)
    if isinstance(v, (list, tuple)) and all(isinstance(x, (int, np.integer)) for x in v):
        return b + b''.join(_f_varint(8, int(x)) for x in v) + _f_varint(20, A_INTS)
    if isinstance(v, (list, tuple)):
        return b + b''.join(_f_float(7, float(x)) for x in v) + _f_varint(20, A_FLOATS)
    raise TypeError(f"attribute {name}: {type(v)}")


class GraphBuilder:
    """Accumulates nodes and initializers; names are unique per graph."""

    def __init__(self, name: str):
        self.name = name
        self.nodes: List[bytes] = []
        self.inits: List[bytes] = []
        self.inputs: List[bytes] = []
        self.outputs: List[bytes] = []
        self._n = 0

    def fresh(self, hint: str) -> str:
        self._n += 1
        return f"{hint}_{self._n}"

    def const(self, hint: str, arr: np.ndarray) -> str:
        name = self.fresh(hint)
        self.inits.append(_tensor(name, arr))
        return name

    def op(self, op_type: str, inputs: Sequence[str], hint: Optional[str] = None, **attrs) -> str:
        out = self.fresh(hint or op_type.lower())
        b = b''.join(_f_str(1, i) for i in inputs) + _f_str(2, out) + _f_str(3, out) + _f_str(4, op_type)
        b += b''.join(_f_bytes(5, _attribute(k, v)) for k, v in attrs.items())
        self.nodes.append(b)
        return out

    def rename_output(self, src: str, dst: str):
        """Identity node so the graph output carries the exported name."""
        b = _f_str(1, src) + _f_str(2, dst) + _f_str(3, dst) + _f_str(4, 'Identity')
        self.nodes.append(b)

    def model(self, doc: str) -> bytes:
        g = b''.join(_f_bytes(1, n) for n in self.nodes) + _f_str(2, self.name)
        g += b''.join(_f_bytes(5, t) for t in self.inits)
        g += b''.join(_f_bytes(11, v) for v in self.inputs) + b''.join(_f_bytes(12, v) for v in self.outputs)
        opset = _f_str(1, '') + _f_varint(2, OPSET)
        return (_f_varint(1, IR_VERSION) + _f_str(2, 'realtime_style_transfer_amd') + _f_str(3, '0.2') +
                _f_str(6, doc) + _f_bytes(7, g) + _f_bytes(8, opset))


# ----------------------------------------------------------------------------------------------------
# transfer network
# ----------------------------------------------------------------------------------------------------
def _same_pads(n: int, k: int, s: int) -> Tuple[int, int]:
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


def _f32(a) -> np.ndarray:
    return np.asarray(a, np.float32)


def _conv(g: GraphBuilder, x: str, kern: np.ndarray, bias: Optional[np.ndarray], stride: int,
          pads: Tuple[int, int, int, int], group: int = 1, hint: str = 'conv') -> str:
    """Keras HWIO kernel (or depthwise (kh, kw, C, 1)) -> ONNX Conv (OIHW)."""
    kh, kw = kern.shape[:2]
    w = np.transpose(_f32(kern), (2, 3, 0, 1)) if group > 1 else np.transpose(_f32(kern), (3, 2, 0, 1))
    ins = [x, g.const(hint + '_w', np.ascontiguousarray(w))]
    if bias is not None:
        ins.append(g.const(hint + '_b', _f32(bias)))
    return g.op('Conv', ins, hint, kernel_shape=[kh, kw], strides=[stride, stride], pads=list(pads),
                group=group, dilations=[1, 1])


def _batch_norm(g: GraphBuilder, x: str, gamma, beta, mean, var, eps: float, hint: str) -> str:
    return g.op('BatchNormalization', [x, g.const(hint + '_gamma', _f32(gamma)), g.const(hint + '_beta', _f32(beta)),
                                       g.const(hint + '_mean', _f32(mean)), g.const(hint + '_var', _f32(var))],
                hint, epsilon=float(eps))


def _style_slice(g: GraphBuilder, sp: str, offset: int, c: int, hint: str) -> str:
    """style_params (N, 1, P)[..., offset:offset+c] -> (N, c, 1, 1)."""
    s = g.op('Slice', [sp, g.const(hint + '_st', np.array([offset], np.int64)),
                       g.const(hint + '_en', np.array([offset + c], np.int64)),
                       g.const(hint + '_ax', np.array([2], np.int64))], hint + '_slice')
    return g.op('Reshape', [s, g.const(hint + '_shape', np.array([0, c, 1, 1], np.int64))], hint)


def _style_weight_mips(g: GraphBuilder, out_w: int, levels: int) -> Dict[int, str]:
    """styleTransfer.py:290-303,335-345: NCHW full weights (N, 2, Ho, Wo) and their AvgPool2 mips by width."""
    w = g.op('Transpose', ['style_weights'], 'sw_nchw', perm=[0, 3, 1, 2])
    total = g.op('ReduceSum', [w, g.const('sw_axes', np.array([1], np.int64))], 'sw_sum', keepdims=1)
    w0 = g.op('Sub', [g.const('sw_one', np.array(1.0, np.float32)), total], 'sw_w0')
    last = g.op('Concat', [w0, w], 'sw_full', axis=1)
    mips, width = {out_w: last}, out_w
    for i in range(levels):
        last = g.op('AveragePool', [last], f'sw_mip{i}', kernel_shape=[2, 2], strides=[2, 2])
        width //= 2
        mips[width] = last
    return mips


def _blended_param(g: GraphBuilder, sp: str, offset: int, c: int, mip: str, hint: str) -> str:
    """_apply_style_weights (styleTransfer.py:36-44) for S == 2: sum_s w_s * params_s -> (N, c, h, w)."""
    terms = []
    for si in range(2):
        p = g.op('Slice', [sp, g.const(hint + f'_st{si}', np.array([si, offset], np.int64)),
                           g.const(hint + f'_en{si}', np.array([si + 1, offset + c], np.int64)),
                           g.const(hint + f'_ax{si}', np.array([1, 2], np.int64))], hint + f'_slice{si}')
        p = g.op('Reshape', [p, g.const(hint + f'_shape{si}', np.array([0, c, 1, 1], np.int64))], hint + f'_p{si}')
        wgt = g.op('Slice', [mip, g.const(hint + f'_wst{si}', np.array([si], np.int64)),
                             g.const(hint + f'_wen{si}', np.array([si + 1], np.int64)),
                             g.const(hint + f'_wax{si}', np.array([1], np.int64))], hint + f'_w{si}')
        terms.append(g.op('Mul', [wgt, p], hint + f'_wp{si}'))
    return g.op('Add', terms, hint)


def _cin(g: GraphBuilder, x: str, sp: str, offset: int, c: int, hint: str, mip: Optional[str] = None) -> str:
    """ConditionalInstanceNormalization.call (styleTransfer.py:57-71); with ``mip`` the two styles' parameters
    are blended per pixel."""
    mean = g.op('ReduceMean', [x], hint + '_mean', axes=[2, 3], keepdims=1)
    d = g.op('Sub', [x, mean], hint + '_d')
    var = g.op('ReduceMean', [g.op('Mul', [d, d], hint + '_d2')], hint + '_var', axes=[2, 3], keepdims=1)
    eps = g.const(hint + '_eps', np.array(CIN_EPS, np.float32))
    inv = g.op('Reciprocal', [g.op('Sqrt', [g.op('Add', [var, eps], hint + '_ve')], hint + '_sd')], hint + '_inv')
    xn = g.op('Add', [g.op('Mul', [x, inv], hint + '_xi'), g.op('Mul', [g.op('Neg', [mean], hint + '_nm'), inv],
                                                                   hint + '_mi')], hint + '_xn')
    if mip is None:
        scale = _style_slice(g, sp, offset, c, hint + '_scale')
        bias = _style_slice(g, sp, offset + c, c, hint + '_bias')
    else:
        scale = _blended_param(g, sp, offset, c, mip, hint + '_scale')
        bias = _blended_param(g, sp, offset + c, c, mip, hint + '_bias')
    return g.op('Add', [bias, g.op('Mul', [xn, scale], hint + '_xs')], hint)


def transfer_graph(plan: Plan, weights: Sequence[np.ndarray], batch: Optional[int] = None) -> bytes:
    """ModelProto bytes of create_style_transfer_model (styleTransfer.py:213-332), num_styles 1 or 2."""
    S = plan.num_styles
    if S not in (1, 2):
        raise NotImplementedError("ONNX export covers num_styles 1 and 2 (for S > 2 the reference's CIN parameters "
                                  "stay unblended (B,1,S,F) and do not broadcast, styleTransfer.py:36-44)")
    shapes = plan.weight_shapes()
    if len(weights) != len(shapes) or any(tuple(w.shape) != s for w, s in zip(weights, shapes)):
        raise ValueError("weights do not match the plan's Keras get_weights() shapes")
    N = batch if batch is not None else 'N'
    H, W, C = plan.input_shape
    Ho, Wo, _ = plan.output_shape
    P = plan.num_style_params
    g = GraphBuilder('StyleTransferModel')
    g.inputs += [_value_info('content', [N, H, W, C]), _value_info('style_params', [N, S, P])]
    mips = None
    if S == 2:
        g.inputs.append(_value_info('style_weights', [N, Ho, Wo, S - 1]))
        n_expand = sum(1 for layer in plan.layers if layer.kind != 'conv' and layer.block != 'expand_last')
        mips = _style_weight_mips(g, Wo, n_expand + 1)
    x = g.op('Transpose', ['content'], 'to_nchw', perm=[0, 3, 1, 2])
    wi = iter(weights)
    block_in = None
    for layer in plan.layers:
        kern, bias = next(wi), next(wi)
        hint = layer.name
        if layer.kind == 'conv':
            pt, pb = _same_pads(layer.in_hw[0], layer.k, layer.stride)
            pl, pr = _same_pads(layer.in_hw[1], layer.k, layer.stride)
            if layer.block.startswith('residual') and layer.name.endswith('conv0'):
                block_in = x
            x = g.op('Relu', [_conv(g, x, kern, bias, layer.stride, (pt, pl, pb, pr), hint=hint)], hint + '_relu')
            if layer.norm == 'bn':
                gamma, beta, mm, mv = next(wi), next(wi), next(wi), next(wi)
                x = g.op('Relu', [_batch_norm(g, x, gamma, beta, mm, mv, BN_EPS, hint + '_bn')], hint + '_bnrelu')
            else:
                x = _cin(g, x, 'style_params', layer.style_offset, layer.cout, hint + '_cin',
                         mips[layer.out_hw[1]] if mips is not None else None)
                if layer.post_act == 'relu':
                    x = g.op('Relu', [x], hint + '_post')
                elif not layer.residual_first:   # second conv of blocks 1..4: skip Add (:184)
                    x = g.op('Add', [block_in, x], hint + '_add')
        else:
            crop = max(layer.k - layer.stride, 0)
            pads = [crop // 2, crop // 2, crop - crop // 2, crop - crop // 2]
            w = np.ascontiguousarray(np.transpose(_f32(kern), (3, 2, 0, 1)))   # (kh,kw,out,in) -> (in,out,kh,kw)
            x = g.op('ConvTranspose', [x, g.const(hint + '_w', w), g.const(hint + '_b', _f32(bias))], hint,
                     kernel_shape=[layer.k, layer.k], strides=[layer.stride, layer.stride], pads=pads,
                     dilations=[1, 1], group=1)
            x = _cin(g, x, 'style_params', layer.style_offset, layer.cout, hint + '_cin',
                     mips[layer.out_hw[1]] if mips is not None else None)
            x = g.op('Sigmoid' if layer.post_act == 'sigmoid' else 'Relu', [x], hint + '_post')
    assert next(wi, None) is None
    y = g.op('Transpose', [x], 'to_nhwc', perm=[0, 2, 3, 1])
    g.rename_output(y, 'output')
    g.outputs.append(_value_info('output', [N, Ho, Wo, 3]))
    return g.model("realtime style transfer network (styleTransfer.py:213-332); inputs content (NHWC) and "
                   "style_params (N, num_styles, P)")


# ----------------------------------------------------------------------------------------------------
# style predictor
# ----------------------------------------------------------------------------------------------------
def _make_divisible(v: float, divisor: int = 8) -> int:
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def _correct_pad(hw, k) -> Tuple[int, int, int, int]:
    adjust = (1 - hw[0] % 2, 1 - hw[1] % 2)
    c = k // 2
    return c - adjust[0], c - adjust[1], c, c


def predictor_graph(input_shape, feature_extractor: str, weights: Sequence[np.ndarray], num_top_parameters: int,
                    batch: Optional[int] = None) -> bytes:
    """ModelProto bytes of create_style_prediction_model (stylePrediction.py:25-75)."""
    from .stylePrediction import _MOBILENET_V3_SMALL, StyleFeatureExtractor
    N = batch if batch is not None else 'N'
    H, W, C = (int(v) for v in input_shape)
    g = GraphBuilder('StylePredictionModel')
    g.inputs.append(_value_info('style', [N, H, W, C]))
    x = g.op('Transpose', ['style'], 'to_nchw', perm=[0, 3, 1, 2])
    wi = iter(weights)
    hw = (H, W)

    def same(n, k, s):
        return _same_pads(n, k, s)

    if feature_extractor == StyleFeatureExtractor.DUMMY:
        pt, pb = same(H, 9, 5)
        pl, pr = same(W, 9, 5)
        x = _conv(g, x, next(wi), next(wi), 5, (pt, pl, pb, pr), hint='dummy_conv')
    elif feature_extractor == StyleFeatureExtractor.MOBILE_NET:
        x = g.op('Add', [g.op('Mul', [x, g.const('rescale_a', np.array(2.0, np.float32))], 'rescale_mul'),
                         g.const('rescale_b', np.array(-1.0, np.float32))], 'rescale')
        pt, pb = same(hw[0], 3, 2)
        pl, pr = same(hw[1], 3, 2)
        x = _conv(g, x, next(wi), None, 2, (pt, pl, pb, pr), hint='Conv')
        hw = (-(-hw[0] // 2), -(-hw[1] // 2))
        x = g.op('HardSwish', [_batch_norm(g, x, next(wi), next(wi), next(wi), next(wi), BN_EPS, 'Conv_bn')], 'Conv_act')
        cin = 16
        for bi, (e, f, k, s, se, act) in enumerate(_MOBILENET_V3_SMALL):
            p = f'block{bi}'
            shortcut = x
            ce = _make_divisible(cin * e)

            def activate(t, nm):
                return g.op('Relu' if act == 'relu' else 'HardSwish', [t], nm)

            if bi:
                x = _conv(g, x, next(wi), None, 1, (0, 0, 0, 0), hint=p + '_expand')
                x = activate(_batch_norm(g, x, next(wi), next(wi), next(wi), next(wi), BN_EPS, p + '_expand_bn'),
                             p + '_expand_act')
            if s == 2:
                pads = _correct_pad(hw, k)
                hw = ((hw[0] + pads[0] + pads[2] - k) // 2 + 1, (hw[1] + pads[1] + pads[3] - k) // 2 + 1)
            else:
                pt, pb = same(hw[0], k, 1)
                pl, pr = same(hw[1], k, 1)
                pads = (pt, pl, pb, pr)
            x = _conv(g, x, next(wi), None, s, pads, group=ce, hint=p + '_dw')
            x = activate(_batch_norm(g, x, next(wi), next(wi), next(wi), next(wi), BN_EPS, p + '_dw_bn'), p + '_dw_act')
            if se:
                r = g.op('ReduceMean', [x], p + '_se_pool', axes=[2, 3], keepdims=1)
                r = g.op('Relu', [_conv(g, r, next(wi), next(wi), 1, (0, 0, 0, 0), hint=p + '_se_reduce')], p + '_se_relu')
                r = _conv(g, r, next(wi), next(wi), 1, (0, 0, 0, 0), hint=p + '_se_expand')
                r = g.op('HardSigmoid', [r], p + '_se_gate', alpha=1.0 / 6.0, beta=0.5)
                x = g.op('Mul', [x, r], p + '_se')
            x = _conv(g, x, next(wi), None, 1, (0, 0, 0, 0), hint=p + '_project')
            x = _batch_norm(g, x, next(wi), next(wi), next(wi), next(wi), BN_EPS, p + '_project_bn')
            if s == 1 and cin == f:
                x = g.op('Add', [shortcut, x], p + '_add')
            cin = f
        x = _conv(g, x, next(wi), None, 1, (0, 0, 0, 0), hint='Conv_1')
        x = g.op('HardSwish', [_batch_norm(g, x, next(wi), next(wi), next(wi), next(wi), BN_EPS, 'Conv_1_bn')],
                 'Conv_1_act')
    else:
        raise NotImplementedError(f"ONNX export of feature extractor {feature_extractor}")
    x = g.op('ReduceMean', [x], 'avg_pool', axes=[2, 3], keepdims=1)                       # :54-55
    x = _conv(g, x, next(wi), next(wi), 1, (0, 0, 0, 0), hint='StylePredictor')            # :57-64
    x = _conv(g, x, next(wi), next(wi), 1, (0, 0, 0, 0), hint='StyleNormPredictor')        # :66-71
    assert next(wi, None) is None
    y = g.op('Reshape', [x, g.const('squeeze_shape', np.array([0, num_top_parameters], np.int64))], 'squeeze')  # :72
    g.rename_output(y, 'style_params')
    g.outputs.append(_value_info('style_params', [N, num_top_parameters]))
    return g.model("style predictor (stylePrediction.py:25-75); input style (NHWC in [0, 1])")


def save_onnx(outpath, plan: Plan, transfer_weights: Sequence[np.ndarray], style_input_shape=None,
              feature_extractor: Optional[str] = None, predictor_weights: Optional[Sequence[np.ndarray]] = None,
              batch: Optional[int] = None) -> Dict[str, Path]:
    """Write ``<out>.transfer.onnx`` (and ``<out>.predictor.onnx`` when predictor weights are given) with the
    file naming of save_using_checkpoint.py:73-103."""
    outpath = Path(outpath)
    paths = {'transfer': outpath.with_suffix('.transfer.onnx')}
    paths['transfer'].write_bytes(transfer_graph(plan, transfer_weights, batch))
    if predictor_weights is not None:
        paths['predictor'] = outpath.with_suffix('.predictor.onnx')
        paths['predictor'].write_bytes(predictor_graph(style_input_shape, feature_extractor, predictor_weights,
                                                       plan.num_style_params, batch))
    return paths


# ----------------------------------------------------------------------------------------------------
# reader
# ----------------------------------------------------------------------------------------------------
def _decode_tensor(buf: bytes) -> Tuple[str, np.ndarray]:
    dims, dt, name, raw = [], FLOAT, '', b''
    for f, wt, v in _parse(buf):
        if f == 1:
            if wt == 2:   # packed
                i = 0
                while i < len(v):
                    d, i = _read_varint(v, i)
                    dims.append(_signed(d))
            else:
                dims.append(_signed(v))
        elif f == 2:
            dt = v
        elif f == 8:
            name = v.decode()
        elif f == 9:
            raw = v
    dtype = {FLOAT: '<f4', INT64: '<i8'}[dt]
    return name, np.frombuffer(raw, dtype).reshape(dims).astype(dtype[1:] if dt == FLOAT else np.int64)


def _decode_attribute(buf: bytes):
    name, val, ints, floats, atype = '', None, [], [], 0
    for f, wt, v in _parse(buf):
        if f == 1:
            name = v.decode()
        elif f == 2:
            val = struct.unpack('<f', v)[0]
        elif f == 3:
            val = _signed(v)
        elif f == 4:
            val = v.decode()
        elif f == 7:
            floats.append(struct.unpack('<f', v)[0])
        elif f == 8:
            ints.append(_signed(v))
        elif f == 20:
            atype = v
    if atype == A_INTS:
        val = ints
    elif atype == A_FLOATS:
        val = floats
    return name, val


def _decode_value_info(buf: bytes):
    name, shape = '', []
    for f, _, v in _parse(buf):
        if f == 1:
            name = v.decode()
        elif f == 2:
            for f2, _, tt in _parse(v):
                if f2 != 1:
                    continue
                for f3, _, sh in _parse(tt):
                    if f3 != 2:
                        continue
                    for f4, _, dim in _parse(sh):
                        for f5, _, dv in _parse(dim):
                            shape.append(_signed(dv) if f5 == 1 else dv.decode())
    return name, shape


def read_model(data) -> dict:
    """Decode a ModelProto written by this module (or any ONNX model using the same fields) into
    {ir_version, opset, producer, graph: {name, nodes [(op_type, inputs, outputs, attrs)], initializers
    {name: array}, inputs [(name, shape)], outputs [(name, shape)]}}."""
    if isinstance(data, (str, Path)):
        data = Path(data).read_bytes()
    model = {'ir_version': None, 'opset': {}, 'producer': ''}
    graph_buf = b''
    for f, _, v in _parse(data):
        if f == 1:
            model['ir_version'] = v
        elif f == 2:
            model['producer'] = v.decode()
        elif f == 7:
            graph_buf = v
        elif f == 8:
            dom, ver = '', None
            for f2, _, v2 in _parse(v):
                if f2 == 1:
                    dom = v2.decode()
                elif f2 == 2:
                    ver = v2
            model['opset'][dom] = ver
    graph = {'name': '', 'nodes': [], 'initializers': {}, 'inputs': [], 'outputs': []}
    for f, _, v in _parse(graph_buf):
        if f == 1:
            ins, outs, op, attrs = [], [], '', {}
            for f2, _, v2 in _parse(v):
                if f2 == 1:
                    ins.append(v2.decode())
                elif f2 == 2:
                    outs.append(v2.decode())
                elif f2 == 4:
                    op = v2.decode()
                elif f2 == 5:
                    k, val = _decode_attribute(v2)
                    attrs[k] = val
            graph['nodes'].append((op, ins, outs, attrs))
        elif f == 2:
            graph['name'] = v.decode()
        elif f == 5:
            name, arr = _decode_tensor(v)
            graph['initializers'][name] = arr
        elif f == 11:
            graph['inputs'].append(_decode_value_info(v))
        elif f == 12:
            graph['outputs'].append(_decode_value_info(v))
    model['graph'] = graph
    return model
