"""Float64 numpy evaluator for the ONNX operators realtime_style_transfer_amd.onnx_export emits.

Test infrastructure: executes a graph decoded by ``onnx_export.read_model`` so the exported files can
be compared with the float64 oracle. Operator semantics follow the ONNX operator specification (opset
17): NCHW Conv / ConvTranspose with explicit pads [begin_h, begin_w, end_h, end_w], BatchNormalization
in inference mode, ReduceMean with the ``axes`` attribute, Slice with tensor inputs, Reshape with 0 =
copy the input dimension, HardSigmoid max(0, min(1, alpha x + beta)), HardSwish x HardSigmoid(1/6, 1/2),
ReduceSum with axes as an input, Concat, AveragePool (no pads, floor mode).
"""
import numpy as np


def _conv(x, w, b, strides, pads, group):
    N, C, H, W = x.shape
    O, Cg, kh, kw = w.shape
    s = strides[0]
    xp = np.pad(x, ((0, 0), (0, 0), (pads[0], pads[2]), (pads[1], pads[3])))
    Ho = (H + pads[0] + pads[2] - kh) // s + 1
    Wo = (W + pads[1] + pads[3] - kw) // s + 1
    out = np.zeros((N, O, Ho, Wo))
    og = O // group
    for gi in range(group):
        xs = xp[:, gi * Cg:(gi + 1) * Cg]
        ws = w[gi * og:(gi + 1) * og]
        for ky in range(kh):
            for kx in range(kw):
                patch = xs[:, :, ky:ky + s * (Ho - 1) + 1:s, kx:kx + s * (Wo - 1) + 1:s]
                out[:, gi * og:(gi + 1) * og] += np.einsum('nchw,oc->nohw', patch, ws[:, :, ky, kx])
    if b is not None:
        out += b.reshape(1, -1, 1, 1)
    return out


def _conv_transpose(x, w, b, strides, pads):
    N, C, H, W = x.shape
    _, O, kh, kw = w.shape
    s = strides[0]
    full = np.zeros((N, O, (H - 1) * s + kh, (W - 1) * s + kw))
    for ky in range(kh):
        for kx in range(kw):
            full[:, :, ky:ky + s * (H - 1) + 1:s, kx:kx + s * (W - 1) + 1:s] += np.einsum('nchw,co->nohw', x,
                                                                                          w[:, :, ky, kx])
    out = full[:, :, pads[0]:full.shape[2] - pads[2], pads[1]:full.shape[3] - pads[3]]
    if b is not None:
        out = out + b.reshape(1, -1, 1, 1)
    return out


def _hard_sigmoid(x, alpha, beta):
    return np.clip(alpha * x + beta, 0.0, 1.0)


def run(model, feeds):
    """Evaluate ``model`` (read_model output) on ``feeds`` {name: array}; returns {output name: array}."""
    g = model['graph']
    env = {k: np.asarray(v, np.float64) if v.dtype != np.int64 else v for k, v in g['initializers'].items()}
    env.update({k: np.asarray(v, np.float64) for k, v in feeds.items()})
    for op, ins, outs, at in g['nodes']:
        a = [env[i] for i in ins]
        if op == 'Transpose':
            y = np.transpose(a[0], at['perm'])
        elif op == 'Conv':
            y = _conv(a[0], a[1], a[2] if len(a) > 2 else None, at['strides'], at['pads'], at.get('group', 1))
        elif op == 'ConvTranspose':
            y = _conv_transpose(a[0], a[1], a[2] if len(a) > 2 else None, at['strides'], at['pads'])
        elif op == 'Relu':
            y = np.maximum(a[0], 0.0)
        elif op == 'Sigmoid':
            y = 1.0 / (1.0 + np.exp(-a[0]))
        elif op == 'HardSigmoid':
            y = _hard_sigmoid(a[0], at['alpha'], at['beta'])
        elif op == 'HardSwish':
            y = a[0] * _hard_sigmoid(a[0], 1.0 / 6.0, 0.5)
        elif op == 'BatchNormalization':
            x, gam, bet, mu, var = a
            sh = (1, -1, 1, 1)
            y = (x - mu.reshape(sh)) / np.sqrt(var.reshape(sh) + at['epsilon']) * gam.reshape(sh) + bet.reshape(sh)
        elif op == 'ReduceMean':
            y = a[0].mean(axis=tuple(at['axes']), keepdims=bool(at.get('keepdims', 1)))
        elif op == 'Add':
            y = a[0] + a[1]
        elif op == 'Sub':
            y = a[0] - a[1]
        elif op == 'Mul':
            y = a[0] * a[1]
        elif op == 'Neg':
            y = -a[0]
        elif op == 'Sqrt':
            y = np.sqrt(a[0])
        elif op == 'Reciprocal':
            y = 1.0 / a[0]
        elif op == 'Slice':
            x, st, en, ax = a[0], a[1], a[2], a[3]
            sl = [slice(None)] * x.ndim
            for s_, e_, ax_ in zip(st, en, ax):
                sl[int(ax_)] = slice(int(s_), int(e_))
            y = x[tuple(sl)]
        elif op == 'Reshape':
            shape = [int(d) if int(d) != 0 else a[0].shape[i] for i, d in enumerate(a[1])]
            y = a[0].reshape(shape)
        elif op == 'Identity':
            y = a[0]
        elif op == 'ReduceSum':                       # opset 13+: axes as the second input
            y = a[0].sum(axis=tuple(int(v) for v in a[1]), keepdims=bool(at.get('keepdims', 1)))
        elif op == 'Concat':
            y = np.concatenate(a, axis=at['axis'])
        elif op == 'AveragePool':                     # no pads, floor mode: Keras AvgPool2D(2) 'valid'
            kh, kw = at['kernel_shape']
            sh, sw = at['strides']
            N, C, H, W = a[0].shape
            Ho, Wo = (H - kh) // sh + 1, (W - kw) // sw + 1
            y = np.zeros((N, C, Ho, Wo))
            for ky in range(kh):
                for kx in range(kw):
                    y += a[0][:, :, ky:ky + sh * (Ho - 1) + 1:sh, kx:kx + sw * (Wo - 1) + 1:sw]
            y /= kh * kw
        else:
            raise NotImplementedError(op)
        env[outs[0]] = y
    return {name: env[name] for name, _ in g['outputs']}
