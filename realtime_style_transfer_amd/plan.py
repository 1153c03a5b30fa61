"""Block plan of the transfer network, derived exactly as the reference derives it.

``network_plan`` restates the shape arithmetic of ``create_style_transfer_model``
(``realtime_style_transfer/models/styleTransfer.py:213-332``):

* ``num_contract_blocks = ceil(log2(H_in) - log2(bottleneck_res_y))``            (:217)
* contract filter table ``(16,3,2),(32,3,2),(32,3,2),(32,3,2)``                  (:218-223)
* ``contract("start", 32 filters, 9x9, s1)`` then the strided contract blocks     (:224-232)
* five residual blocks, block 0 ``is_first`` (no skip add)                         (:239-245)
* expand filter table ``(32,16,8,4,3,3,3,3)``, all 3x3 s2                          (:247-256)
* ``num_expand_blocks = ceil(log2(H_out) - log2(H_bottleneck))``                   (:258)
* final ``expand("last", 3 filters, 9x9, s1, sigmoid)``                            (:269-276)
* style-parameter count ``P`` = sum of CIN params over residual + expand blocks    (:278-279)

The weight list order is the Keras ``model.get_weights()`` order of that graph
(conv kernel, conv bias[, BN gamma, beta, moving_mean, moving_variance]) so a
checkpoint reader can map 1:1 onto it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

CONTRACT_FILTER_SIZES = [(16, 3, 2), (32, 3, 2), (32, 3, 2), (32, 3, 2)]          # styleTransfer.py:218-223
EXPAND_FILTER_SIZES = [(32, 3, 2), (16, 3, 2), (8, 3, 2), (4, 3, 2),
                       (3, 3, 2), (3, 3, 2), (3, 3, 2), (3, 3, 2)]                # styleTransfer.py:247-256
CIN_EPS = 1e-5     # ConditionalInstanceNormalization default epsilon (styleTransfer.py:51)
BN_EPS = 1e-3      # tf.keras.layers.BatchNormalization default epsilon (styleTransfer.py:201)


@dataclass
class Layer:
    """One conv of the plan (a conv + its normalisation/activation)."""
    name: str
    kind: str              # 'conv' or 'convT'
    k: int
    stride: int
    cin: int
    cout: int
    in_hw: Tuple[int, int]
    out_hw: Tuple[int, int]
    conv_relu: bool        # Conv2D(activation=relu) built into the conv (contract/residual)
    norm: str              # 'bn' (contract) or 'cin' (residual/expand)
    post_act: str          # after the norm: 'relu', 'none' or 'sigmoid'
    style_offset: int = -1  # offset of [scale(F), bias(F)] in the style-param vector (CIN only)
    residual_first: bool = False   # residual block index (for bookkeeping)
    block: str = ''
    weight_shapes: List[Tuple[int, ...]] = field(default_factory=list)


@dataclass
class Plan:
    input_shape: Tuple[int, int, int]
    output_shape: Tuple[int, int, int]
    bottleneck_res_y: int
    bottleneck_num_filters: int
    num_styles: int
    num_contract_blocks: int
    num_expand_blocks: int
    layers: List[Layer]
    num_style_params: int

    def weight_shapes(self) -> List[Tuple[int, ...]]:
        out = []
        for layer in self.layers:
            out.extend(layer.weight_shapes)
        return out

    def num_weights(self) -> int:
        return int(sum(int(np.prod(s)) for s in self.weight_shapes()))


def _same_out(n: int, s: int) -> int:
    return -(-n // s)


def network_plan(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters, num_styles=1) -> Plan:
    H, W, C = (int(v) for v in input_shape)
    Ho, Wo, Co = (int(v) for v in output_shape)
    if Co != 3:
        raise ValueError(f"output must have 3 channels, got {output_shape}")
    n_c = math.ceil(math.log2(H) - math.log2(bottleneck_res_y))                  # :217
    layers: List[Layer] = []

    # contract("start") :224 — Conv2D(32, 9, s1, same, relu) -> BN -> ReLU (:188-205)
    hw = (H, W)
    layers.append(Layer('contract_start', 'conv', 9, 1, C, 32, hw, hw, True, 'bn', 'relu', block='contract_start',
                        weight_shapes=[(9, 9, C, 32), (32,), (32,), (32,), (32,), (32,)]))
    cin = 32
    for i in range(n_c):                                                          # :225-232
        f, k, s = CONTRACT_FILTER_SIZES[i]
        ohw = (_same_out(hw[0], s), _same_out(hw[1], s))
        layers.append(Layer(f'contract_{i}', 'conv', k, s, cin, f, hw, ohw, True, 'bn', 'relu', block=f'contract_{i}',
                            weight_shapes=[(k, k, cin, f), (f,), (f,), (f,), (f,), (f,)]))
        hw, cin = ohw, f
    F = bottleneck_num_filters
    offset = 0
    for r in range(5):                                                            # :239-245, :144-185
        for j in range(2):
            layers.append(Layer(f'residual_block_{r}_conv{j}', 'conv', 3, 1, cin, F, hw, hw, True, 'cin',
                                'relu' if j == 0 else 'none', style_offset=offset, residual_first=(r == 0),
                                block=f'residual_block_{r}', weight_shapes=[(3, 3, cin, F), (F,)]))
            offset += 2 * F
            cin = F
    n_e = math.ceil(math.log2(Ho) - math.log2(hw[0]))                             # :258
    for i in range(n_e):                                                          # :260-267, :95-141
        f, k, s = EXPAND_FILTER_SIZES[i]
        ohw = (hw[0] * s, hw[1] * s)
        # Conv2DTranspose kernel layout is (kh, kw, out, in)
        layers.append(Layer(f'expand_{i}', 'convT', k, s, cin, f, hw, ohw, False, 'cin', 'relu',
                            style_offset=offset, block=f'expand_{i}', weight_shapes=[(k, k, f, cin), (f,)]))
        offset += 2 * f
        hw, cin = ohw, f
    # expand("last", 3, 9, 1, sigmoid) :269-276
    layers.append(Layer('expand_last', 'convT', 9, 1, cin, 3, hw, hw, False, 'cin', 'sigmoid',
                        style_offset=offset, block='expand_last', weight_shapes=[(9, 9, 3, cin), (3,)]))
    offset += 6
    if hw != (Ho, Wo):
        raise ValueError(f"plan ends at {hw}, output_shape asks for {(Ho, Wo)}")
    return Plan((H, W, C), (Ho, Wo, Co), bottleneck_res_y, F, num_styles, n_c, n_e, layers, offset)


def init_weights(plan: Plan, seed: int = 2, perturb_bn: bool = True) -> List[np.ndarray]:
    """Seeded weights mirroring the reference initialisers.

    contract/expand kernels ~ N(0, 0.02) (styleTransfer.py:97,190), residual kernels ~
    U(0, 0.05) (:146), biases zero (Keras default). BN gamma=1/beta=0/mean=0/var=1 are
    the Keras defaults; with ``perturb_bn`` they are moved off identity so parity tests
    exercise the BN path (trained checkpoints have non-trivial statistics).
    Biases are also perturbed slightly (a trained net's are non-zero).
    """
    rng = np.random.default_rng(seed)
    out: List[np.ndarray] = []
    for layer in plan.layers:
        kshape = layer.weight_shapes[0]
        if layer.block.startswith('residual'):
            kern = rng.uniform(0.0, 0.05, size=kshape)
        else:
            kern = rng.normal(0.0, 0.02, size=kshape)
        out.append(kern.astype(np.float32))
        bias = rng.normal(0.0, 0.01, size=kshape[-1] if layer.kind == 'conv' else kshape[2]) if perturb_bn \
            else np.zeros(layer.cout)
        out.append(bias.astype(np.float32))
        if layer.norm == 'bn':
            c = layer.cout
            if perturb_bn:
                gamma = rng.uniform(0.8, 1.2, c)
                beta = rng.normal(0.0, 0.1, c)
                mean = rng.uniform(0.0, 0.2, c)
                var = rng.uniform(0.5, 1.5, c)
            else:
                gamma, beta, mean, var = np.ones(c), np.zeros(c), np.zeros(c), np.ones(c)
            out.extend(a.astype(np.float32) for a in (gamma, beta, mean, var))
    shapes = plan.weight_shapes()
    assert [tuple(w.shape) for w in out] == [tuple(s) for s in shapes]
    return out


def synthetic_style_params(batch: int, num_styles: int, P: int, plan: Optional[Plan] = None, seed: int = 1) -> np.ndarray:
    """Style params (B,S,P): CIN scales ~ U[0.5,1.5), biases ~ N(0, 0.1)."""
    rng = np.random.default_rng(seed)
    sp = np.empty((batch, num_styles, P), dtype=np.float64)
    sp[...] = rng.normal(0.0, 0.1, size=sp.shape)
    if plan is not None:
        for layer in plan.layers:
            if layer.norm == 'cin':
                o, F = layer.style_offset, layer.cout
                sp[..., o:o + F] = rng.uniform(0.5, 1.5, size=(batch, num_styles, F))
    return sp.astype(np.float32)
