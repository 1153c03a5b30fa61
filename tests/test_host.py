"""CPU tests of the host side: ShapeConfig mirror, block plan, weight layout, and the C ABI
(library loads and exports every symbol include/rst.h declares; host-only entry points)."""
import ctypes
import os
import re

import numpy as np
import pytest

from realtime_style_transfer_amd.plan import network_plan, init_weights, synthetic_style_params
from realtime_style_transfer_amd.shape_config import ShapeConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shape_config_from_spec_matches_reference_arithmetic():
    """shape_config.py:33-48: rst-960-120-128-17 -> divider 2 -> 480 x 960 x 17 in, 480 x 960 x 3 out."""
    c = ShapeConfig.from_spec("rst-960-120-128-17")
    assert c.input_shape['content'] == (480, 960, 17)
    assert c.input_shape['style'] == (1, 480, 960, 3)
    assert c.output_shape == (480, 960, 3)
    assert c.bottleneck_res_y == 120 and c.bottleneck_num_filters == 128 and c.num_channels == 17
    assert [n for n, _ in c.channels] == ["FinalImage", "BaseColor", "AmbientOcclusion", "Metallic", "Specular",
                                         "Roughness", "ViewNormal", "SceneDepth", "LightingModel"]
    assert ShapeConfig(num_channels=18).num_channels == 18
    assert ShapeConfig(num_channels=6).num_channels == 6
    assert ShapeConfig(num_channels=3).num_channels == 3
    two = ShapeConfig(num_styles=2)
    assert two.input_shape['style_weights'] == (480, 960, 1)
    sdr = ShapeConfig(hdr=False)
    assert sdr.input_shape['content'] == (480, 960, 3)
    assert ShapeConfig.explicit((256, 256), (256, 256), num_channels=3).input_shape['content'] == (256, 256, 3)


def test_plan_matches_reference_structure():
    p = network_plan((480, 960, 17), (480, 960, 3), 120, 128)
    assert p.num_contract_blocks == 2 and p.num_expand_blocks == 2
    assert p.num_style_params == 2662
    assert [l.name for l in p.layers][:3] == ['contract_start', 'contract_0', 'contract_1']
    assert p.layers[-1].name == 'expand_last' and p.layers[-1].post_act == 'sigmoid'
    conv_w = sum(int(np.prod(l.weight_shapes[0])) + l.cout for l in p.layers)
    assert conv_w == 1464019
    assert p.num_weights() == 1464019 + 320                            # + BN (4 x 80)
    # reference test geometries (styleTransferInferenceModelTest.py:16-43, TrainingModelTest.py:15-20)
    up = network_plan((480, 960, 3), (1920, 3840, 3), 120, 128, num_styles=2)
    assert up.num_expand_blocks == 4 and up.layers[-1].out_hw == (1920, 3840)
    tr = network_plan((240, 480, 3), (480, 960, 3), 30, 4)
    assert tr.num_contract_blocks == 3 and tr.num_expand_blocks == 4 and tr.layers[-1].out_hw == (480, 960)


def test_init_weights_follow_reference_initialisers():
    p = network_plan((32, 64, 17), (32, 64, 3), 8, 8)
    ws = init_weights(p, seed=2, perturb_bn=False)
    assert [tuple(w.shape) for w in ws] == [tuple(s) for s in p.weight_shapes()]
    res = [w for l, w in zip([l for l in p.layers for _ in l.weight_shapes], ws) if l.block.startswith('residual')]
    assert all((w >= 0).all() and (w <= 0.05).all() for w in res[0::2])   # U(0, 0.05) kernels
    sp = synthetic_style_params(2, 1, p.num_style_params, p)
    assert sp.shape == (2, 1, 262) and sp.dtype == np.float32


def _lib():
    from realtime_style_transfer_amd import build
    build.build()
    from realtime_style_transfer_amd import _lib as L
    return L, L.load()


def test_library_exports_every_header_symbol():
    L, lib = _lib()
    header = open(os.path.join(ROOT, 'include', 'rst.h')).read()
    declared = set(re.findall(r'\b(rst_[a-z0-9_]+)\s*\(', header))
    assert declared, "no symbols parsed from rst.h"
    assert declared == set(L.EXPORTED_SYMBOLS), declared ^ set(L.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), f"librst.so does not export {name}"
    assert b"gfx950" in lib.rst_version()


def test_abi_host_only_entry_points():
    """rst_num_weights_for_shape runs the C++ plan derivation without touching the device."""
    L, lib = _lib()
    for ins, outs, br, bf in [((480, 960, 17), (480, 960, 3), 120, 128), ((24, 48, 3), (48, 96, 3), 3, 4),
                              ((256, 256, 3), (256, 256, 3), 120, 128)]:
        shape = L.RstShape(ins[0], ins[1], ins[2], outs[0], outs[1], br, bf, 1, 1)
        assert lib.rst_num_weights_for_shape(ctypes.byref(shape)) == network_plan(ins, outs, br, bf).num_weights()
    bad = L.RstShape(480, 960, 17, 480, 960, 0, 128, 1, 1)
    assert lib.rst_num_weights_for_shape(ctypes.byref(bad)) == 0
    assert lib.rst_gram_workspace_size(2, 1000, 64) > 0
    assert lib.rst_instance_norm_workspace_size(2, 1000, 64) > 0


def test_create_rejects_bad_arguments_without_device_work():
    L, lib = _lib()
    h = ctypes.c_void_p()
    shape = L.RstShape(32, 64, 17, 32, 64, 8, 8, 1, 1)
    w = np.zeros(10, np.float32)
    rc = lib.rst_create(ctypes.byref(shape), w.ctypes.data, w.size, ctypes.byref(h))
    assert rc == L.RST_ERR_INVALID and b"expected" in lib.rst_last_error()
    shape3 = L.RstShape(32, 64, 17, 32, 64, 8, 8, 3, 1)   # the reference blends only two styles
    rc = lib.rst_create(ctypes.byref(shape3), w.ctypes.data, w.size, ctypes.byref(h))
    assert rc == L.RST_ERR_UNSUPPORTED


def _cin_fixed_split(v: float):
    """Python restatement of kernels.h cin_fixed_split (same IEEE double operations)."""
    import math
    a = abs(v)
    h = math.floor(a * 2.0 ** -32)
    r = a - h * 2.0 ** 32
    m = math.floor(r * 2.0 ** 8)
    r2 = r - m * 2.0 ** -8
    k = (int(math.floor(r2 * 2.0 ** 48)), int(m), int(h))
    return tuple(-x for x in k) if v < 0 else k


def _cin_fixed_value(l0: int, l1: int, l2: int) -> float:
    """kernels.h cin_fixed_value."""
    def carry(a0, a1, a2):
        c = a0 >> 40
        a0 -= c << 40
        a1 += c
        c = a1 >> 40
        a1 -= c << 40
        return a0, a1, a2 + c
    m0, m1, m2 = carry(l0, l1, l2)
    neg = m2 < 0
    if neg:
        m0, m1, m2 = carry(-l0, -l1, -l2)
    v = float(m2) * 2.0 ** 32 + (float(m1) * 2.0 ** -8 + float(m0) * 2.0 ** -48)
    return -v if neg else v


def test_cin_fixed_point_accumulation_is_order_independent():
    """The inference CIN statistics are added as 64-bit integer limbs (kernels.h cin_fixed_split / cin_fixed_value):
    integer adds commute exactly, so any arrival order of the atomics gives the same bits; the merged value is the
    exact sum of the addends truncated at 2^-48 (per addend), i.e. at least as accurate as f64 atomics."""
    from fractions import Fraction
    rng = np.random.default_rng(0)
    for scale in (1e-9, 1.0, 3e4, 1e12, 3e18):
        vals = (rng.standard_normal(300) * scale).tolist() + [0.0, -0.0, scale, -scale]
        limbs = [_cin_fixed_split(v) for v in vals]
        for v, (l0, l1, l2) in zip(vals, limbs):
            assert 0 <= abs(l0) < 2 ** 40 and 0 <= abs(l1) < 2 ** 40 and abs(l2) < 2 ** 52
            exact = Fraction(l2) * 2 ** 32 + Fraction(l1) / 2 ** 8 + Fraction(l0) / 2 ** 48
            assert abs(Fraction(v) - exact) < Fraction(1, 2 ** 48)            # truncation only below 2^-48
        sums = set()
        for _ in range(5):
            order = rng.permutation(len(vals))
            s = [0, 0, 0]
            for i in order:
                for q in range(3):
                    s[q] += limbs[i][q]
            sums.add(_cin_fixed_value(*s))
        assert len(sums) == 1                                                  # bitwise independent of order
        got = sums.pop()
        exact = sum(Fraction(v) for v in vals)
        assert abs(Fraction(got) - exact) <= len(vals) * Fraction(1, 2 ** 48) + abs(exact) * Fraction(1, 2 ** 52)


def test_mixed_precision_policy_selects_the_loss_network_arithmetic():
    """tf.keras.mixed_precision.set_global_policy (train_network.py:26) -> the VGG16 loss network's precision:
    float32 by default (the reference's run), bf16 under 'mixed_bfloat16' (BASELINE config 4)."""
    from realtime_style_transfer_amd import mixed_precision as mp
    try:
        assert mp.global_policy().name == "float32" and mp.loss_network_precision() == "fp32"
        mp.set_global_policy("mixed_bfloat16")
        pol = mp.global_policy()
        assert (pol.name, pol.compute_dtype, pol.variable_dtype) == ("mixed_bfloat16", "bfloat16", "float32")
        assert mp.loss_network_precision() == "bf16"
        mp.set_global_policy(mp.Policy("float32"))
        assert mp.loss_network_precision() == "fp32"
        with pytest.raises(NotImplementedError):
            mp.set_global_policy("mixed_float16")
        with pytest.raises(ValueError):
            mp.set_global_policy("float64")
        assert mp.global_policy().name == "float32"   # a refused policy leaves the global one unchanged
    finally:
        mp.set_global_policy("float32")
