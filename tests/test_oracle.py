"""CPU tests of the oracle: golden fixtures, the reference's known-answer test, and TF-semantics pins.

The oracle (oracle/numpy_ref.py, float64) is the checker for the GPU path. It is pinned by:
* the reference's only numeric KAT, models/styleTransferTest.py:28-49 (_apply_style_weights);
* the committed golden fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py);
* agreement with an independent torch-CPU restatement (oracle/torch_ref.py);
* property tests that pin TF semantics the reference relies on (SAME padding asymmetry,
  Conv2DTranspose == adjoint of the SAME forward conv, biased moments, Gram definition).
Conv/CIN/BN numerics are otherwise "parity unpinned" against TF itself (TF is not installed).
"""
import os

import numpy as np
import pytest

from oracle import numpy_ref as R

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def _fixture(name):
    d = np.load(os.path.join(GOLDEN, name))
    ws = [d[k] for k in sorted(k for k in d.files if k.startswith('w') and k[1:].isdigit())]
    shape = d['shape']
    return d, ws, tuple(shape[0:3]), tuple(shape[3:6]), int(shape[6]), int(shape[7])


def test_apply_style_weights_known_answer():
    """models/styleTransferTest.py:28-49 re-run against the oracle's _apply_style_weights."""
    d = np.load(os.path.join(GOLDEN, 'apply_style_weights_kat.npz'))
    out = R.apply_style_weights(d['style_weights'], d['style_params'])
    assert out.shape == (2, 10, 20, 6)
    np.testing.assert_almost_equal(out, d['expected'])


def test_apply_style_weights_passthrough_for_other_style_counts():
    """styleTransfer.py:38-44: only S == 2 blends; S == 1 returns the params unchanged."""
    sp = np.arange(12, dtype=np.float32).reshape(1, 1, 1, 12)
    assert np.array_equal(R.apply_style_weights(None, sp), sp)


@pytest.mark.parametrize("name", ["transfer_small.npz", "transfer_up.npz"])
def test_oracle_reproduces_golden(name):
    d, ws, ins, outs, bres, bf = _fixture(name)
    y = R.transfer_forward(d['content'], d['style_params'], ws, ins, outs, bres, bf)
    np.testing.assert_allclose(y, d['output'], rtol=0, atol=1e-12)
    stats = np.array([y.mean(), y.var(), y.min(), y.max()])   # metrics.get_stats format
    np.testing.assert_allclose(stats, d['stats'], atol=1e-12)
    assert ((y > 0) & (y < 1)).all()                            # sigmoid output range


@pytest.mark.parametrize("name", ["transfer_small.npz", "transfer_up.npz"])
def test_torch_restatement_agrees(name):
    from oracle.torch_ref import TorchTransfer
    d, ws, ins, outs, bres, bf = _fixture(name)
    y = TorchTransfer(ws, ins, outs, bres, bf)(d['content'], d['style_params'])
    assert np.abs(y - d['output']).max() < 5e-6


def test_same_padding_stride2_is_asymmetric():
    """TF SAME, k=3, s=2 on an even size pads 0 before / 1 after (not torch's symmetric 1/1)."""
    x = np.arange(1, 9, dtype=np.float64).reshape(1, 1, 8, 1)        # row of 8 pixels
    w = np.ones((1, 3, 1, 1))
    y = R.conv2d_same(x, w, np.zeros(1), 2)[0, 0, :, 0]
    # windows start at 0,2,4,6: [1+2+3, 3+4+5, 5+6+7, 7+8+0]
    assert np.array_equal(y, [6, 12, 18, 15])
    y1 = R.conv2d_same(x, np.ones((1, 9, 1, 1)), np.zeros(1), 1)[0, 0, :, 0]   # 9-wide s1: pad 4/4
    assert y1[0] == 1 + 2 + 3 + 4 + 5 and y1[-1] == 4 + 5 + 6 + 7 + 8


@pytest.mark.parametrize("k,s,hw", [(3, 2, (5, 6)), (9, 1, (7, 5)), (3, 2, (4, 4))])
def test_conv_transpose_is_adjoint_of_same_conv(k, s, hw):
    """Conv2DTranspose(padding='same') is the gradient of Conv2D(padding='same') w.r.t. its
    input: <convT(x), y> == <x, conv(y)> with the kernel's in/out roles swapped."""
    rng = np.random.default_rng(k * 10 + s)
    cin, cout = 3, 4
    x = rng.standard_normal((1, hw[0], hw[1], cin))
    wT = rng.standard_normal((k, k, cout, cin))                        # (kh, kw, out, in)
    y = rng.standard_normal((1, hw[0] * s, hw[1] * s, cout))
    lhs = np.sum(R.conv2d_transpose_same(x, wT, np.zeros(cout), s) * y)
    w_fwd = np.transpose(wT, (0, 1, 2, 3))                             # forward conv: in=cout -> out=cin
    rhs = np.sum(x * R.conv2d_same(y, w_fwd, np.zeros(cin), s))
    assert abs(lhs - rhs) < 1e-9 * max(1.0, abs(lhs))


def test_instance_norm_uses_biased_moments():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((2, 4, 5, 3)) * 3 + 7
    y = R.conditional_instance_norm(x, np.ones((2, 1, 1, 3)), np.zeros((2, 1, 1, 3)))
    assert np.allclose(y.mean(axis=(1, 2)), 0, atol=1e-12)
    v = y.var(axis=(1, 2))                                             # numpy var is biased
    assert np.allclose(v, x.var(axis=(1, 2)) / (x.var(axis=(1, 2)) + 1e-5), atol=1e-12)


def test_gram_and_loss_terms_golden():
    d = np.load(os.path.join(GOLDEN, 'gram_loss.npz'))
    for c in (64, 128):
        f = d[f'f{c}']
        g = R.gram_matrix(f)
        np.testing.assert_allclose(g, d[f'gram_f{c}'], atol=1e-12)
        # definition: G = F^T F / (H W), symmetric PSD
        B, H, W, C = f.shape
        ref = np.einsum('bhwc,bhwd->bcd', f.astype(np.float64), f.astype(np.float64)) / (H * W)
        np.testing.assert_allclose(g, ref, atol=1e-12)
        assert np.allclose(g, np.transpose(g, (0, 2, 1)))
    np.testing.assert_allclose(R.total_variation(d['img']), d['tv'], atol=1e-9)
    img = d['img'].astype(np.float64)
    tv = np.abs(np.diff(img, axis=1)).sum(axis=(1, 2, 3)) + np.abs(np.diff(img, axis=2)).sum(axis=(1, 2, 3))
    np.testing.assert_allclose(d['tv'], tv, atol=1e-9)
    np.testing.assert_allclose(R.mean_l2_loss_on_batch(d['img'] - 0.5), d['l2'], atol=1e-12)


def test_two_style_golden_and_limits():
    """num_styles=2 (styleTransfer.py:36-44, 288-303, 335-345): the oracle reproduces its fixture, and a
    weight map of all 0 (all 1) gives the single-style network with style 0's (style 1's) parameters."""
    d = np.load(os.path.join(GOLDEN, 'transfer_two_styles.npz'))
    ws = [d[k] for k in sorted(k for k in d.files if k.startswith('w') and k[1:].isdigit())]
    shape = d['shape']
    ins, outs, bres, bf = tuple(shape[0:3]), tuple(shape[3:6]), int(shape[6]), int(shape[7])
    y = R.transfer_forward(d['content'], d['style_params'], ws, ins, outs, bres, bf, style_weights=d['style_weights'])
    np.testing.assert_allclose(y, d['output'], rtol=0, atol=1e-12)
    sp = d['style_params']
    for val, s in ((0.0, 0), (1.0, 1)):
        sw = np.full_like(d['style_weights'], val)
        y2 = R.transfer_forward(d['content'], sp, ws, ins, outs, bres, bf, style_weights=sw)
        y1 = R.transfer_forward(d['content'], sp[:, s:s + 1], ws, ins, outs, bres, bf)
        np.testing.assert_allclose(y2, y1, rtol=0, atol=1e-12)
