"""CPU tests of the style-predictor oracle and host plan (stylePrediction.py:25-75).

The predictor's numerics are not pinned by the reference's tests (they only run the DUMMY
extractor on zeros for output shapes) and Keras is not installed, so the oracle is pinned by:
* the published size of keras.applications.MobileNetV3Small(include_top=False): 939,120 weights,
  and its 7x7x576 feature map at 224x224 (structure of the restatement);
* TF semantics of correct_pad + 'valid' == SAME for the stride-2 depthwise convs;
* agreement of two independent restatements (numpy float64 loops vs torch float32 grouped convs);
* the committed golden fixtures (tests/golden/predictor_*.npz) — parity unpinned against Keras itself.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import predictor_ref as PR
from realtime_style_transfer_amd.stylePrediction import (StyleFeatureExtractor, create_style_prediction_model,
                                                         init_predictor_weights, predictor_weight_spec)

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def _digest(ws):
    import hashlib
    h = hashlib.sha256()
    for w in ws:
        h.update(np.ascontiguousarray(w, np.float32).tobytes())
    return h.hexdigest()


def _golden(name):
    d = np.load(os.path.join(GOLDEN, name))
    shape = d['shape']
    ins, P, seed = tuple(int(v) for v in shape[:3]), int(shape[3]), int(shape[4])
    ext = str(d['extractor'])
    ws = init_predictor_weights(predictor_weight_spec(ins, ext, P), seed=seed, perturb=True)
    assert _digest(ws) == str(d['weights_sha256']), "seeded predictor weights no longer regenerate bit-identically"
    return d, ws, ins, P, ext


def test_mobilenet_v3_small_matches_published_size():
    spec = predictor_weight_spec((224, 224, 3), StyleFeatureExtractor.MOBILE_NET, 10)
    trunk = [s for n, s, _ in spec if not n.startswith('Style')]
    assert sum(int(np.prod(s)) for s in trunk) == 939120
    ws = init_predictor_weights(spec, seed=0)
    _, feat = PR.style_predictor_forward(np.zeros((1, 224, 224, 3)), ws, 'MOBILE_NET', return_features=True)
    assert feat.shape == (1, 7, 7, 576)


@pytest.mark.parametrize("n", [7, 8, 15, 16, 240, 241])
@pytest.mark.parametrize("k", [3, 5])
def test_correct_pad_valid_equals_tf_same(n, k):
    (pt, pb), _ = PR.correct_pad((n, n), k)
    out_valid = (n + pt + pb - k) // 2 + 1
    out_same, st, _ = PR._same(n, k, 2)
    assert out_valid == out_same and pt == st


@pytest.mark.parametrize("name", ["predictor_mobilenet.npz", "predictor_dummy.npz"])
def test_oracle_reproduces_golden(name):
    d, ws, ins, P, ext = _golden(name)
    y, feat = PR.style_predictor_forward(d['style'], ws, ext, return_features=True)
    np.testing.assert_allclose(y, d['output'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(feat, d['features'], rtol=0, atol=1e-12)
    assert y.shape == (d['style'].shape[0], P)


@pytest.mark.parametrize("name", ["predictor_mobilenet.npz", "predictor_dummy.npz"])
def test_torch_restatement_agrees(name):
    d, ws, ins, P, ext = _golden(name)
    y = PR.torch_style_predictor_forward(d['style'], ws, ext)
    assert np.abs(y - d['output']).max() <= 1e-5 * np.abs(d['output']).max()


def test_host_spec_matches_oracle_and_library():
    from realtime_style_transfer_amd import _lib
    lib = _lib.load()
    for ext in ('DUMMY', 'MOBILE_NET'):
        for ins in ((480, 960, 3), (33, 47, 3)):
            spec = predictor_weight_spec(ins, ext, 2662)
            assert [s for _, s, _ in spec] == [tuple(s) for s in PR.predictor_weight_shapes(ins, ext, 2662)]
            sh = _lib.RstPredictorShape(ins[0], ins[1], ins[2], _lib.EXTRACTORS[ext], 2662, 100, 1)
            assert lib.rst_predictor_num_weights(ctypes.byref(sh)) == sum(int(np.prod(s)) for _, s, _ in spec)
    bad = _lib.RstPredictorShape(480, 960, 3, 2, 2662, 100, 1)       # EFFICIENT_NET is not built
    assert lib.rst_predictor_num_weights(ctypes.byref(bad)) == 0


def test_factory_errors_mirror_reference():
    with pytest.raises(ValueError):                  # stylePrediction.py:44-46
        create_style_prediction_model((64, 64, 3), 'RESNET', 10)
    with pytest.raises(NotImplementedError):
        create_style_prediction_model((64, 64, 3), StyleFeatureExtractor.EFFICIENT_NET, 10)


@pytest.mark.parametrize("ext", ["MOBILE_NET", "DUMMY"])
def test_training_oracle_matches_finite_differences(ext):
    """predictor_train_reference (float64 autograd, BN on batch statistics) vs central differences."""
    ins, P = (32, 48, 3), 24
    spec = predictor_weight_spec(ins, ext, P)
    ws = [w.astype(np.float64) for w in init_predictor_weights(spec, seed=3, perturb=True)]
    rng = np.random.default_rng(0)
    x = rng.random((2,) + ins)
    dP = rng.normal(size=(2, P))
    ref = PR.predictor_train_reference(x, ws, ext, dP)

    def loss(wl):
        return float((PR.predictor_train_reference(x, wl, ext, dP)['output'] * dP).sum())

    checked = 0
    for i, (name, shape, kind) in enumerate(spec):
        if kind in ('mean', 'var') or (ext == 'MOBILE_NET' and i % 7 != 0):
            continue
        j = int(rng.integers(ws[i].size))
        wp = [w.copy() for w in ws]
        wm = [w.copy() for w in ws]
        wp[i].flat[j] += 1e-6
        wm[i].flat[j] -= 1e-6
        fd = (loss(wp) - loss(wm)) / 2e-6
        assert abs(fd - ref['grads'][i].flat[j]) <= 1e-5 * max(1.0, abs(fd)), (name, fd, ref['grads'][i].flat[j])
        checked += 1
    assert checked >= 4
    for (name, shape, kind), g in zip(spec, ref['grads']):
        if kind in ('mean', 'var'):
            assert not g.any()
