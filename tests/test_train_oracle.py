"""CPU tests of the training-step oracle (oracle/torch_train.py, float64 autograd).

* its inference-mode forward reproduces the numpy oracle (and so the golden fixtures' semantics);
* its loss equals oracle/numpy_ref.style_loss_terms;
* its gradients agree with central finite differences of the batch-summed loss, for weights of
  every layer kind (9x9 contract + BN gamma/beta, stride-2 contract, residual, expand, last),
  and for the style parameters;
* its RMSprop / moving-statistics update follows the Keras formulas.
"""
import numpy as np
import pytest
import torch

from oracle import numpy_ref as R
from oracle import torch_train as T
from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
from realtime_style_transfer_amd.styleLoss import init_vgg16_weights

CFG = dict(input_shape=(16, 32, 3), output_shape=(16, 32, 3), bottleneck_res_y=4, bottleneck_num_filters=4)


def _case(B=2, seed=5):
    plan = network_plan(CFG['input_shape'], CFG['output_shape'], CFG['bottleneck_res_y'],
                        CFG['bottleneck_num_filters'])
    w = init_weights(plan, seed=2)
    vgg = init_vgg16_weights(seed=3)
    rng = np.random.default_rng(seed)
    content = rng.random((B,) + CFG['input_shape']).astype(np.float32)
    sp = synthetic_style_params(B, 1, plan.num_style_params, plan, seed=1)
    gtc = rng.random((B,) + CFG['output_shape']).astype(np.float32)
    gts = rng.random((B, 1) + CFG['output_shape']).astype(np.float32)
    return plan, w, vgg, content, sp, gtc, gts


def test_inference_mode_forward_matches_numpy_oracle():
    plan, w, vgg, content, sp, gtc, gts = _case()
    blocks, P = R.transfer_structure(**CFG)
    wt = [torch.tensor(np.asarray(a, np.float64)) for a in w]
    y, _ = T.transfer_forward_train(T._nchw(content), torch.tensor(sp[:, 0], dtype=torch.float64), wt, blocks,
                                    bn_mode="inference")
    ref = R.transfer_forward(content, sp, w, **CFG)
    assert np.abs(y.permute(0, 2, 3, 1).numpy() - ref).max() < 1e-12


def test_loss_matches_numpy_oracle():
    plan, w, vgg, content, sp, gtc, gts = _case()
    out = T.training_step(w, vgg, content, sp, gtc, gts, **CFG)
    from realtime_style_transfer_amd.styleLoss import vgg_weight_dict
    ref = R.style_loss_terms(out['prediction'], gtc, gts, vgg_weight_dict(vgg))
    for i, k in enumerate(('loss', 'feature_loss', 'style_loss', 'total_variation_loss')):
        np.testing.assert_allclose(out['losses'][:, i], ref[k], rtol=1e-9)


def test_gradients_match_finite_differences():
    plan, w, vgg, content, sp, gtc, gts = _case()
    out = T.training_step(w, vgg, content, sp, gtc, gts, **CFG)
    w64 = [np.asarray(a, np.float64) for a in w]
    rng = np.random.default_rng(0)
    # one weight array per layer kind: contract_start kernel, its gamma, beta; contract_0 kernel;
    # residual kernels/bias; expand kernel; last kernel/bias
    names = [(i, s) for i, s in enumerate(plan.weight_shapes())]
    picks = [0, 1, 2, 3, 6, 12, 13, len(names) - 4, len(names) - 2, len(names) - 1]
    for wi in picks:
        g = out['grads'][wi]
        for _ in range(2):
            idx = tuple(int(rng.integers(0, n)) for n in g.shape)
            h = 1e-6 * max(1.0, abs(w64[wi][idx]))
            wp = [a.copy() for a in w64]
            wm = [a.copy() for a in w64]
            wp[wi][idx] += h
            wm[wi][idx] -= h
            fd = (T.loss_of(wp, vgg, content, sp, gtc, gts, **CFG) - T.loss_of(wm, vgg, content, sp, gtc, gts, **CFG)) \
                / (2 * h)
            scale = max(np.abs(g).max(), 1e-12)   # 1e-3 absolute: FD round-off (loss ~1e5, h 1e-6)
            assert abs(fd - g[idx]) < 1e-4 * scale + 1e-3, (wi, idx, fd, g[idx], scale)
    # style parameters
    gs = out['grad_style_params']
    sp64 = sp.astype(np.float64)
    for _ in range(4):
        b, j = int(rng.integers(0, gs.shape[0])), int(rng.integers(0, gs.shape[1]))
        h = 1e-6
        spp, spm = sp64.copy(), sp64.copy()
        spp[b, 0, j] += h
        spm[b, 0, j] -= h
        fd = (T.loss_of(w64, vgg, content, spp, gtc, gts, **CFG) - T.loss_of(w64, vgg, content, spm, gtc, gts, **CFG)) \
            / (2 * h)
        assert abs(fd - gs[b, j]) < 1e-4 * np.abs(gs).max() + 1e-3, (b, j, fd, gs[b, j])


def test_rmsprop_and_moving_statistics_update():
    plan, w, vgg, content, sp, gtc, gts = _case()
    out = T.training_step(w, vgg, content, sp, gtc, gts, **CFG)
    g = out['grads'][0].astype(np.float64)
    ms = 0.1 * g * g
    np.testing.assert_allclose(out['ms'][0], ms, rtol=1e-12)
    np.testing.assert_allclose(out['weights'][0], w[0] - 1e-3 * g / (np.sqrt(ms) + 1e-7), rtol=1e-12)
    # BN moving mean/var of contract_start: only the momentum update, gradient exactly zero
    assert not out['grads'][4].any() and not out['grads'][5].any()
    assert not np.allclose(out['weights'][4], w[4])
    # first RMSprop step moves every trained weight with a nonzero gradient by ~lr/sqrt(0.1)
    step = np.abs(out['weights'][0] - w[0])[np.abs(g) > 1e-6]
    np.testing.assert_allclose(step, 1e-3 / np.sqrt(0.1), rtol=1e-3)
