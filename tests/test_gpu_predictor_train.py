"""GPU parity of the style predictor's training step (rst_predictor_trainer_*) against the float64
autograd oracle (oracle/predictor_ref.predictor_train_reference, itself checked against central
finite differences in tests/test_predictor_oracle.py).

train_network.py fits the predictor (stylePrediction.py:25-75, Keras training=True: BatchNormalization
on batch statistics, moving statistics with momentum 0.999) jointly with the transfer network.
Tolerances (f32 vs f64): output 1e-4 of its max; every weight gradient 2e-3 in L2 relative to the
oracle's (BatchNorm backward over small batches amplifies f32 rounding); moving statistics 1e-5;
RMSprop update exact to f32 rounding.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("ext,ins,B", [("MOBILE_NET", (64, 96, 3), 2), ("MOBILE_NET", (65, 97, 3), 3),
                                       ("DUMMY", (60, 90, 3), 2)])
def test_predictor_training_step_matches_oracle(ext, ins, B):
    _need_gpu()
    import json
    from oracle import predictor_ref as PR
    from realtime_style_transfer_amd.stylePrediction import (StylePredictionTrainer, init_predictor_weights,
                                                             predictor_weight_spec)
    P = 48
    spec = predictor_weight_spec(ins, ext, P)
    ws = init_predictor_weights(spec, seed=3, perturb=True)
    rng = np.random.default_rng(11)
    x = rng.random((B,) + ins).astype(np.float32)
    dP = rng.normal(size=(B, P)).astype(np.float32)
    ref = PR.predictor_train_reference(x, ws, ext, dP)
    tr = StylePredictionTrainer(ins, ext, P, weights=ws, max_batch=4)
    xs = torch.from_numpy(x).cuda()
    y = tr.forward(xs)
    g = tr.backward(torch.from_numpy(dP).cuda())
    torch.cuda.synchronize()
    y = y.cpu().numpy()
    out_err = float(np.abs(y - ref['output']).max() / np.abs(ref['output']).max())
    grads = tr.unflatten(g)
    report, fails = [], []
    gscale = max(float(np.linalg.norm(r)) for r in ref['grads'])
    for (name, shape, kind), a, r in zip(spec, grads, ref['grads']):
        nr = float(np.linalg.norm(r))
        if kind in ('mean', 'var'):
            if np.abs(a).max() != 0.0:
                fails.append((name, 'nonzero gradient for a moving statistic'))
            continue
        if nr <= 1e-9 * gscale:
            # mathematically zero: a shift of this BN's output only reaches the loss through a later
            # BatchNorm on batch statistics, which removes it (both sides are round-off)
            report.append((name + '(zero)', float(np.linalg.norm(a)) / gscale))
            if not np.linalg.norm(a) <= 1e-5 * gscale:
                fails.append((name, 'zero gradient', float(np.linalg.norm(a)), gscale))
            continue
        e = float(np.linalg.norm(a - r) / nr)
        report.append((name, e))
        if not e <= 2e-3:
            fails.append((name, e))
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f'predictor_train_parity_{ext}_{ins[0]}x{ins[1]}.json'), 'w') as f:
        json.dump({'output_rel': out_err, 'grad_rel': report, 'failures': fails}, f, indent=1)
    assert out_err < 1e-4, out_err
    assert not fails, fails
    # moving statistics were updated by the training-mode forward
    w_after = tr.get_weights()
    for (name, shape, kind), a, r in zip(spec, w_after, ref['weights']):
        if kind in ('mean', 'var'):
            np.testing.assert_allclose(a, r, rtol=1e-5, atol=1e-6, err_msg=name)
    # RMSprop (Keras defaults) on the device weights
    tr.apply_gradients(g)
    w_new = tr.get_weights()
    slots = tr.optimizer_slots()
    for (name, shape, kind), a0, a1, gg, ms in zip(spec, w_after, w_new, grads, slots):
        m = 0.1 * gg.astype(np.float64) ** 2
        np.testing.assert_allclose(ms, m, rtol=1e-5, atol=1e-30, err_msg=name)
        np.testing.assert_allclose(a1, a0 - 1e-3 * gg / (np.sqrt(m) + 1e-7), rtol=1e-5, atol=1e-7, err_msg=name)
    # deterministic: a second identical step from the same weights gives bitwise-identical gradients
    tr2 = StylePredictionTrainer(ins, ext, P, weights=ws, max_batch=4)
    tr2.forward(xs)
    g2 = tr2.backward(torch.from_numpy(dP).cuda())
    assert torch.equal(g, g2)
