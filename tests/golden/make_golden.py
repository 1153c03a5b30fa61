"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

Run: ``python tests/golden/make_golden.py`` (CPU only, a few seconds).

Fixtures (all float32 inputs/weights, float64 expected outputs, npz):
* transfer_small.npz — config (i) of SURVEY §8c: 32x64x17 -> 32x64x3, bottleneck 8 rows,
  8 filters (2 contract + 2 expand blocks), B=2, S=1.
* transfer_up.npz — config (ii): the reference training-test geometry
  (styleTransferTrainingModelTest.py:15-20: 240x480x3 -> 480x960x3, bottleneck 30 rows x 4
  filters) scaled by 1/10: 24x48x3 -> 48x96x3, bottleneck 3 rows, 4 filters
  (3 contract + 4 expand blocks, SDR content), B=2.
* apply_style_weights_kat.npz — the reference's only numeric known-answer test,
  models/styleTransferTest.py:12-49, recomputed from its formula.
* gram_loss.npz — gram matrices / mean_l2 / total_variation of seeded tensors.
* transfer_two_styles.npz — config (i) with num_styles=2: per-pixel blending of the CIN
  parameters with a (B, 32, 64, 1) style-weight map and its AvgPool2 mips
  (styleTransfer.py:36-44, 288-303, 335-345).
* predictor_mobilenet.npz / predictor_dummy.npz — the style predictor
  (stylePrediction.py:25-75) at 64x96x3 (MOBILE_NET, B=2) and 60x90x3 (DUMMY, B=2), P=200, with
  perturbed seeded weights (regenerated from the seed by init_predictor_weights; the fixture
  stores a sha256 of the float32 weight bytes instead of the 1.2 M weights), the per-block
  outputs and the (B, P) output.
Each transfer fixture also stores ``stats`` in the metrics.get_stats format
(realtime_style_transfer/metrics.py:4-12: mean/var/min/max).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import numpy_ref as R  # noqa: E402
from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params  # noqa: E402


def stats(t):
    return np.array([np.mean(t), np.var(t), np.min(t), np.max(t)])


def transfer_fixture(name, ins, outs, bres, bf, batch=2, num_styles=1):
    plan = network_plan(ins, outs, bres, bf, num_styles)
    w = init_weights(plan, seed=2)
    sp = synthetic_style_params(batch, num_styles, plan.num_style_params, plan, seed=1)
    x = np.random.default_rng(0).random((batch,) + tuple(ins)).astype(np.float32)
    sw = None
    if num_styles > 1:
        # smooth left-to-right blend plus noise, in [0, 1]
        ramp = np.linspace(0.0, 1.0, outs[1], dtype=np.float32)[None, None, :, None]
        noise = np.random.default_rng(4).random((batch, outs[0], outs[1], num_styles - 1)).astype(np.float32)
        sw = (0.8 * ramp + 0.2 * noise).astype(np.float32)
    y, inter = R.transfer_forward(x, sp, w, ins, outs, bres, bf, style_weights=sw, return_intermediates=True)
    arrays = {'content': x, 'style_params': sp, 'output': y, 'stats': stats(y),
              'shape': np.array(list(ins) + list(outs) + [bres, bf])}
    if sw is not None:
        arrays['style_weights'] = sw
    for i, wi in enumerate(w):
        arrays[f'w{i:02d}'] = wi
    np.savez_compressed(os.path.join(HERE, name), **arrays)


def vertical_gradient(min_max, shape):
    """_generate_vertical_gradient_tensor (styleTransferTest.py:12-24), including its use of
    shape[0] (the batch) as the divisor."""
    out = []
    for b in range(shape[0]):
        for i in range(shape[1]):
            out.append([min_max[0] + (i / shape[0]) * (min_max[1] - min_max[0]) for _ in range(shape[2])])
    return np.array(out, np.float32).reshape(shape)


def kat_fixture():
    sw = np.stack([vertical_gradient((0, 1), (2, 10, 20)), vertical_gradient((1, 0), (2, 10, 20))], axis=-1)
    sp = np.array([[[[10, 20, 30, 40, 50, 60], [70, 80, 90, 100, 110, 120]]]] * 2, np.float32).reshape(2, 1, 2, 6)
    expected = np.zeros((2, 10, 20, 6))
    for b in range(2):
        for x in range(10):
            for y in range(20):
                for c in range(6):
                    expected[b, x, y, c] = sw[b, x, y, 0] * sp[b, 0, 0, c] + sw[b, x, y, 1] * sp[b, 0, 1, c]
    np.savez_compressed(os.path.join(HERE, 'apply_style_weights_kat.npz'), style_weights=sw, style_params=sp,
                        expected=expected)


def gram_fixture():
    rng = np.random.default_rng(5)
    f = {f'f{c}': rng.random((2, 4, 6, c)).astype(np.float32) for c in (64, 128)}
    arrays = dict(f)
    for k, v in f.items():
        arrays['gram_' + k] = R.gram_matrix(v)
    img = rng.random((2, 12, 16, 3)).astype(np.float32)
    arrays['img'] = img
    arrays['tv'] = R.total_variation(img)
    arrays['l2'] = R.mean_l2_loss_on_batch(img - 0.5)
    np.savez_compressed(os.path.join(HERE, 'gram_loss.npz'), **arrays)


def weights_digest(ws):
    import hashlib
    h = hashlib.sha256()
    for w in ws:
        h.update(np.ascontiguousarray(w, np.float32).tobytes())
    return h.hexdigest()


def predictor_fixture(name, extractor, ins, batch=2, P=200, seed=3):
    from oracle import predictor_ref as PR
    from realtime_style_transfer_amd.stylePrediction import init_predictor_weights, predictor_weight_spec
    spec = predictor_weight_spec(ins, extractor, P)
    ws = init_predictor_weights(spec, seed=seed, perturb=True)
    x = np.random.default_rng(6).random((batch,) + tuple(ins)).astype(np.float32)
    y, feat = PR.style_predictor_forward(x, ws, extractor, return_features=True)
    arrays = {'style': x, 'output': y, 'features': feat, 'shape': np.array(list(ins) + [P, seed]),
              'extractor': np.array(extractor), 'weights_sha256': np.array(weights_digest(ws))}
    if extractor == 'MOBILE_NET':
        _, blocks = PR.mobilenet_v3_small(x * 2.0 - 1.0, iter(ws), return_blocks=True)
        for i, b in enumerate(blocks):
            arrays[f'block{i:02d}'] = b
    np.savez_compressed(os.path.join(HERE, name), **arrays)


if __name__ == '__main__':
    only = sys.argv[1:]
    jobs = {
        'transfer_small.npz': lambda: transfer_fixture('transfer_small.npz', (32, 64, 17), (32, 64, 3), 8, 8),
        'transfer_up.npz': lambda: transfer_fixture('transfer_up.npz', (24, 48, 3), (48, 96, 3), 3, 4),
        'apply_style_weights_kat.npz': kat_fixture,
        'gram_loss.npz': gram_fixture,
        'transfer_two_styles.npz': lambda: transfer_fixture('transfer_two_styles.npz', (32, 64, 17), (32, 64, 3), 8, 8,
                                                            num_styles=2),
        'predictor_mobilenet.npz': lambda: predictor_fixture('predictor_mobilenet.npz', 'MOBILE_NET', (64, 96, 3)),
        'predictor_dummy.npz': lambda: predictor_fixture('predictor_dummy.npz', 'DUMMY', (60, 90, 3)),
    }
    for name, job in jobs.items():
        if not only or name in only:
            job()
    print('golden fixtures written to', HERE)
