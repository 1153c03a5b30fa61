"""GPU parity of the style predictor and the inference model (librst on MI355X) against the oracle.

create_style_prediction_model (stylePrediction.py:25-75) and make_style_transfer_inference_model
(styleTransferInferenceModel.py:9-48). The HIP path computes in f32 (fmaf chains); the oracle is
float64 (numpy) or float32 (torch-CPU, full size). Tolerance: 1e-4 of the output's max magnitude
(f32 rounding through 13 stages is ~1e-6 relative); the transferred image keeps the 2e-4 absolute
bar of test_gpu_transfer.py.
"""
import os

import numpy as np
import pytest
import torch

from test_predictor_oracle import _golden

pytestmark = pytest.mark.gpu

REL = 1e-4


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("name", ["predictor_mobilenet.npz", "predictor_dummy.npz"])
def test_predictor_matches_golden(name):
    _need_gpu()
    from realtime_style_transfer_amd.stylePrediction import create_style_prediction_model
    d, ws, ins, P, ext = _golden(name)
    model = create_style_prediction_model(ins, ext, P, weights=ws, max_batch=2)
    y = model(torch.from_numpy(d['style']).cuda()).cpu().numpy()
    assert y.shape == d['output'].shape
    assert _rel(y, d['output']) < REL, _rel(y, d['output'])
    n = model.num_stages()
    feat = model.stage_output(n - 1, 2).cpu().numpy()
    assert _rel(feat, d['features']) < REL
    if ext == 'MOBILE_NET':
        for i in range(11):
            blk = model.stage_output(1 + i, 2).cpu().numpy()
            assert _rel(blk, d[f'block{i:02d}']) < REL, (i, _rel(blk, d[f'block{i:02d}']))


@pytest.mark.parametrize("ins", [(33, 47, 3), (97, 130, 3)])
def test_predictor_odd_sizes(ins):
    """Odd spatial sizes: correct_pad's adjust term and partial pixel tiles."""
    _need_gpu()
    from oracle import predictor_ref as PR
    from realtime_style_transfer_amd.stylePrediction import (create_style_prediction_model, init_predictor_weights,
                                                             predictor_weight_spec)
    ws = init_predictor_weights(predictor_weight_spec(ins, 'MOBILE_NET', 64), seed=7, perturb=True)
    x = np.random.default_rng(8).random((3,) + ins).astype(np.float32)
    model = create_style_prediction_model(ins, 'MOBILE_NET', 64, weights=ws, max_batch=4)
    y = model(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = PR.style_predictor_forward(x, ws, 'MOBILE_NET')
    assert _rel(y, ref) < REL


def test_predictor_full_size_vs_torch_cpu():
    """rst-960-120-128-17 style input (480 x 960 x 3, P = 2662) against the torch-CPU f32 restatement."""
    _need_gpu()
    from oracle import predictor_ref as PR
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.stylePrediction import (create_style_prediction_model, init_predictor_weights,
                                                             predictor_weight_spec)
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins = cfg.input_shape['style'][1:]
    ws = init_predictor_weights(predictor_weight_spec(ins, cfg.style_feature_extractor_type, 2662), seed=3,
                                perturb=True)
    x = np.random.default_rng(9).random((2,) + tuple(ins)).astype(np.float32)
    model = create_style_prediction_model(ins, cfg.style_feature_extractor_type, 2662, weights=ws, max_batch=2)
    y = model(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = PR.torch_style_predictor_forward(x, ws, 'MOBILE_NET')
    assert y.shape == (2, 2662)
    assert _rel(y, ref) < REL
    # deterministic: no atomics, fixed reduction order
    y2 = model(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(y, y2)
    # batch independence (BatchNorm in inference mode, per-image pooling)
    y1 = model(torch.from_numpy(x[1:]).cuda()).cpu().numpy()
    assert np.array_equal(y1[0], y[1])


def test_inference_model_matches_oracle():
    """make_style_transfer_inference_model with MOBILE_NET (S=1): predictor -> transfer vs float64."""
    _need_gpu()
    from oracle import numpy_ref as R
    from oracle import predictor_ref as PR
    from realtime_style_transfer_amd.plan import init_weights, network_plan
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    from realtime_style_transfer_amd.stylePrediction import (create_style_prediction_model, init_predictor_weights,
                                                             predictor_weight_spec)
    from realtime_style_transfer_amd.styleTransferInferenceModel import make_style_transfer_inference_model
    ins, outs, bres, bf = (32, 64, 17), (32, 64, 3), 8, 8
    plan = network_plan(ins, outs, bres, bf)
    tw = init_weights(plan, seed=2)
    sins = (32, 64, 3)
    pw = init_predictor_weights(predictor_weight_spec(sins, 'MOBILE_NET', plan.num_style_params), seed=3, perturb=True)
    m = make_style_transfer_inference_model(
        num_styles=1,
        style_predictor_factory_func=lambda P: create_style_prediction_model(sins, 'MOBILE_NET', P, weights=pw),
        style_transfer_factory_func=lambda: create_style_transfer_model(ins, outs, bres, bf, 1, weights=tw,
                                                                        max_batch=2))
    assert m.inference.output_shape == (None,) + outs
    rng = np.random.default_rng(10)
    content = rng.random((2,) + ins).astype(np.float32)
    style = rng.random((2, 1) + sins).astype(np.float32)
    y = m.inference({'content': torch.from_numpy(content).cuda(), 'style': torch.from_numpy(style).cuda()})
    y = y.cpu().numpy()
    sp = PR.style_predictor_forward(style[:, 0], pw, 'MOBILE_NET')[:, None, :]
    ref = R.transfer_forward(content, sp, tw, ins, outs, bres, bf)
    assert np.abs(y - ref).max() < 2e-4


def test_inference_model_reference_geometry_two_styles():
    """styleTransferInferenceModelTest.py:18-53: 480x960x3 -> 1920x3840x3, two styles, DUMMY predictor."""
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    from realtime_style_transfer_amd.stylePrediction import StyleFeatureExtractor, create_style_prediction_model
    from realtime_style_transfer_amd.styleTransferInferenceModel import make_style_transfer_inference_model
    ie, oe, S = (480, 960, 3), (1920, 3840, 3), 2
    m = make_style_transfer_inference_model(
        num_styles=S,
        style_transfer_factory_func=lambda: create_style_transfer_model(
            input_shape=ie, output_shape=oe, bottleneck_res_y=120, bottleneck_num_filters=128, num_styles=S,
            name="StyleTransferTestModel", max_batch=1),
        style_predictor_factory_func=lambda P: create_style_prediction_model(ie, StyleFeatureExtractor.DUMMY, P),
        name="StyleTransferInferenceTestModel")
    assert m.inference.output_shape == (None,) + oe                       # test_output_shape_matches
    inputs = {'style': torch.zeros((1, S) + ie, device='cuda'), 'style_weights': torch.zeros((1,) + oe[:2] + (1,),
                                                                                                device='cuda'),
              'content': torch.zeros((1,) + ie, device='cuda')}
    y = m.inference.predict(inputs)                                       # test_inference (numpy, as Keras)
    assert isinstance(y, np.ndarray) and y.shape == (1,) + oe
    assert np.isfinite(y).all() and float(y.min()) > 0.0 and float(y.max()) < 1.0
