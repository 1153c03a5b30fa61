"""GPU parity of the training step (rst_trainer_*, librst) against the float64 autograd oracle.

Config A uses the production kernel shapes of rst-960-120-128-17 at a small frame (17 input
channels, 128 bottleneck filters); config B upsamples (output 2x the input, like the
reference's training-model test geometry, styleTransferTrainingModelTest.py:15-20) with
few filters. Tolerances (float32 GPU vs float64 oracle):
  prediction max-abs 2e-5; per-image losses rel 1e-4;
  every gradient tensor: relative L2 error ||g - ref|| / ||ref|| <= 2e-3 (biases feeding an
  instance norm are mathematically zero: there |g| <= 1e-5 x the layer's kernel-gradient scale);
  style-parameter gradients: relative L2 2e-3.
  Max-pool routing: VGG16's max-pool backward sends each window's gradient to its maximum, a
  discontinuous choice. Near-equal window values (e.g. 36.45983 vs 36.46031 at block4_conv3 in
  config B) are ordered differently by any float32 forward (this build's, and TF's own) than by
  the float64 oracle; one such flip moved a gradient entry to its neighbour and shifted every
  upstream gradient by ~1%. The oracle therefore takes the pool routing (only the choice of
  WHICH maximum) from the GPU's float32 activations of the four pooled layers; all arithmetic
  stays float64. The same holds for VGG16's ReLU masks: a pre-activation within rounding distance
  of 0 is active in one float32 forward and not in another (the exact-f32 and Winograd transfer
  convs give predictions 1.7e-6 apart, and one such unit moved dL/dprediction by 1.9 %), so the
  oracle's ReLU backward masks come from the GPU's post-ReLU activations too (relu_route).
  Max-norm errors are reported in gpurun_out/train_parity_*.json.
  after RMSprop: weights 1e-6 abs where |g_ref| > 5e-2 max|g_ref| of the tensor (elsewhere the
  first RMSprop step is lr*sign(g)/sqrt(1-rho) and only its size is checked), slots L2 5e-3.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CONFIGS = {
    'A': dict(input_shape=(32, 64, 17), output_shape=(32, 64, 3), bottleneck_res_y=8, bottleneck_num_filters=128),
    'B': dict(input_shape=(16, 32, 3), output_shape=(32, 64, 3), bottleneck_res_y=4, bottleneck_num_filters=4),
}
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _case(cfg, B, seed=5):
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.styleLoss import init_vgg16_weights
    plan = network_plan(cfg['input_shape'], cfg['output_shape'], cfg['bottleneck_res_y'], cfg['bottleneck_num_filters'])
    w = init_weights(plan, seed=2)
    vgg = init_vgg16_weights(seed=3)
    rng = np.random.default_rng(seed)
    content = rng.random((B,) + cfg['input_shape']).astype(np.float32)
    sp = synthetic_style_params(B, 1, plan.num_style_params, plan, seed=1)
    gtc = rng.random((B,) + cfg['output_shape']).astype(np.float32)
    gts = rng.random((B, 1) + cfg['output_shape']).astype(np.float32)
    return plan, w, vgg, content, sp, gtc, gts


def _trainer(cfg, w, vgg, B, precision="fp32", transfer="fp32"):
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
    from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
    lm = StyleLossModelVGG(cfg['output_shape'], weights=vgg, max_batch=B, precision=precision)
    return StyleTransferTrainingModel(cfg['input_shape'], cfg['output_shape'], cfg['bottleneck_res_y'],
                                      cfg['bottleneck_num_filters'], loss_model=lm, weights=w, max_batch=B,
                                      precision=transfer)


def _cuda(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


VGG_CONV_NAMES = ['block1_conv1', 'block1_conv2', 'block2_conv1', 'block2_conv2', 'block3_conv1', 'block3_conv2',
                  'block3_conv3', 'block4_conv1', 'block4_conv2', 'block4_conv3', 'block5_conv1', 'block5_conv2',
                  'block5_conv3']


def _relu_route(tr, B):
    return {i: tr.vgg_feature(n, B).cpu().numpy() for i, n in enumerate(VGG_CONV_NAMES)}


def _pool_route(tr, B):
    names = {1: 'block1_conv2', 3: 'block2_conv2', 6: 'block3_conv3', 9: 'block4_conv3'}
    return {i: tr.vgg_feature(n, B).cpu().numpy() for i, n in names.items()}


# precision: arithmetic of the VGG16 3x3 convs (forward and input gradient) — BASELINE config 4 trains
# in bf16; "bf16x6" is the exact 3-piece bf16 split (fp32-level products: same errors as fp32, L2 <= 1e-4),
# "bf16x3" the 2-piece split (16-bit operands). Round 1 measured a 2.26 % L2 deviation on
# residual_block_0_conv1 and loosened this bound to 5e-2; the cause was not bf16x3 rounding but ReLU
# routing: a VGG16 pre-activation within rounding distance of 0 was active in the GPU's float32 forward
# and inactive in the float64 oracle's, which moves every upstream gradient by ~1 %. With the oracle
# taking its ReLU masks from the GPU activations (relu_route) the worst bf16x3 gradient is 1.4e-4
# relative L2 (profiles/r02/train_parity_A_bf16x3.json), so the bound is back to 1e-3.
# "bf16": plain bf16 operands of the VGG16 convs, checked against the float64 oracle run with the same
# bf16 rounding of every VGG conv's input/kernel (forward) and output gradient/kernel (input gradient).
# That simulation matches block1_conv2 to 1e-6; beyond it the fp32-vs-float64 activation differences
# flip bf16 rounding decisions and the deviation grows layer by layer (tools/bf16_diag.py: 1.5e-4 after
# the first pool, 5.7e-3 at block5_conv3), so the transfer-net gradients carry bf16 noise (with the
# ReLU masks aligned: worst layer 1.8 % L2, loss terms 9e-4 / 1.8e-3 relative with the exact-f32 /
# Winograd transfer convs, measured)
# transfer: arithmetic of the transfer network's convs — "fp32" (exact-f32 MFMA), "fp32_winograd"
# (residual-block convs, forward + input gradient, as Winograd F(2x2,3x3): ~1e-6 relative per conv) or
# "winograd_bf16x6" (those residual convs and their weight gradient, and the 9x9 start conv's forward
# (wino9_x6 in its training mode: raw ReLU output + per-block statistics), on exact 3-piece split-bf16
# MFMA products: dropped terms <= 2^-25 per product, the same 2e-3 bound)
@pytest.mark.parametrize("name,precision,gtol,transfer", [
    ("A", "fp32", 2e-3, "fp32"), ("B", "fp32", 2e-3, "fp32"), ("A", "bf16x6", 2e-3, "fp32"),
    ("A", "bf16x3", 1e-3, "fp32"), ("A", "bf16", 0.05, "fp32"),
    ("A", "fp32", 2e-3, "fp32_winograd"), ("B", "fp32", 2e-3, "fp32_winograd"), ("A", "bf16", 0.05, "fp32_winograd"),
    ("A", "fp32", 2e-3, "winograd_bf16x6"), ("B", "fp32", 2e-3, "winograd_bf16x6"), ("A", "bf16", 0.05, "winograd_bf16x6")])
def test_training_step_matches_oracle(name, precision, gtol, transfer):
    _need_gpu()
    from oracle import torch_train as T
    cfg = CONFIGS[name]
    B = 2
    plan, w, vgg, content, sp, gtc, gts = _case(cfg, B)
    tr = _trainer(cfg, w, vgg, B, precision, transfer)
    c, s, gc, gs = _cuda(content, sp, gtc, gts)
    pred, losses, grad, gsp = tr.compute_gradients(c, s, gc, gs)
    torch.cuda.synchronize()
    ref = T.training_step(w, vgg, content, sp, gtc, gts, pool_route=_pool_route(tr, B), vgg_bf16=precision == "bf16",
                          relu_route=_relu_route(tr, B), **cfg)
    report = {}
    perr = float(np.abs(pred.cpu().numpy() - ref['prediction']).max())
    report['prediction_max_abs'] = perr
    lrel = float((np.abs(losses.cpu().numpy() - ref['losses']) / np.abs(ref['losses'])).max())
    report['loss_rel'] = lrel
    grads = tr._unflatten(grad.cpu().numpy())
    gerr = float(np.linalg.norm(gsp.cpu().numpy() - ref['grad_style_params']) /
                 np.linalg.norm(ref['grad_style_params']))
    report['style_grad_rel'] = gerr
    og = []
    for li in range(len(plan.layers) - 1, -1, -1):
        r = ref['output_grads'][li]
        g = tr.output_gradient(li, B).cpu().numpy()
        og.append((plan.layers[li].name, float(np.linalg.norm(g - r) / np.linalg.norm(r)),
                   float(np.abs(g - r).max() / np.abs(r).max())))
    report['output_grad_rel'] = og
    worst = []
    failures = []
    # kernel-gradient scale per layer (for the mathematically-zero biases before an instance norm)
    layer_of = []
    for layer in plan.layers:
        layer_of += [layer] * len(layer.weight_shapes)
    for i, (g, r) in enumerate(zip(grads, ref['grads'])):
        layer = layer_of[i]
        first = sum(len(l.weight_shapes) for l in plan.layers[:plan.layers.index(layer)])
        kscale = np.abs(ref['grads'][first]).max()
        err = float(np.linalg.norm(g - r))
        scale = float(np.linalg.norm(r))
        maxrel = float(np.abs(g - r).max() / max(np.abs(r).max(), 1e-30))
        # a bias feeding an instance norm (directly, or through a ReLU that never clips) has zero gradient
        zero_bias = (i == first + 1) and layer.norm == 'cin' and np.abs(r).max() <= 1e-9 * kscale
        if zero_bias:
            worst.append((layer.name + '/bias(zero)', float(np.abs(g).max() / kscale)))
            if not np.abs(g).max() <= 1e-5 * kscale:
                failures.append((layer.name, 'zero-bias', float(np.abs(g).max()), float(kscale)))
        elif scale == 0.0:
            if g.any():
                failures.append((layer.name, i - first, 'moving statistics got a gradient'))
        else:
            worst.append((f"{layer.name}/{i - first}", err / scale, maxrel))
            if not err <= gtol * scale:
                failures.append((layer.name, i - first, err, scale))
    report['grad_rel'] = worst
    report['failures'] = failures
    os.makedirs(OUT, exist_ok=True)
    tag = '' if transfer == 'fp32' else '_' + transfer
    with open(os.path.join(OUT, f'train_parity_{name}_{precision}{tag}.json'), 'w') as f:
        json.dump(report, f, indent=1, default=float)
    assert not failures, failures
    # moving statistics are updated by the forward (read back before the optimizer step)
    w_after_fwd = tr.get_weights()
    for i, layer in enumerate(layer_of):
        first = sum(len(l.weight_shapes) for l in plan.layers[:plan.layers.index(layer)])
        if layer.norm == 'bn' and i - first in (4, 5):
            np.testing.assert_allclose(w_after_fwd[i], ref['weights'][i], rtol=1e-5, atol=1e-6)
    # RMSprop
    tr.apply_gradients(grad)
    new_w = tr.get_weights()
    slots = tr.optimizer_slots()
    gmax = max(np.abs(g).max() for g in ref['grads'])
    for i, (a, r, g) in enumerate(zip(new_w, ref['weights'], ref['grads'])):
        if not g.any():
            continue   # BN moving statistics: not trained (checked after the forward above)
        assert np.abs(a - w_after_fwd[i]).max() <= 1e-3 / np.sqrt(0.1) * 1.001 + 1e-6, i
        if np.abs(g).max() <= 1e-9 * gmax:
            continue   # no gradient / round-off-only gradient (bias before an instance norm): sign is arbitrary
        strong = np.abs(g) > (0.5 if precision == "bf16" else 5e-2) * np.abs(g).max()   # no sign flips there
        assert np.abs(a - r)[strong].max() <= 1e-6 + 1e-6 * np.abs(r).max(), (i, np.abs(a - r)[strong].max())
        # ms = (1 - rho) g^2: its relative error is about twice the gradient's
        assert np.linalg.norm(slots[i] - ref['ms'][i]) <= max(5e-3, 2.5 * gtol) * np.linalg.norm(ref['ms'][i]), i
    assert perr < 2e-5, perr
    assert lrel < {"bf16x3": 1e-3, "bf16": 5e-3}.get(precision, 1e-4), lrel
    assert gerr < gtol, gerr


@pytest.mark.parametrize("transfer", ["fp32", "fp32_winograd", "winograd_bf16x6"])
def test_training_step_is_deterministic_and_learns(transfer):
    _need_gpu()
    cfg = CONFIGS['A']
    B = 2
    plan, w, vgg, content, sp, gtc, gts = _case(cfg, B)
    tr = _trainer(cfg, w, vgg, B, transfer=transfer)
    c, s, gc, gs = _cuda(content, sp, gtc, gts)
    _, l1, g1, s1 = tr.compute_gradients(c, s, gc, gs)
    g1, s1, l1 = g1.clone(), s1.clone(), l1.clone()
    _, l2, g2, s2 = tr.compute_gradients(c, s, gc, gs)
    assert torch.equal(g1, g2) and torch.equal(s1, s2) and torch.equal(l1, l2)   # no atomics anywhere
    first = None
    for _ in range(5):
        m = tr.train_step({'content': c, 'style_params': s}, {'content': gc, 'style': gs})
        first = first if first is not None else float(m['loss'])
    last = float(tr.compute_metrics()['loss'])
    assert last < first, (first, last)


def test_loss_targets_beside_the_predictor_are_bitwise_the_same():
    """rst_trainer_compute_targets (the style Grams and content features started on the trainer's side stream before
    the step's predictor forward) gives bitwise the losses and gradients of compute_gradients starting them itself;
    targets started for other ground truth are refused (RST_ERR_INVALID -> ValueError) and the trainer recovers."""
    _need_gpu()
    cfg = CONFIGS['A']
    B = 2
    plan, w, vgg, content, sp, gtc, gts = _case(cfg, B)
    tr = _trainer(cfg, w, vgg, B, precision="bf16", transfer="winograd_bf16x6")
    c, s, gc, gs = _cuda(content, sp, gtc, gts)
    _, l1, g1, s1 = tr.compute_gradients(c, s, gc, gs)
    l1, g1, s1 = l1.clone(), g1.clone(), s1.clone()
    tr.compute_targets(gc, gs)
    x = torch.randn(1 << 22, device=c.device)   # unrelated work queued on the main stream meanwhile
    for _ in range(4):
        x = torch.tanh(x)
    _, l2, g2, s2 = tr.compute_gradients(c, s, gc, gs)
    assert torch.equal(l1, l2) and torch.equal(g1, g2) and torch.equal(s1, s2)
    tr.compute_targets(gc, gs)
    with pytest.raises(ValueError, match="targets started for other inputs"):
        tr.compute_gradients(c, s, gc.clone(), gs)                    # other ground truth than the targets'
    _, l3, g3, _ = tr.compute_gradients(c, s, gc, gs)
    assert torch.equal(l1, l3) and torch.equal(g1, g3)


def test_trainer_rejects_bad_shapes():
    _need_gpu()
    from realtime_style_transfer_amd._lib import RstError
    cfg = CONFIGS['B']
    plan, w, vgg, content, sp, gtc, gts = _case(cfg, 1)
    tr = _trainer(cfg, w, vgg, 1)
    c, s, gc, gs = _cuda(content, sp, gtc, gts)
    with pytest.raises(ValueError):
        tr.compute_gradients(torch.cat([c, c]), s, gc, gs)            # batch > max_batch
    with pytest.raises(ValueError):
        tr.compute_gradients(c, s, gc, torch.cat([gs, gs], dim=1))    # two styles
    with pytest.raises(RstError):   # contract_1 sees 5 rows: odd size at a stride-2 level
        _trainer(dict(cfg, input_shape=(10, 20, 3), output_shape=(48, 80, 3), bottleneck_res_y=3), None, vgg, 1)


@pytest.mark.parametrize("factors", [(1e4, 0.0, 0.0), (0.0, 1e-3, 0.0), (0.0, 0.0, 1e-1)],
                         ids=["content", "style", "tv"])
def test_prediction_gradient_per_loss_term(factors):
    """d loss / d prediction (the VGG16 backward) for each loss term alone."""
    _need_gpu()
    from oracle import torch_train as T
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
    from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
    cfg = CONFIGS['B']
    B = 2
    plan, w, vgg, content, sp, gtc, gts = _case(cfg, B)
    lm = StyleLossModelVGG(cfg['output_shape'], weights=vgg, max_batch=B)
    lm.content_loss_factor, lm.style_loss_factor, lm.total_variation_loss_factor = factors
    tr = StyleTransferTrainingModel(cfg['input_shape'], cfg['output_shape'], cfg['bottleneck_res_y'],
                                    cfg['bottleneck_num_filters'], loss_model=lm, weights=w, max_batch=B)
    c, s, gc, gs = _cuda(content, sp, gtc, gts)
    from realtime_style_transfer_amd import _lib
    from realtime_style_transfer_amd.styleLoss import VGG16_CHANNELS
    lib = _lib.load()
    for i in range(13):
        _lib.check(lib.rst_trainer_debug_vgg_gradient(tr._handle, i, None, 0, B, _lib.stream_ptr()))
    tr.compute_gradients(c, s, gc, gs)
    ref = T.training_step(w, vgg, content, sp, gtc, gts, factors=factors, pool_route=_pool_route(tr, B),
                          relu_route=_relu_route(tr, B), **cfg)
    g = tr.output_gradient(len(plan.layers) - 1, B).cpu().numpy()
    r = ref['output_grads'][-1]
    rel = float(np.linalg.norm(g - r) / np.linalg.norm(r))
    vrel = []
    H, W = cfg['output_shape'][:2]
    for i in range(13):
        div = 2 ** sum(1 for p in (1, 3, 6, 9) if p < i)
        t = torch.empty((B, H // div, W // div, VGG16_CHANNELS[i]), device='cuda')
        _lib.check(lib.rst_trainer_debug_vgg_gradient(tr._handle, i, _lib.dev_ptr(t), t.numel(), B, _lib.stream_ptr()))
        rv = ref['vgg_grads'][i]
        vrel.append(float(np.linalg.norm(t.cpu().numpy() - rv) / max(np.linalg.norm(rv), 1e-30)))
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f'train_dpred_{factors}.json'), 'w') as f:
        json.dump({'rel': rel, 'scale': float(np.abs(r).max()), 'vgg_rel': vrel}, f)
    assert rel < 1e-3, rel


def test_joint_training_with_style_predictor_matches_oracle():
    """train_network.py's joint step: MobileNetV3Small predictor (training mode) -> style params -> transfer
    network -> VGG/Gram loss -> gradients of both weight sets (config B geometry, B=2)."""
    _need_gpu()
    from oracle import predictor_ref as PR
    from oracle import torch_train as T
    from realtime_style_transfer_amd.stylePrediction import (StylePredictionTrainer, init_predictor_weights,
                                                             predictor_weight_spec)
    cfg = CONFIGS['B']
    B = 2
    plan, w, vgg, content, _, gtc, gts = _case(cfg, B)
    P = plan.num_style_params
    sins = cfg['output_shape']
    spec = predictor_weight_spec(sins, 'MOBILE_NET', P)
    pw = init_predictor_weights(spec, seed=3, perturb=True)
    style = np.random.default_rng(12).random((B,) + sins).astype(np.float32)
    tr = _trainer(cfg, w, vgg, B)
    pr = StylePredictionTrainer(sins, 'MOBILE_NET', P, weights=pw, max_batch=B)
    c, gc, gs, st = _cuda(content, gtc, gts, style)
    sp = pr.forward(st)
    pred, losses, grad, gsp = tr.compute_gradients(c, sp, gc, gs)
    pgrad = pr.backward(gsp)
    torch.cuda.synchronize()
    sp_ref = PR.predictor_train_reference(style, pw, 'MOBILE_NET', np.zeros((B, P)))['output']
    assert np.abs(sp.cpu().numpy() - sp_ref).max() <= 1e-4 * np.abs(sp_ref).max()
    ref = T.training_step(w, vgg, content, sp.cpu().numpy().astype(np.float64), gtc, gts,
                          pool_route=_pool_route(tr, B), relu_route=_relu_route(tr, B), **cfg)
    gerr = float(np.linalg.norm(gsp.cpu().numpy() - ref['grad_style_params']) /
                 np.linalg.norm(ref['grad_style_params']))
    assert gerr < 2e-3, gerr
    pref = PR.predictor_train_reference(style, pw, 'MOBILE_NET', ref['grad_style_params'])
    got = pr.unflatten(pgrad)
    gscale = max(float(np.linalg.norm(r)) for r in pref['grads'])
    worst = 0.0
    for (name, shape, kind), a, r in zip(spec, got, pref['grads']):
        nr = float(np.linalg.norm(r))
        if kind in ('mean', 'var') or nr <= 1e-9 * gscale:
            assert np.linalg.norm(a) <= 1e-5 * gscale, name
            continue
        e = float(np.linalg.norm(a - r) / nr)
        worst = max(worst, e)
        assert e < 5e-3, (name, e)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, 'train_parity_joint_predictor.json'), 'w') as f:
        json.dump({'style_params_rel': float(np.abs(sp.cpu().numpy() - sp_ref).max() / np.abs(sp_ref).max()),
                   'grad_style_params_rel': gerr, 'predictor_grad_worst_rel': worst}, f, indent=1)


def test_predictor_backward_beside_the_transfer_backward_is_bitwise_serial():
    """train_step runs the style predictor's backward on a side stream from the point where the transfer network's
    backward has made d loss / d style_params final (rst_trainer_wait_style_gradient, after its last conditional
    instance norm), beside the contract layers' backward, and inside it the weight gradients and SE / head outer
    products run on a third stream beside its input-gradient chain: two joint steps give bitwise the weights (both
    networks) and losses of the fully serial order."""
    _need_gpu()
    from realtime_style_transfer_amd.stylePrediction import (StylePredictionTrainer, init_predictor_weights,
                                                             predictor_weight_spec)
    from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
    cfg = CONFIGS['B']
    B = 2
    plan, w, vgg, content, _, gtc, gts = _case(cfg, B)
    P = plan.num_style_params
    sins = cfg['output_shape']
    pw = init_predictor_weights(predictor_weight_spec(sins, 'MOBILE_NET', P), seed=3, perturb=True)
    style = np.random.default_rng(12).random((B, 1) + sins).astype(np.float32)
    c, gc, gs, st = _cuda(content, gtc, gts, style)
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
    runs = []
    for overlap in (False, True):
        lm = StyleLossModelVGG(cfg['output_shape'], weights=vgg, max_batch=B)
        # the serial reference also keeps the predictor's weight gradients on its backward's stream
        os.environ["RST_SERIAL_PREDICTOR_WGRAD"] = "0" if overlap else "1"
        try:
            pr = StylePredictionTrainer(sins, 'MOBILE_NET', P, weights=pw, max_batch=B)
        finally:
            del os.environ["RST_SERIAL_PREDICTOR_WGRAD"]
        tr = StyleTransferTrainingModel(cfg['input_shape'], cfg['output_shape'], cfg['bottleneck_res_y'],
                                        cfg['bottleneck_num_filters'], loss_model=lm, weights=w, max_batch=B,
                                        style_predictor=pr)
        tr._overlap_pbwd = overlap
        losses = []
        for _ in range(2):
            tr.train_step({'content': c, 'style': st}, {'content': gc, 'style': gs})
            losses.append(tr.style_losses['loss'].cpu().numpy())
        torch.cuda.synchronize()
        runs.append((np.concatenate([x.reshape(-1) for x in tr.get_weights()]),
                     np.concatenate([x.reshape(-1) for x in pr.get_weights()]), np.stack(losses)))
    for a, b in zip(runs[0], runs[1]):
        assert np.array_equal(a, b)


def test_joint_training_step_graph_replay_is_bitwise_eager():
    """train_step forks onto the loss targets' side stream and the predictor trainer's weight-gradient stream
    (and, eagerly, runs the predictor's backward on a third stream). A whole joint step captured into a hipGraph
    (tools/train_graph_check.py at test size) replays exactly what an eager step does: two trainers from the same state,
    eager steps vs replays -> bitwise weights (both networks) and losses, twice."""
    _need_gpu()
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
    from realtime_style_transfer_amd.stylePrediction import (StylePredictionTrainer, init_predictor_weights,
                                                             predictor_weight_spec)
    from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
    cfg = CONFIGS['A']
    B = 2
    plan, w, vgg, content, _, gtc, gts = _case(cfg, B)
    P = plan.num_style_params
    sins = cfg['output_shape']
    pw = init_predictor_weights(predictor_weight_spec(sins, 'MOBILE_NET', P), seed=3, perturb=True)
    style = np.random.default_rng(12).random((B, 1) + sins).astype(np.float32)
    c, gc, gs, st = _cuda(content, gtc, gts, style)
    x, y = {'content': c, 'style': st}, {'content': gc, 'style': gs}

    def make():
        lm = StyleLossModelVGG(cfg['output_shape'], weights=vgg, max_batch=B, precision="bf16")
        pr = StylePredictionTrainer(sins, 'MOBILE_NET', P, weights=pw, max_batch=B)
        return StyleTransferTrainingModel(cfg['input_shape'], cfg['output_shape'], cfg['bottleneck_res_y'],
                                          cfg['bottleneck_num_filters'], loss_model=lm, weights=w, max_batch=B,
                                          style_predictor=pr, precision="winograd_bf16x6")
    a, b = make(), make()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        a.train_step(x, y)
        b.train_step(x, y)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.train_step(x, y)
    for _ in range(2):
        a.train_step(x, y)
        g.replay()
        torch.cuda.synchronize()
        wa = np.concatenate([q.ravel() for q in a.get_weights()] + [q.ravel() for q in a.style_predictor.get_weights()])
        wb = np.concatenate([q.ravel() for q in b.get_weights()] + [q.ravel() for q in b.style_predictor.get_weights()])
        assert np.array_equal(wa, wb)
        assert np.array_equal(a.style_losses['loss'].cpu().numpy(), b.style_losses['loss'].cpu().numpy())


def test_training_model_reference_geometry_with_dummy_predictor():
    """styleTransferTrainingModelTest.py:15-58: 240x480x3 -> 480x960x3, bottleneck 30 rows x 4 filters,
    DUMMY predictor, a fit over two zero samples in one batch of 2 (the VGG loss stands in for
    StyleLossModelDummy; the MiDaS depth term is a TF-Hub download, so with_depth_loss=False)."""
    _need_gpu()
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG, make_style_loss_function
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    from realtime_style_transfer_amd.stylePrediction import StyleFeatureExtractor, create_style_prediction_model
    from realtime_style_transfer_amd.styleTransferTrainingModel import make_style_transfer_training_model
    ie, oe = (240, 480, 3), (480, 960, 3)
    m = make_style_transfer_training_model(
        style_transfer_factory_func=lambda: create_style_transfer_model(ie, oe, 30, 4, num_styles=1,
                                                                        name="StyleTransferTestModel", max_batch=2),
        style_predictor_factory_func=lambda P: create_style_prediction_model(oe, StyleFeatureExtractor.DUMMY, P),
        style_loss_func_factory_func=lambda: make_style_loss_function(StyleLossModelVGG(oe, max_batch=2), oe, 1,
                                                                  with_depth_loss=False),
        name="StyleTransferTrainingTestModel", max_batch=2)
    x = {'content': torch.zeros((2,) + ie, device='cuda'), 'style': torch.zeros((2, 1) + oe, device='cuda')}
    y = {'content': torch.zeros((2,) + oe, device='cuda'), 'style': torch.zeros((2, 1) + oe, device='cuda')}
    w0 = m.training.style_predictor.get_weights()
    metrics = m.training.train_step(x, y)
    torch.cuda.synchronize()
    assert set(metrics) == {'loss', 'feature_loss', 'style_loss', 'total_variation_loss'}
    assert all(bool(torch.isfinite(v)) for v in metrics.values())
    w1 = m.training.style_predictor.get_weights()
    assert any(not np.array_equal(a, b) for a, b in zip(w0, w1)), "the predictor was not trained"
    m.refresh()
    out = m.inference({'content': x['content'], 'style': x['style']})
    assert tuple(out.shape) == (2,) + oe


@pytest.mark.parametrize("transfer,joint", [("fp32_winograd", False), ("winograd_bf16x6", True)],
                         ids=["fp32_winograd", "bench_line"])
def test_full_size_bf16_training_step_properties(transfer, joint):
    """BASELINE config 4 at its real size (train_network.py:61: B=4, 480x960 frames, rst-960-120-128-17;
    the VGG16 convs in bf16 as bench.py's training headline). ``bench_line`` is exactly bench.py's config-4
    line: transfer convs on winograd_bf16x6, bf16 VGG16 and the MobileNetV3Small style predictor trained
    jointly (x = {'content', 'style'}, train_network.py:86-138). The float64 oracle cannot run this size, so
    the test checks size-independent properties — every loss / gradient / weight finite, two trainers from
    the same weights and inputs bitwise identical after three steps (no atomics, fixed reduction order),
    and the batch loss decreasing over three RMSprop steps on one batch."""
    _need_gpu()
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.stylePrediction import StylePredictionTrainer
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
    from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
    sc = ShapeConfig.from_spec("rst-960-120-128-17")
    cfg = dict(input_shape=sc.input_shape['content'], output_shape=sc.output_shape,
               bottleneck_res_y=sc.bottleneck_res_y, bottleneck_num_filters=sc.bottleneck_num_filters)
    B = 4
    plan, w, vgg, content, sp, gtc, gts = _case(cfg, B)
    c, s, gc, gs = _cuda(content, sp, gtc, gts)
    sins = tuple(sc.input_shape['style'][1:])
    style = torch.from_numpy(np.random.default_rng(11).random((B, 1) + sins, dtype=np.float32)).cuda()
    runs = []
    for _ in range(2):
        pr = StylePredictionTrainer(sins, sc.style_feature_extractor_type, plan.num_style_params,
                                    max_batch=B) if joint else None
        lm = StyleLossModelVGG(cfg['output_shape'], weights=vgg, max_batch=B, precision="bf16")
        tr = StyleTransferTrainingModel(cfg['input_shape'], cfg['output_shape'], cfg['bottleneck_res_y'],
                                        cfg['bottleneck_num_filters'], loss_model=lm, weights=w, max_batch=B,
                                        precision=transfer, style_predictor=pr)
        x = {'content': c, 'style': style} if joint else {'content': c, 'style_params': s}
        losses = []
        for _step in range(3):
            m = tr.train_step(x, {'content': gc, 'style': gs})
            losses.append(float(m['loss']))
            assert all(np.isfinite(float(v)) for v in m.values())
            assert bool(torch.isfinite(tr._bucket).all())
        torch.cuda.synchronize()
        flat = np.concatenate([a.reshape(-1) for a in tr.get_weights()])
        assert np.all(np.isfinite(flat))
        pflat = np.concatenate([a.reshape(-1) for a in pr.get_weights()]) if joint else np.zeros(0)
        assert np.all(np.isfinite(pflat))
        runs.append((losses, flat, pflat, tr.last_prediction.cpu().numpy()))
        del tr, pr, lm
        torch.cuda.empty_cache()
    (l0, w0, q0, p0), (l1, w1, q1, p1) = runs
    assert l0 == l1 and np.array_equal(w0, w1) and np.array_equal(p0, p1), "training is not bitwise deterministic"
    assert np.array_equal(q0, q1), "predictor training is not bitwise deterministic"
    assert l0[2] < l0[1] < l0[0], l0


def _grad_report(plan, tr, grads, ref, B):
    """Relative L2 error per trainable transfer tensor (zero-gradient biases before an instance norm and the BN moving
    statistics reported apart) and per layer output gradient."""
    layer_of = []
    for layer in plan.layers:
        layer_of += [layer] * len(layer.weight_shapes)
    rows, zero_bias = [], []
    for i, (g, r) in enumerate(zip(grads, ref['grads'])):
        layer = layer_of[i]
        first = sum(len(l.weight_shapes) for l in plan.layers[:plan.layers.index(layer)])
        kscale = float(np.abs(ref['grads'][first]).max())
        scale = float(np.linalg.norm(r))
        # a bias feeding an instance norm through a ReLU that never clips: zero up to round-off, which the float32
        # oracle leaves at ~1e-7 of the kernel gradient's scale (the float64 small tests: 1e-9)
        if i == first + 1 and layer.norm == 'cin' and np.abs(r).max() <= 1e-4 * kscale:
            zero_bias.append((layer.name, float(np.abs(g).max() / kscale), float(np.abs(r).max() / kscale)))
        elif scale > 0.0:
            rows.append((f"{layer.name}/{i - first}", float(np.linalg.norm(g - r)) / scale))
    og = []
    for li in range(len(plan.layers)):
        r = ref['output_grads'][li]
        g = tr.output_gradient(li, B).cpu().numpy()
        og.append((plan.layers[li].name, float(np.linalg.norm(g - r) / np.linalg.norm(r))))
    return rows, zero_bias, og


@pytest.mark.parametrize("size,precision,transfer", [
    ("full", "fp32", "winograd_bf16x6"),     # BASELINE config 4's transfer arithmetic at 480x960 (bench.py's trainer)
    ("quarter", "bf16", "winograd_bf16x6"),  # the bench's bf16 VGG16 line against its bf16 simulation, 128x256
    ("full", "bf16", "winograd_bf16x6"),     # ... and at the bench's own 480x960
], ids=["config4_480x960_fp32_vgg", "config4_128x256_bf16_vgg", "config4_480x960_bf16_vgg"])
def test_training_step_at_scale_matches_f32_oracle(size, precision, transfer):
    """Config 4 (train_network.py:61,102,128-138) past the small parity shapes: one training step of the benchmarked
    trainer (winograd_bf16x6 transfer convs, its default split-bf16 start-conv weight gradient, style parameters as
    input) against oracle/torch_train.py run in float32 autograd on the host (the float64 oracle would take minutes at
    this size; the reference's own arithmetic is float32), max-pool / ReLU routing from the GPU as in the small tests.
    ``full``: 480x960 (rst-960-120-128-17), B=1, VGG16 in fp32 or in plain bf16. ``quarter``: 128x256 (bottleneck
    32 x 128; VGG16's four pools need multiples of 16), B=1. Plain bf16 is checked against the oracle's _Bf16Conv /
    _Bf16Store / _Bf16Gram simulation of it (bf16 operands, layer outputs and input gradients).
    Bounds (float32-level GPU vs float32 host, both rounding): prediction max-abs 5e-5, per-image loss terms rel 5e-4,
    style-parameter gradient and every transfer gradient tensor rel L2 5e-3 (bf16 VGG: 0.05 / loss 5e-3, the
    small-shape bf16 bounds: bf16 rounding flips between two different float32 forwards)."""
    _need_gpu()
    from oracle import torch_train as T
    if size == "full":
        from realtime_style_transfer_amd.shape_config import ShapeConfig
        sc = ShapeConfig.from_spec("rst-960-120-128-17")
        cfg = dict(input_shape=sc.input_shape['content'], output_shape=sc.output_shape,
                   bottleneck_res_y=sc.bottleneck_res_y, bottleneck_num_filters=sc.bottleneck_num_filters)
    else:
        cfg = dict(input_shape=(128, 256, 17), output_shape=(128, 256, 3), bottleneck_res_y=32,
                   bottleneck_num_filters=128)
    B = 1
    plan, w, vgg, content, sp, gtc, gts = _case(cfg, B, seed=9)
    tr = _trainer(cfg, w, vgg, B, precision, transfer)
    c, s, gc, gs = _cuda(content, sp, gtc, gts)
    pred, losses, grad, gsp = tr.compute_gradients(c, s, gc, gs)
    torch.cuda.synchronize()
    pool, relu = _pool_route(tr, B), _relu_route(tr, B)
    ref = T.training_step(w, vgg, content, sp, gtc, gts, pool_route=pool, relu_route=relu, vgg_bf16=precision == "bf16",
                          dtype=torch.float32, **cfg)
    del pool, relu
    perr = float(np.abs(pred.cpu().numpy() - ref['prediction']).max())
    lrel = float((np.abs(losses.cpu().numpy() - ref['losses']) / np.abs(ref['losses'])).max())
    gerr = float(np.linalg.norm(gsp.cpu().numpy() - ref['grad_style_params']) /
                 np.linalg.norm(ref['grad_style_params']))
    rows, zero_bias, og = _grad_report(plan, tr, tr._unflatten(grad.cpu().numpy()), ref, B)
    report = dict(size=size, precision=precision, transfer=transfer, prediction_max_abs=perr, loss_rel=lrel,
                  style_grad_rel=gerr, grad_rel=rows, zero_bias_rel_to_kernel_scale=zero_bias, output_grad_rel=og)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f'train_parity_scale_{size}_{precision}_{transfer}.json'), 'w') as f:
        json.dump(report, f, indent=1, default=float)
    gtol, ltol, ptol = (0.05, 5e-3, 5e-4) if precision == "bf16" else (5e-3, 5e-4, 5e-5)
    assert perr < ptol, perr
    assert lrel < ltol, lrel
    assert gerr < gtol, gerr
    bad = [r for r in rows if not r[1] <= gtol]
    assert not bad, bad
    # biases feeding an instance norm: mathematically zero gradient, round-off only on both sides
    assert all(g <= 1e-4 for _, g, _r in zero_bias), zero_bias
