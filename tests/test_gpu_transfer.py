"""GPU parity of the transfer network (librst on MI355X) against the CPU oracle.

Tolerances: the HIP path computes in exact f32 (f32-input MFMA = fmaf chains); the oracle
is float64 (numpy) or float32 (torch-CPU, full size). North-star bar: <= 1e-3 max-abs on
the [0, 1] output; observed deviations are ~1e-5, so the tests assert 2e-4 on outputs.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

OUT_TOL = 2e-4
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _load_fixture(name):
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), 'golden', name))
    ws = [d[k] for k in sorted(k for k in d.files if k.startswith('w') and k[1:].isdigit())]
    shape = d['shape']
    ins, outs, bres, bf = tuple(shape[0:3]), tuple(shape[3:6]), int(shape[6]), int(shape[7])
    return d, ws, ins, outs, bres, bf


@pytest.mark.parametrize("fixture", ["transfer_small.npz", "transfer_up.npz"])
def test_transfer_matches_golden(fixture):
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    d, ws, ins, outs, bres, bf = _load_fixture(fixture)
    model, P = create_style_transfer_model(ins, outs, bres, bf, 1, weights=ws, max_batch=2)
    assert P == d['style_params'].shape[-1]
    content = torch.from_numpy(d['content']).cuda()
    sp = torch.from_numpy(d['style_params']).cuda()
    y = model({'content': content, 'style_params': sp}).cpu().numpy()
    err = np.abs(y - d['output']).max()
    assert y.shape == d['output'].shape
    assert err < OUT_TOL, f"max abs err {err}"


def test_layer_outputs_match_oracle():
    """Every block's emitted tensor (as the Keras sub-model returns it) vs the float64 oracle."""
    _need_gpu()
    from oracle import numpy_ref as R
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    d, ws, ins, outs, bres, bf = _load_fixture("transfer_small.npz")
    model, _ = create_style_transfer_model(ins, outs, bres, bf, 1, weights=ws, max_batch=2)
    x, sp = d['content'], d['style_params']
    model({'content': torch.from_numpy(x).cuda(), 'style_params': torch.from_numpy(sp).cuda()})
    _, inter = R.transfer_forward(x, sp, ws, ins, outs, bres, bf, return_intermediates=True)
    ref = list(inter.values())
    # conv layer idx -> oracle block idx: contract layers 1:1, residual blocks emit after conv1
    layers = model.plan.layers
    bi = 0
    for li, layer in enumerate(layers):
        if layer.block.startswith('residual') and layer.name.endswith('conv0'):
            continue
        got = model.layer_output(li, 2).cpu().numpy()
        want = ref[bi]
        scale = max(1.0, float(np.abs(want).max()))
        err = np.abs(got - want).max() / scale
        assert err < 1e-4, f"layer {layer.name}: rel err {err}"
        bi += 1
    assert bi == len(ref)


def test_full_size_matches_torch_oracle():
    """rst-960-120-128-17 (480x960x17 -> 480x960x3), B=1, vs the torch-CPU f32 restatement."""
    _need_gpu()
    from oracle.torch_ref import TorchTransfer
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    ws = init_weights(plan, seed=2)
    model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                           weights=ws, max_batch=1)
    assert P == 2662
    x = np.random.default_rng(0).random((1,) + ins).astype(np.float32)
    sp = synthetic_style_params(1, 1, P, plan, seed=1)
    y = model({'content': torch.from_numpy(x).cuda(), 'style_params': torch.from_numpy(sp).cuda()}).cpu().numpy()
    ref = TorchTransfer(ws, ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)(x, sp)
    err = np.abs(y - ref).max()
    assert err < 1e-3, f"max abs err {err} (north-star bound 1e-3)"
    assert err < OUT_TOL, f"max abs err {err}"
    # pixel export parity: uint8(x*255) truncation (predict_using_checkpoint.py:99)
    mism = np.mean(np.uint8(y * 255) != np.uint8(ref * 255))
    assert mism < 1e-3


def test_l2_weight_prefetch_is_numerically_neutral():
    """The next-layer weight touches (kernels.h l2_touch_xcd_slice; RST_NO_U_PREFETCH=1 turns them off at handle
    creation) only move lines into L2: the full-size frame is bitwise the same with and without them (the CIN
    statistics are fixed-point limb sums, kernels.h, so their arrival order cannot change a rounding)."""
    _need_gpu()
    import os
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    ws = init_weights(plan, seed=2)
    rng = np.random.default_rng(11)
    x = torch.from_numpy(rng.random((1,) + ins).astype(np.float32)).cuda()
    sp = torch.from_numpy(np.ascontiguousarray(synthetic_style_params(1, 1, plan.num_style_params, plan, seed=4))).cuda()
    ys = []
    for off in ("1", None):
        old = os.environ.pop("RST_NO_U_PREFETCH", None)
        if off:
            os.environ["RST_NO_U_PREFETCH"] = off
        try:
            m, _ = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                               weights=ws, max_batch=1)
        finally:
            os.environ.pop("RST_NO_U_PREFETCH", None)
            if old is not None:
                os.environ["RST_NO_U_PREFETCH"] = old
        ys.append(m({'content': x, 'style_params': sp}).cpu().numpy())
        del m
    assert np.isfinite(ys[0]).all()
    assert np.array_equal(ys[0], ys[1]), np.abs(ys[0] - ys[1]).max()


def test_timeline_stamps_are_neutral_and_ordered():
    """rst_timeline_* (bench.graph_layer_ms's in-graph layer times): the stamping kernels' extra vector store per
    wave leaves the frame bitwise unchanged, eager and replayed from a captured hipGraph; every residual conv and
    narrow conv stamps, and the stamps of one frame's stamped layers are increasing (one stream, in layer order)."""
    _need_gpu()
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    m, _ = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                       weights=init_weights(plan, seed=2), max_batch=1, precision="winograd_bf16x6")
    rng = np.random.default_rng(12)
    x = torch.from_numpy(rng.random((1,) + ins).astype(np.float32)).cuda()
    sp = torch.from_numpy(np.ascontiguousarray(synthetic_style_params(1, 1, plan.num_style_params, plan, seed=5))).cuda()
    inp = {'content': x, 'style_params': sp}
    y0 = m(inp).cpu().numpy()
    m.timeline_begin()
    try:
        y1 = m(inp).cpu().numpy()
        e_eager = m.timeline_read()
        out = torch.empty_like(torch.from_numpy(y0)).cuda()
        s = torch.cuda.Stream()   # bench.capture_graph's recipe: a warm-up launch on a side stream, then the capture
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(inp, out=out)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            m(inp, out=out)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        y2 = out.cpu().numpy()
        e_graph = m.timeline_read()
        del g
        torch.cuda.synchronize()
    finally:
        m.timeline_end()
    assert np.array_equal(y0, y1) and np.array_equal(y0, y2)
    for e in (e_eager, e_graph):
        st = e[np.isfinite(e)]
        assert st.size >= 14, e            # ten residual convs, four narrow convs
        assert np.all(np.diff(st) > 0), e


def test_full_size_repeated_calls_mixed_batch():
    """Full size, one handle: B=2, then B=1 on other content, then B=2 again all match the oracle and
    the repeated call is bitwise equal (no state — CIN partials, affines, workspaces — carries over
    from a previous call; expand_1's finalize walks 14400 partials per channel here)."""
    _need_gpu()
    from oracle.torch_ref import TorchTransfer
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    ws = init_weights(plan, seed=2)
    model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                           weights=ws, max_batch=2)
    ref_net = TorchTransfer(ws, ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    rng = np.random.default_rng(7)
    x2 = rng.random((2,) + ins).astype(np.float32)
    x1 = rng.random((1,) + ins).astype(np.float32)
    sp2 = synthetic_style_params(2, 1, P, plan, seed=3)

    def run(x, sp):
        return model({'content': torch.from_numpy(x).cuda(),
                      'style_params': torch.from_numpy(np.ascontiguousarray(sp)).cuda()}).cpu().numpy()

    ya = run(x2, sp2)
    yb = run(x1, sp2[1:])
    yc = run(x2, sp2)
    assert np.array_equal(ya, yc)
    for y, x, sp in ((ya[:1], x2[:1], sp2[:1]), (ya[1:], x2[1:], sp2[1:]), (yb, x1, sp2[1:])):
        err = np.abs(y - ref_net(x, sp)).max()
        assert err < OUT_TOL, f"max abs err {err}"


def test_batch_and_determinism():
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    d, ws, ins, outs, bres, bf = _load_fixture("transfer_small.npz")
    model, _ = create_style_transfer_model(ins, outs, bres, bf, 1, weights=ws, max_batch=2)
    content = torch.from_numpy(d['content']).cuda()
    sp = torch.from_numpy(d['style_params']).cuda()
    y2 = model({'content': content, 'style_params': sp})
    y2b = model({'content': content, 'style_params': sp})
    assert torch.equal(y2, y2b), "forward is not bitwise deterministic"
    y0 = model({'content': content[:1].contiguous(), 'style_params': sp[:1].contiguous()})
    y1 = model({'content': content[1:].contiguous(), 'style_params': sp[1:].contiguous()})
    assert torch.equal(torch.cat([y0, y1]), y2), "batched result differs from per-frame result"


def test_shape_errors_raise():
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    d, ws, ins, outs, bres, bf = _load_fixture("transfer_small.npz")
    model, P = create_style_transfer_model(ins, outs, bres, bf, 1, weights=ws, max_batch=2)
    good = torch.zeros((1,) + ins, device='cuda')
    with pytest.raises(ValueError):
        model({'content': torch.zeros((1, 8, 8, ins[2]), device='cuda'), 'style_params': torch.zeros(1, 1, P,
                                                                                                  device='cuda')})
    with pytest.raises(ValueError):
        model({'content': good, 'style_params': torch.zeros(1, 1, P + 1, device='cuda')})
    with pytest.raises(ValueError):
        model({'content': torch.zeros((3,) + ins, device='cuda'), 'style_params': torch.zeros(3, 1, P, device='cuda')})
    with pytest.raises(ValueError):
        create_style_transfer_model(ins, outs, bres, bf, 1, weights=ws[:-1])


def test_instance_norm_op():
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import instance_norm
    g = torch.Generator().manual_seed(3)
    x = (torch.rand(2, 37, 53, 24, generator=g) * 3 + 10).cuda()     # large mean: cancellation check
    scale = torch.rand(2, 24, generator=g).cuda() + 0.5
    bias = torch.randn(2, 24, generator=g).cuda()
    y = instance_norm(x, scale, bias, relu=True)
    xd = x.double()
    mean = xd.mean(dim=(1, 2), keepdim=True)
    var = ((xd - mean) ** 2).mean(dim=(1, 2), keepdim=True)
    ref = torch.relu(bias.double()[:, None, None, :] + (xd - mean) / torch.sqrt(var + 1e-5) *
                     scale.double()[:, None, None, :])
    assert (y.double() - ref).abs().max().item() < 1e-4


def test_two_style_blending_matches_golden():
    """num_styles=2: per-pixel blend of the CIN parameters with the style-weight mips."""
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    d = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'transfer_two_styles.npz'))
    ws = [d[k] for k in sorted(k for k in d.files if k.startswith('w') and k[1:].isdigit())]
    shape = d['shape']
    ins, outs, bres, bf = tuple(shape[0:3]), tuple(shape[3:6]), int(shape[6]), int(shape[7])
    model, P = create_style_transfer_model(ins, outs, bres, bf, 2, weights=ws, max_batch=2)
    inputs = {'content': torch.from_numpy(d['content']).cuda(), 'style_params': torch.from_numpy(d['style_params']).cuda(),
              'style_weights': torch.from_numpy(d['style_weights']).cuda()}
    y = model(inputs).cpu().numpy()
    assert np.abs(y - d['output']).max() < 2e-5, np.abs(y - d['output']).max()
    # limits: all-zero / all-one weights == single-style model with style 0 / style 1
    single, _ = create_style_transfer_model(ins, outs, bres, bf, 1, weights=ws, max_batch=2)
    for val, s in ((0.0, 0), (1.0, 1)):
        inputs['style_weights'] = torch.full_like(inputs['style_weights'], val)
        y2 = model(inputs).cpu().numpy()
        y1 = single({'content': inputs['content'], 'style_params': inputs['style_params'][:, s:s + 1].contiguous()})
        assert np.abs(y2 - y1.cpu().numpy()).max() < 1e-5
    with pytest.raises(ValueError):
        model({'content': inputs['content'], 'style_params': inputs['style_params']})   # weights missing


@pytest.mark.parametrize("precision", ["winograd_bf16x6", "fp32"])
def test_two_styles_on_fast_kernels_match_oracle(precision):
    """num_styles=2 (styleTransfer.py:36-44,288-303) with the production residual width (128 filters): the
    headline precision runs the residual convs on the split-bf16 Winograd kernel with its per-pixel blend
    prologue (wino_x6 BLEND), the start conv on wino9_x6 and the last layer on last_x6 (blended input
    materialised); checked against the float64 oracle and, at the 0/1 weight limits, against the single-style
    model with each style."""
    _need_gpu()
    from oracle import numpy_ref as R
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    ins, outs, br, bf = (32, 64, 17), (32, 64, 3), 8, 128
    plan = network_plan(ins, outs, br, bf, 2)
    w = init_weights(plan, seed=2)
    rng = np.random.default_rng(21)
    x = rng.random((2,) + ins).astype(np.float32)
    sp = synthetic_style_params(2, 2, plan.num_style_params, plan, seed=4)
    sw = rng.random((2,) + outs[:2] + (1,)).astype(np.float32)
    m, P = create_style_transfer_model(ins, outs, br, bf, 2, weights=w, max_batch=2, precision=precision)
    inputs = {'content': torch.from_numpy(x).cuda(), 'style_params': torch.from_numpy(sp).cuda(),
              'style_weights': torch.from_numpy(sw).cuda()}
    y = m(inputs).cpu().numpy()
    ref = R.transfer_forward(x, sp, w, ins, outs, br, bf, style_weights=sw)
    err = np.abs(y - ref).max()
    assert err < 2e-5, f"max abs err {err}"
    single, _ = create_style_transfer_model(ins, outs, br, bf, 1, weights=w, max_batch=2, precision=precision)
    for val, s in ((0.0, 0), (1.0, 1)):
        inputs['style_weights'] = torch.full_like(inputs['style_weights'], val)
        y2 = m(inputs).cpu().numpy()
        y1 = single({'content': inputs['content'], 'style_params': inputs['style_params'][:, s:s + 1].contiguous()})
        assert np.abs(y2 - y1.cpu().numpy()).max() < 1e-5


def test_two_styles_full_size_properties():
    """rst-960-120-128-17 with two styles at full size (480x960): finite, in (0, 1), deterministic, and
    between-the-styles behaviour at the 0/1 weight limits (the float64 oracle is too slow at this size)."""
    _need_gpu()
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17", num_styles=2)
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 2)
    w = init_weights(plan, seed=2)
    m, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 2, weights=w,
                                       max_batch=1)
    single, _ = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1, weights=w,
                                            max_batch=1)
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.random((1,) + ins, dtype=np.float32)).cuda()
    sp = torch.from_numpy(synthetic_style_params(1, 2, P, plan, seed=6)).cuda()
    sw = torch.from_numpy(rng.random((1,) + outs[:2] + (1,), dtype=np.float32)).cuda()
    y = m({'content': x, 'style_params': sp, 'style_weights': sw})
    y2 = m({'content': x, 'style_params': sp, 'style_weights': sw})
    assert torch.equal(y, y2)
    assert bool(torch.isfinite(y).all()) and float(y.min()) > 0.0 and float(y.max()) < 1.0
    for val, s in ((0.0, 0), (1.0, 1)):
        yl = m({'content': x, 'style_params': sp, 'style_weights': torch.full_like(sw, val)})
        ys = single({'content': x, 'style_params': sp[:, s:s + 1].contiguous()})
        assert float((yl - ys).abs().max()) < 1e-5


@pytest.mark.parametrize("precision,tol", [("bf16x3", 2e-4), ("bf16x6", 2e-5), ("bf16", 2e-4)])
def test_split_bf16_precision_modes(precision, tol):
    """RST_PRECISION_BF16X3 / BF16X6 / BF16: residual convs on the bf16 MFMA pipe, vs the float64 oracle
    (for plain bf16: the oracle with the same bf16 rounding of the residual convs' operands)."""
    _need_gpu()
    from oracle import numpy_ref as R
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    ins, outs, br, bf = (32, 64, 17), (32, 64, 3), 8, 128
    plan = network_plan(ins, outs, br, bf)
    w = init_weights(plan, seed=2)
    sp = synthetic_style_params(2, 1, plan.num_style_params, plan, seed=1)
    x = np.random.default_rng(0).random((2,) + ins).astype(np.float32)
    ref = R.transfer_forward(x, sp, w, ins, outs, br, bf,
                             operand_round=R.bf16_round if precision == "bf16" else None)
    m, _ = create_style_transfer_model(ins, outs, br, bf, 1, weights=w, max_batch=2, precision=precision,
                                       allow_reduced_precision=precision == "bf16")
    kid = {"bf16x3": 102, "bf16x6": 113, "bf16": 134}[precision]
    assert [m.layer_kernel_id(i) for i in range(m.num_layers())][3:13] == [kid] * 10   # residual convs
    inp = {'content': torch.from_numpy(x).cuda(), 'style_params': torch.from_numpy(sp).cuda()}
    err = float(np.abs(m(inp).cpu().numpy() - ref).max())
    import json
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f'{precision}_parity.json'), 'w') as f:
        json.dump({'max_abs': err}, f)
    assert err < tol, err   # bf16x3: the float64 simulation of the split gives ~2e-5 here; fp32 gives ~2e-6


WINO_MODES = {"fp32_winograd": (201, 200), "winograd_bf16x6": (205, 202)}   # (start conv, residual) kernel ids


@pytest.mark.parametrize("precision", list(WINO_MODES))
def test_winograd_residual_convs_match_oracle(precision):
    """RST_PRECISION_FP32_WINOGRAD: residual convs as fused Winograd F(2x2,3x3) and the 9x9 start conv as
    nine F(2x2,3x3) sub-convolutions on f32 MFMA vs float64, small geometry (production channel counts)
    and odd sizes (partial 8x16 tiles). RST_PRECISION_WINOGRAD_BF16X6: the same with the residual convs'
    transform-domain products as exact 3-piece split-bf16 MFMA terms (fp32-level: same bounds)."""
    _need_gpu()
    from oracle import numpy_ref as R
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    for ins, outs, br in (((32, 64, 17), (32, 64, 3), 8), ((44, 76, 17), (44, 76, 3), 11)):
        bf = 128
        plan = network_plan(ins, outs, br, bf)
        w = init_weights(plan, seed=2)
        sp = synthetic_style_params(2, 1, plan.num_style_params, plan, seed=1)
        x = np.random.default_rng(0).random((2,) + ins).astype(np.float32)
        ref = R.transfer_forward(x, sp, w, ins, outs, br, bf)
        m, _ = create_style_transfer_model(ins, outs, br, bf, 1, weights=w, max_batch=2, precision=precision)
        ids = [m.layer_kernel_id(i) for i in range(m.num_layers())]
        assert ids[0] == WINO_MODES[precision][0] and ids[3:13] == [WINO_MODES[precision][1]] * 10, ids
        inp = {'content': torch.from_numpy(x).cuda(), 'style_params': torch.from_numpy(sp).cuda()}
        y = m(inp)
        err = float(np.abs(y.cpu().numpy() - ref).max())
        assert err < OUT_TOL, (ins, err)
        assert torch.equal(y, m(inp)), "Winograd forward is not deterministic"
        # every residual block output against the float64 oracle
        _, inter = R.transfer_forward(x, sp, w, ins, outs, br, bf, return_intermediates=True)
        # the 9x9 start conv (composite Winograd, ReLU -> BN -> ReLU) against the float64 oracle
        r0 = list(inter.values())[0]
        g0 = m.layer_output(0, 2).cpu().numpy()
        assert g0.shape == r0.shape and np.abs(g0 - r0).max() / max(1.0, np.abs(r0).max()) < 1e-5
        ref_blocks = [v for k, v in inter.items() if 'residual' in k]
        got = [m.layer_output(i, 2).cpu().numpy() for i, l in enumerate(plan.layers)
               if l.block.startswith('residual') and l.name.endswith('conv1')]
        assert len(got) == len(ref_blocks) == 5
        for g, r in zip(got, ref_blocks):
            assert np.abs(g - r).max() / max(1.0, np.abs(r).max()) < 1e-4


def test_expand0_ksplit_and_four_wave_forms_match_oracle():
    """expand_0 (the 3x3 s2 transposed 128 -> 32 conv, conv_lite.hip) runs its K-split form (8 waves, LDS-DMA weights)
    while its LDS with the prologue table of the batch fits, and the four-wave form above that (here B = 12). Both
    against float64: the same two images repeated to B = 2 and B = 12 (instance norm is per image)."""
    _need_gpu()
    from oracle import numpy_ref as R
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    ins, outs, br, bf = (32, 64, 17), (32, 64, 3), 8, 128
    plan = network_plan(ins, outs, br, bf)
    w = init_weights(plan, seed=2)
    sp = synthetic_style_params(2, 1, plan.num_style_params, plan, seed=1)
    x = np.random.default_rng(0).random((2,) + ins).astype(np.float32)
    ref, inter = R.transfer_forward(x, sp, w, ins, outs, br, bf, return_intermediates=True)
    names = [l.name for l in plan.layers]
    e0 = names.index('expand_0')
    r_e0 = [v for k, v in inter.items() if k.endswith('_expand')][0]   # the first expand block's CIN + ReLU output
    m, _ = create_style_transfer_model(ins, outs, br, bf, 1, weights=w, max_batch=12, precision="winograd_bf16x6")
    for B in (2, 12):
        k = B // 2
        inp = {'content': torch.from_numpy(np.tile(x, (k, 1, 1, 1))).cuda(),
               'style_params': torch.from_numpy(np.tile(sp, (k, 1, 1))).cuda()}
        y = m(inp).cpu().numpy()
        g = m.layer_output(e0, B).cpu().numpy()
        for j in range(k):
            assert np.abs(y[2 * j:2 * j + 2] - ref).max() < OUT_TOL, (B, j)
            gj = g[2 * j:2 * j + 2]
            assert gj.shape == r_e0.shape and np.abs(gj - r_e0).max() / max(1.0, np.abs(r_e0).max()) < 1e-4, (B, j)


@pytest.mark.parametrize("cin", [3, 12, 17])
def test_start_conv_f3_channel_chunks_match_oracle(cin):
    """wino9f3 (the inference start conv on F(3x3, 3x3) tiles) with 1, 2 and 3 input-channel chunks (cin <= 8: chunk A
    only; <= 16: A and B; 17: A, B and the channel-16 K-step) at sizes that leave partial 24 x 24 blocks, against the
    float64 oracle (ReLU -> BN -> ReLU output, 1e-5 of the output range), deterministic."""
    _need_gpu()
    from oracle import numpy_ref as R
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    ins, outs, br, bf = (52, 100, cin), (52, 100, 3), 13, 128
    plan = network_plan(ins, outs, br, bf)
    w = init_weights(plan, seed=4)
    sp = synthetic_style_params(2, 1, plan.num_style_params, plan, seed=2)
    x = np.random.default_rng(7).random((2,) + ins).astype(np.float32)
    _, inter = R.transfer_forward(x, sp, w, ins, outs, br, bf, return_intermediates=True)
    r0 = list(inter.values())[0]
    m, _ = create_style_transfer_model(ins, outs, br, bf, 1, weights=w, max_batch=2, precision="winograd_bf16x6")
    assert m.layer_kernel_id(0) == 205
    inp = {'content': torch.from_numpy(x).cuda(), 'style_params': torch.from_numpy(sp).cuda()}
    m(inp)
    g0 = m.layer_output(0, 2).cpu().numpy()
    rel = float(np.abs(g0 - r0).max() / max(1.0, np.abs(r0).max()))
    assert g0.shape == r0.shape and rel < 1e-5, rel
    m(inp)
    assert np.array_equal(g0, m.layer_output(0, 2).cpu().numpy()), "start conv is not deterministic"


@pytest.mark.parametrize("precision", list(WINO_MODES))
def test_winograd_full_size_matches_torch_oracle(precision):
    _need_gpu()
    from oracle.torch_ref import TorchTransfer
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    ws = init_weights(plan, seed=2)
    model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                           weights=ws, max_batch=1, precision=precision)
    x = np.random.default_rng(0).random((1,) + ins).astype(np.float32)
    sp = synthetic_style_params(1, 1, P, plan, seed=1)
    y = model({'content': torch.from_numpy(x).cuda(), 'style_params': torch.from_numpy(sp).cuda()}).cpu().numpy()
    ref = TorchTransfer(ws, ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)(x, sp)
    err = float(np.abs(y - ref).max())
    import json
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f'{precision}_parity.json'), 'w') as f:
        json.dump({'max_abs_full_size': err}, f)
    assert err < OUT_TOL, err


def test_apply_style_weights_kat_on_gpu():
    """The reference's only numeric known answer, styleTransferTest.py:28-49 (``_apply_style_weights``,
    two styles, vertical-gradient weights), through the device blend formula the conv prologues use.
    The KAT's weights satisfy w0 == 1 - w1 exactly (as the model completes them, styleTransfer.py:297-302),
    and every value is a small dyadic rational, so the f32 result is exact: assert_almost_equal(decimal=7)."""
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import apply_style_weights
    d = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'apply_style_weights_kat.npz'))
    w, p = d['style_weights'], d['style_params']
    assert np.array_equal(w[..., 0], (1.0 - w[..., 1]).astype(np.float32))
    got = apply_style_weights(torch.from_numpy(w).cuda(), torch.from_numpy(p).cuda()).cpu().numpy()
    assert got.shape == (2, 10, 20, 6)                                      # expected_shape
    np.testing.assert_almost_equal(got, d['expected'])
    # S != 2: the reference returns the params unblended
    p3 = torch.ones((2, 1, 3, 6), device='cuda')
    assert apply_style_weights(torch.zeros((2, 10, 20, 3), device='cuda'), p3) is p3


def test_bf16_inference_needs_explicit_opt_in():
    """Plain bf16 operands miss the 1e-3 fp32 parity bar: the factory refuses it by default."""
    _need_gpu()
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    d, ws, ins, outs, bres, bf = _load_fixture("transfer_small.npz")
    with pytest.raises(ValueError, match="allow_reduced_precision"):
        create_style_transfer_model(ins, outs, bres, bf, 1, weights=ws, max_batch=2, precision="bf16")


@pytest.mark.gpu
def test_two_networks_on_two_streams_are_bitwise_their_lone_runs():
    """Co-residency: two full-size networks (480x960x17, the headline precision) launched on two streams at
    once give bitwise the outputs each gives alone (tools/concurrent_infer_check.py, profiles/r06/r06bo)."""
    _need_gpu()
    import bench
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    nets = []
    for k in range(2):
        model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                               weights=init_weights(plan, seed=3 + k), max_batch=1,
                                               precision=bench.DEFAULT_PRECISION)
        rng = np.random.default_rng(100 + k)
        inp = {'content': torch.from_numpy(rng.random((1,) + ins, dtype=np.float32)).cuda(),
               'style_params': torch.from_numpy(synthetic_style_params(1, 1, P, plan, seed=7 + k)).cuda()}
        nets.append((model, inp, torch.empty((1,) + outs, device='cuda')))
    refs = []
    for model, inp, out in nets:
        model(inp, out=out)
        torch.cuda.synchronize()
        refs.append(out.clone())
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for _ in range(5):
        for (model, inp, out), s in zip(nets, streams):
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                model(inp, out=out)
        torch.cuda.synchronize()
        for (_, _, out), ref in zip(nets, refs):
            assert torch.equal(out, ref), "a network's output changed while another ran beside it"
