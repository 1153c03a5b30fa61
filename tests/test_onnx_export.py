"""ONNX export (save_using_checkpoint.py:90-103): the transfer net and the style predictor
written as ONNX ModelProto files, read back with the repo's own protobuf reader, executed with a numpy
evaluator of the emitted operators (tests/onnx_runner.py) and compared with the float64 oracle.

Loading the files in onnxruntime / tf2onnx-produced graphs is *parity unpinned*: neither onnx nor
onnxruntime is installed here; the checks pin the graph semantics and the interface names (``content``,
``style_params``; ``style``) the Unreal plugin binds.
"""
import numpy as np
import pytest

from oracle import numpy_ref as R
from oracle import predictor_ref as PR
from realtime_style_transfer_amd import onnx_export as OX
from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
from realtime_style_transfer_amd.stylePrediction import init_predictor_weights, predictor_weight_spec
from tests import onnx_runner


def test_protobuf_varint_round_trip():
    for v in (0, 1, 127, 128, 300, 2 ** 31, 2 ** 63 - 1):
        b = OX._varint(v)
        assert OX._read_varint(b, 0) == (v, len(b))
    assert OX._signed(OX._read_varint(OX._varint(-1), 0)[0]) == -1


@pytest.mark.parametrize("ins,outs,br,bf", [((32, 64, 17), (32, 64, 3), 8, 8), ((36, 52, 5), (72, 104, 3), 9, 8)])
def test_transfer_onnx_matches_oracle(tmp_path, ins, outs, br, bf):
    plan = network_plan(ins, outs, br, bf)
    ws = init_weights(plan, seed=4)
    paths = OX.save_onnx(tmp_path / "model", plan, ws)
    assert paths['transfer'].name == "model.transfer.onnx"
    m = OX.read_model(paths['transfer'])
    assert m['ir_version'] == OX.IR_VERSION and m['opset'][''] == OX.OPSET
    g = m['graph']
    assert [n for n, _ in g['inputs']] == ['content', 'style_params']
    assert g['inputs'][0][1] == ['N', *ins] and g['inputs'][1][1] == ['N', 1, plan.num_style_params]
    assert [n for n, _ in g['outputs']] == ['output'] and g['outputs'][0][1] == ['N', *outs]
    # every Keras weight is stored once, as float32 (permuted to OIHW / IOHW for the convs)
    floats = [v for k, v in g['initializers'].items() if v.dtype == np.float32 and '_eps_' not in k]
    assert sum(v.size for v in floats) == plan.num_weights()
    assert sorted(np.concatenate([v.ravel() for v in floats]).tolist()) == \
        sorted(np.concatenate([w.ravel() for w in ws]).tolist())
    rng = np.random.default_rng(5)
    content = rng.random((2,) + tuple(ins)).astype(np.float32)
    sp = synthetic_style_params(2, 1, plan.num_style_params, plan, seed=6)
    y = onnx_runner.run(m, {'content': content, 'style_params': sp})['output']
    ref = R.transfer_forward(content, sp, ws, ins, outs, br, bf)
    assert y.shape == ref.shape
    np.testing.assert_allclose(y, ref, rtol=0, atol=1e-9)


@pytest.mark.parametrize("ins,outs,br,bf", [((32, 64, 17), (32, 64, 3), 8, 8), ((36, 52, 5), (72, 104, 3), 9, 8)])
def test_two_style_transfer_onnx_matches_oracle(tmp_path, ins, outs, br, bf):
    """save_using_checkpoint.py:90-103 on a num_styles=2 model: inputs content, style_params (N,2,P) and
    style_weights (N,Ho,Wo,1); the weight mips and the per-pixel blend (styleTransfer.py:36-44,288-303,335-345)
    executed by the numpy evaluator match the float64 oracle."""
    plan = network_plan(ins, outs, br, bf, num_styles=2)
    ws = init_weights(plan, seed=4)
    m = OX.read_model(OX.save_onnx(tmp_path / "two", plan, ws)['transfer'])
    g = m['graph']
    assert [n for n, _ in g['inputs']] == ['content', 'style_params', 'style_weights']
    assert g['inputs'][1][1] == ['N', 2, plan.num_style_params] and g['inputs'][2][1] == ['N', *outs[:2], 1]
    rng = np.random.default_rng(9)
    content = rng.random((2,) + tuple(ins)).astype(np.float32)
    sp = synthetic_style_params(2, 2, plan.num_style_params, plan, seed=6)
    sw = rng.random((2,) + tuple(outs[:2]) + (1,)).astype(np.float32)
    y = onnx_runner.run(m, {'content': content, 'style_params': sp, 'style_weights': sw})['output']
    ref = R.transfer_forward(content, sp, ws, ins, outs, br, bf, style_weights=sw)
    assert y.shape == ref.shape
    np.testing.assert_allclose(y, ref, rtol=0, atol=1e-9)
    # the blend matters: style 1 alone differs
    ref1 = R.transfer_forward(content, sp[:, :1], ws, ins, outs, br, bf)
    assert np.abs(ref - ref1).max() > 1e-3


def test_transfer_onnx_rejects_three_styles(tmp_path):
    plan = network_plan((32, 64, 17), (32, 64, 3), 8, 8, num_styles=3)
    with pytest.raises(NotImplementedError):
        OX.transfer_graph(plan, init_weights(plan, seed=4))


def test_transfer_onnx_rejects_wrong_weights():
    plan = network_plan((32, 64, 17), (32, 64, 3), 8, 8)
    ws = init_weights(plan, seed=4)
    with pytest.raises(ValueError):
        OX.transfer_graph(plan, ws[:-1])


@pytest.mark.parametrize("extractor,hw", [("MOBILE_NET", (64, 96)), ("MOBILE_NET", (65, 97)), ("DUMMY", (60, 90))])
def test_predictor_onnx_matches_oracle(tmp_path, extractor, hw):
    ins = (hw[0], hw[1], 3)
    top = 48
    ws = init_predictor_weights(predictor_weight_spec(ins, extractor, top), seed=7, perturb=True)
    data = OX.predictor_graph(ins, extractor, ws, top, batch=2)
    m = OX.read_model(data)
    g = m['graph']
    assert [n for n, _ in g['inputs']] == ['style'] and g['inputs'][0][1] == [2, *ins]
    assert g['outputs'][0][1] == [2, top]
    style = np.random.default_rng(8).random((2,) + ins).astype(np.float32)
    y = onnx_runner.run(m, {'style': style})['style_params']
    ref = PR.style_predictor_forward(style, ws, extractor)
    assert y.shape == ref.shape == (2, top)
    np.testing.assert_allclose(y, ref, rtol=0, atol=1e-9)


def test_save_onnx_writes_both_files(tmp_path):
    plan = network_plan((32, 64, 17), (32, 64, 3), 8, 8)
    ins = (64, 96, 3)
    pw = init_predictor_weights(predictor_weight_spec(ins, "MOBILE_NET", plan.num_style_params), seed=1)
    paths = OX.save_onnx(tmp_path / "run7", plan, init_weights(plan, seed=4), ins, "MOBILE_NET", pw)
    assert paths['predictor'].name == "run7.predictor.onnx" and paths['predictor'].stat().st_size > 0
    assert OX.read_model(paths['predictor'])['graph']['outputs'][0][1] == ['N', plan.num_style_params]
