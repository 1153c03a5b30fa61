"""The reference's inference / export entry scripts' model-building sequences, restated against the mirror
modules and run on the device at the scripts' own configuration (ShapeConfig(hdr=True): 480x960x18 G-buffer
frames, MOBILE_NET style predictor, StyleLossModelMobileNet, the depth term on by default). No checkpoint
ships with the reference, so the seeded initial weights stand in for load_weights / Checkpoint.restore.

* predict_using_checkpoint.py:42-99   one and two styles: build the inference model, setup_model (trainable,
                                      compile), call it on the dummy element, predict -> uint8 export
* predict_video_using_checkpoint.py:35-98   training model with the MobileNet loss and the depth term:
                                      training(element), style_predictor(style), transfer.predict per frame
* save_using_checkpoint.py:34-71      ShapeConfig.from_spec; training(element); loss_model((x, y)) raises
                                      (construct-only loss); train_step raises
"""
import numpy as np
import pytest
import torch

from realtime_style_transfer_amd import styleLoss, stylePrediction, styleTransfer, styleTransferTrainingModel
from realtime_style_transfer_amd.shape_config import ShapeConfig

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _setup_model(model):                     # predict_*_using_checkpoint.py setup_model
    model.trainable = False
    model.compile(run_eagerly=False)


@pytest.mark.parametrize("num_styles", [1, 2])
def test_predict_using_checkpoint_sequence(num_styles):
    _need_gpu()
    config = ShapeConfig(hdr=True, num_styles=num_styles)
    style_loss_model = styleLoss.StyleLossModelMobileNet(config.output_shape)
    m = styleTransferTrainingModel.make_style_transfer_inference_model(
        num_styles=config.num_styles,
        style_predictor_factory_func=lambda num_top_parameters: stylePrediction.create_style_prediction_model(
            config.input_shape['style'][1:], config.style_feature_extractor_type, num_top_parameters),
        style_transfer_factory_func=lambda: styleTransfer.create_style_transfer_model(
            config.input_shape['content'], config.output_shape, config.bottleneck_res_y,
            config.bottleneck_num_filters, config.num_styles))
    element = config.get_dummy_input_element()[0]          # host tensors, as the reference's
    for model in (m.style_predictor, m.transfer, m.inference):
        _setup_model(model)
    m.inference(element)
    rng = np.random.default_rng(0)
    element = {'style': rng.random((1, num_styles) + config.output_shape, dtype=np.float32),
               'content': rng.random((1,) + config.input_shape['content'], dtype=np.float32)}
    if 'style_weights' in config.input_shape:
        element['style_weights'] = rng.random((1,) + config.input_shape['style_weights'], dtype=np.float32)
    predicted_frame = np.uint8(m.inference.predict(element).squeeze() * 255)
    assert predicted_frame.shape == config.output_shape and predicted_frame.dtype == np.uint8
    assert style_loss_model.input_shape == config.output_shape


def test_predict_video_using_checkpoint_sequence():
    _need_gpu()
    config = ShapeConfig(hdr=True, num_styles=1)
    style_loss_model = styleLoss.StyleLossModelMobileNet(config.output_shape)
    m = styleTransferTrainingModel.make_style_transfer_training_model(
        style_predictor_factory_func=lambda num_top_parameters: stylePrediction.create_style_prediction_model(
            config.input_shape['style'][1:], config.style_feature_extractor_type, num_top_parameters),
        style_transfer_factory_func=lambda: styleTransfer.create_style_transfer_model(
            config.input_shape['content'], config.output_shape, config.bottleneck_res_y,
            config.bottleneck_num_filters, config.num_styles),
        style_loss_func_factory_func=lambda: styleLoss.make_style_loss_function(
            style_loss_model, config.output_shape, config.num_styles, config.with_depth_loss))
    element = config.get_dummy_input_element()[0]
    for model in (m.training, m.style_predictor, m.transfer):
        _setup_model(model)
    y0 = m.training(element)
    assert tuple(y0.shape) == (1,) + config.output_shape
    rng = np.random.default_rng(1)
    style_params = m.style_predictor(rng.random((1,) + config.output_shape, dtype=np.float32))
    template = {'style_params': torch.unsqueeze(style_params, 0)}      # tf.expand_dims(style_params, 0)
    frames = []
    for i in range(2):
        element = dict(template)
        element['content'] = torch.from_numpy(rng.random((1,) + config.input_shape['content'], dtype=np.float32))
        predicted_frame = m.transfer.predict(element, batch_size=1, verbose=0)
        frames.append((np.squeeze(predicted_frame) * 255).astype(int))
    assert all(f.shape == config.output_shape for f in frames) and not np.array_equal(frames[0], frames[1])
    # the training model wraps the inference graph: same output as the predictor -> transfer chain
    x = {'content': element['content'], 'style': torch.zeros((1, 1) + config.output_shape)}
    ref = m.transfer({'content': x['content'], 'style_params': m.style_predictor(x['style'][:, 0])[:, None]})
    assert torch.equal(m.training(x), ref)


def test_save_using_checkpoint_sequence():
    _need_gpu()
    config = ShapeConfig.from_spec("rst-960-120-128-17", 1, True)
    style_loss_model = styleLoss.StyleLossModelMobileNet(config.output_shape)
    m = styleTransferTrainingModel.make_style_transfer_training_model(
        style_predictor_factory_func=lambda num_top_parameters: stylePrediction.create_style_prediction_model(
            config.input_shape['style'][1:], config.style_feature_extractor_type, num_top_parameters),
        style_transfer_factory_func=lambda: styleTransfer.create_style_transfer_model(
            config.input_shape['content'], config.output_shape, config.bottleneck_res_y,
            config.bottleneck_num_filters, config.num_styles),
        style_loss_func_factory_func=lambda: styleLoss.make_style_loss_function(
            style_loss_model, config.output_shape, config.num_styles))
    element = {name: torch.zeros((1,) + shape) for name, shape in config.input_shape.items()}
    ground_truth_element = {'content': torch.zeros((1,) + config.output_shape),
                            'style': torch.zeros((1, config.num_styles) + config.output_shape)}
    out = m.training(element)
    assert tuple(out.shape) == (1,) + config.output_shape
    with pytest.raises(NotImplementedError):
        m.loss_model((element, ground_truth_element))
    with pytest.raises(NotImplementedError):
        m.training.train_step(element, ground_truth_element)
    assert len(m.transfer.get_weights()) == len(m.training.get_weights())
