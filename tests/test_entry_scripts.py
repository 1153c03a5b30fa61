"""The model-construction calls of the reference's inference / export entry scripts, restated against the
mirror modules (CPU: everything that does not allocate on a GPU; tests/test_gpu_entry_scripts.py runs the
same sequences end to end on the device):

* predict_using_checkpoint.py:42,55-66      ShapeConfig(hdr=True, num_styles=S); StyleLossModelMobileNet;
                                            styleTransferTrainingModel.make_style_transfer_inference_model(...)
* predict_video_using_checkpoint.py:35-58   StyleLossModelMobileNet; make_style_transfer_training_model(...,
                                            make_style_loss_function(..., config.with_depth_loss))
* save_using_checkpoint.py:34-53            ShapeConfig.from_spec(spec, 1, True); the same, depth term by default

The calls are restated, not copied: the same modules, functions, positional/keyword arguments."""
import inspect

import pytest

from realtime_style_transfer_amd import (shape_config, styleLoss, stylePrediction, styleTransfer,
                                         styleTransferInferenceModel, styleTransferTrainingModel)
from realtime_style_transfer_amd.shape_config import ShapeConfig


def test_mobilenet_loss_model_constructs_and_refuses_evaluation():
    config = ShapeConfig(hdr=True, num_styles=1)
    m = styleLoss.StyleLossModelMobileNet(config.output_shape)              # predict_using_checkpoint.py:55
    assert m.input_shape == (480, 960, 3)
    # styleLoss.py:159-185: layer choice and factors
    assert m.style_layers == ['expanded_conv_2/Add', 'expanded_conv_4/Add', 'expanded_conv_5/Add',
                              'expanded_conv_7/Add']
    assert m.content_layers == ['expanded_conv_9/Add', 'expanded_conv_10/Add']
    assert (m.content_loss_factor, m.style_loss_factor, m.total_variation_loss_factor, m.depth_loss_factor) == \
        (1e-3, 1, 1e-3, 1e-4)
    with pytest.raises(NotImplementedError):
        m(None)


def test_loss_function_with_depth_term_constructs_and_refuses_evaluation():
    config = ShapeConfig(hdr=True, num_styles=1)
    assert config.with_depth_loss is True                                    # shape_config.py:30
    lm = styleLoss.StyleLossModelMobileNet(config.output_shape)
    # predict_video_using_checkpoint.py:53-57 (explicit) and save_using_checkpoint.py:49-52 (default)
    for compute_loss, model in (styleLoss.make_style_loss_function(lm, config.output_shape, config.num_styles,
                                                                   config.with_depth_loss),
                                styleLoss.make_style_loss_function(lm, config.output_shape, config.num_styles)):
        assert compute_loss.with_depth_loss and model.with_depth_loss
        with pytest.raises(NotImplementedError):
            compute_loss(None, {'content': None, 'style': None})
    with pytest.raises(ValueError):                                          # shape mismatch still checked
        styleLoss.make_style_loss_function(lm, (240, 480, 3), 1)


def test_training_module_reexports_inference_factory():
    # models/styleTransferTrainingModel.py:5, called through that module at predict_using_checkpoint.py:57
    assert styleTransferTrainingModel.make_style_transfer_inference_model is \
        styleTransferInferenceModel.make_style_transfer_inference_model


def _bind(fn, *args, **kwargs):
    inspect.signature(fn).bind(*args, **kwargs)


@pytest.mark.parametrize("num_styles", [1, 2])
def test_predict_using_checkpoint_construction_calls_bind(num_styles):
    config = ShapeConfig(hdr=True, num_styles=num_styles)                    # :42
    assert config.input_shape['content'] == (480, 960, config.num_channels)      # 18 G-buffer channels by default
    _bind(styleTransferTrainingModel.make_style_transfer_inference_model,   # :57-66
          num_styles=config.num_styles, style_predictor_factory_func=lambda n: None,
          style_transfer_factory_func=lambda: None)
    _bind(stylePrediction.create_style_prediction_model, config.input_shape['style'][1:],
          config.style_feature_extractor_type, 2662)                         # :59-61
    _bind(styleTransfer.create_style_transfer_model, config.input_shape['content'], config.output_shape,
          config.bottleneck_res_y, config.bottleneck_num_filters, config.num_styles)   # :62-65
    element = config.get_dummy_input_element()[0]                            # :67
    assert set(element) == ({'content', 'style', 'style_weights'} if num_styles > 1 else {'content', 'style'})


def test_video_and_save_construction_calls_bind():
    config = ShapeConfig.from_spec("rst-960-120-128-17", 1, True)            # save_using_checkpoint.py:35
    assert config.input_shape['content'] == (480, 960, 17)
    _bind(styleTransferTrainingModel.make_style_transfer_training_model,     # :41-53 / video :45-58
          style_predictor_factory_func=lambda n: None, style_transfer_factory_func=lambda: None,
          style_loss_func_factory_func=lambda: None)
    _bind(styleLoss.make_style_loss_function, None, config.output_shape, config.num_styles, config.with_depth_loss)
    assert config.style_feature_extractor_type == stylePrediction.StyleFeatureExtractor.MOBILE_NET
    assert shape_config.StyleFeatureExtractor.MOBILE_NET == stylePrediction.StyleFeatureExtractor.MOBILE_NET
