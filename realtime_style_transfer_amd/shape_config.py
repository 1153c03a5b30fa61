"""ShapeConfig — drop-in mirror of the reference's config object.

Follows ``realtime_style_transfer/shape_config.py:4-84`` attribute for attribute:
``input_shape``/``output_shape``/``image_shape``/``channels``/``num_channels``/
``num_styles``/``bottleneck_res_y``/``bottleneck_num_filters``/
``style_feature_extractor_type``/``with_depth_loss``, ``from_spec`` (:33-48) and the
G-buffer channel table (:54-73).

One addition the reference lacks: ``ShapeConfig.explicit(...)`` accepts an arbitrary
H x W (the reference only supports the 1:2 aspect, ``shape_config.py:14``), which
``create_style_transfer_model`` itself already allows (``styleTransfer.py:213``).
"""
from __future__ import annotations

import json


class StyleFeatureExtractor:
    """Mirror of ``models/stylePrediction.py:19-22`` (string enum)."""
    DUMMY = 'DUMMY'
    EFFICIENT_NET = 'EFFICIENT_NET'
    MOBILE_NET = 'MOBILE_NET'


class ShapeConfig:
    def __init__(self, num_styles=1, hdr=True, bottleneck_res_y=120, bottleneck_num_filters=128,
                 resolution_divider=2, num_channels=18):
        # shape_config.py:5-30
        self.bottleneck_res_y = bottleneck_res_y
        self.bottleneck_num_filters = bottleneck_num_filters
        self.num_styles = num_styles
        self.channels = self._get_channels_from_number(num_channels)

        num_channels = sum(c[1] for c in self.channels)
        self.num_channels = num_channels
        input_dimensions = (960 // resolution_divider, 1920 // resolution_divider)
        output_dimensions = (960 // resolution_divider, 1920 // resolution_divider)
        self._set_shapes(input_dimensions, output_dimensions, hdr)
        self.style_feature_extractor_type = StyleFeatureExtractor.MOBILE_NET
        self.with_depth_loss = True

    def _set_shapes(self, input_dimensions, output_dimensions, hdr):
        self.output_shape = tuple(output_dimensions) + (3,)
        self.image_shape = tuple(input_dimensions) + (3,)
        sdr_input_shape = {'content': self.image_shape,
                           'style': (self.num_styles,) + self.output_shape}
        hdr_input_shape = {'content': tuple(input_dimensions) + (self.num_channels,),
                           'style': (self.num_styles,) + self.output_shape}
        self.input_shape = hdr_input_shape if hdr else sdr_input_shape
        if self.num_styles > 1:
            self.input_shape['style_weights'] = tuple(output_dimensions) + (self.num_styles - 1,)

    @staticmethod
    def from_spec(spec: str, num_styles=1, hdr=True):
        """``rst-<res_x>-<bottleneck_res_y>-<bottleneck_filters>-<channels>`` (shape_config.py:33-48)."""
        parts = spec.split('-')
        if len(parts) != 5:
            raise ValueError(f"bad spec {spec!r}; expected rst-<res_x>-<bottleneck_y>-<filters>-<channels>")
        res_x = int(parts[1])
        bottleneck_res_y = int(parts[2])
        bottleneck_num_filters = int(parts[3])
        num_channels = int(parts[4])
        return ShapeConfig(num_styles, hdr, bottleneck_res_y, bottleneck_num_filters, 1920 // res_x,
                           num_channels)

    @staticmethod
    def explicit(input_hw, output_hw, num_channels=17, bottleneck_res_y=120, bottleneck_num_filters=128,
                 num_styles=1, hdr=True):
        """Arbitrary H x W (e.g. BASELINE config 1's 256x256x3 frame)."""
        cfg = ShapeConfig.__new__(ShapeConfig)
        cfg.bottleneck_res_y = bottleneck_res_y
        cfg.bottleneck_num_filters = bottleneck_num_filters
        cfg.num_styles = num_styles
        cfg.channels = cfg._get_channels_from_number(num_channels)
        cfg.num_channels = sum(c[1] for c in cfg.channels)
        cfg._set_shapes(tuple(input_hw), tuple(output_hw), hdr)
        cfg.style_feature_extractor_type = StyleFeatureExtractor.MOBILE_NET
        cfg.with_depth_loss = True
        return cfg

    def __str__(self):
        return json.dumps(self.__dict__, indent=4, default=str)

    @staticmethod
    def _get_channels_from_number(num_channels):
        # shape_config.py:54-73
        channels = [("FinalImage", 3)]
        if num_channels > 3:
            channels += [("BaseColor", 3)]
        if num_channels >= 18:
            channels += [("ShadowMask", 1)]
        if num_channels >= 17:
            channels += [
                ("AmbientOcclusion", 1),
                ("Metallic", 1),
                ("Specular", 1),
                ("Roughness", 1),
                ("ViewNormal", 3),
                ("SceneDepth", 1),
                ("LightingModel", 3),
            ]
        return channels

    def get_dummy_input_element(self, device=None):
        """Zero tensors shaped like the reference's dummy element (shape_config.py:75-84)."""
        import torch
        element = {name: torch.zeros((1,) + tuple(shape), dtype=torch.float32, device=device)
                   for name, shape in self.input_shape.items()}
        ground_truth_element = {
            'content': torch.zeros((1,) + self.output_shape, dtype=torch.float32, device=device),
            'style': torch.zeros((1, self.num_styles) + self.output_shape, dtype=torch.float32, device=device),
        }
        return element, ground_truth_element
