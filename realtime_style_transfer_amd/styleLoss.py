"""Host mirror of ``realtime_style_transfer/models/styleLoss.py`` on librst (MI355X).

* ``StyleLossModelVGG(input_shape)`` — the frozen VGG16 feature extractor with the reference's
  layer choice (style: block1_conv2, block2_conv2, block3_conv3, block4_conv3; content:
  block5_conv3) and factors (content 1e4, style 1e-3, TV 0.1, depth 1e-2) (styleLoss.py:69-109).
  keras.applications ImageNet weights cannot be downloaded here; ``weights=`` accepts the 26
  arrays of ``VGG16(include_top=False).get_weights()``; the default is a seeded He-normal init.
* ``gram_matrix(features)`` — styleLoss.py:21-37 on the f32-MFMA split-K Gram kernel.
* ``make_style_loss_function(loss_model, output_shape, num_styles, with_depth_loss)`` — returns
  ``(compute_loss, model)`` like styleLoss.py:295-369; ``compute_loss(y_pred, y_true)`` returns the
  per-image ``(B,)`` loss dict. The MiDaS depth term needs a TF-Hub download (styleLoss.py:254) and
  is not available: ``with_depth_loss=True`` (ShapeConfig's default, shape_config.py:30) is accepted
  at construction, as the reference's inference/export scripts build the loss without evaluating it
  (predict_video_using_checkpoint.py:53-57, save_using_checkpoint.py:49-52), and raises
  ``NotImplementedError`` when a loss that needs the depth term is computed.
* ``StyleLossModelMobileNet(input_shape)`` (styleLoss.py:155-193) — its layer choice and factors, so the
  scripts that construct it and never evaluate it (predict_using_checkpoint.py:55,
  predict_video_using_checkpoint.py:43, save_using_checkpoint.py:39) run; evaluating it raises
  ``NotImplementedError`` (the MobileNetV3Small loss trunk is not built: ImageNet weights are a download
  and no training entry point of the reference uses it).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

VGG16_CHANNELS = [64, 64, 128, 128, 256, 256, 256, 512, 512, 512, 512, 512, 512]
VGG16_LAYER_NAMES = ['block1_conv1', 'block1_conv2', 'block2_conv1', 'block2_conv2', 'block3_conv1',
                     'block3_conv2', 'block3_conv3', 'block4_conv1', 'block4_conv2', 'block4_conv3',
                     'block5_conv1', 'block5_conv2', 'block5_conv3']


def init_vgg16_weights(seed: int = 3) -> List[np.ndarray]:
    """Seeded stand-in for the ImageNet VGG16 trunk: He-normal kernels, small biases (Keras order)."""
    rng = np.random.default_rng(seed)
    out, cin = [], 3
    for c in VGG16_CHANNELS:
        out.append(rng.normal(0.0, np.sqrt(2.0 / (9 * cin)), size=(3, 3, cin, c)).astype(np.float32))
        out.append(rng.normal(0.0, 0.01, size=(c,)).astype(np.float32))
        cin = c
    return out


def vgg_weight_dict(weights: Sequence[np.ndarray]) -> Dict[str, Tuple[np.ndarray, np.ndarray]]:
    return {n: (weights[2 * i], weights[2 * i + 1]) for i, n in enumerate(VGG16_LAYER_NAMES)}


class StyleLossModelVGG:
    """styleLoss.py:69-109 on librst."""

    def __init__(self, input_shape, weights: Optional[Sequence[np.ndarray]] = None, seed: int = 3,
                 max_batch: int = 4, device=None, precision: Optional[str] = None):
        """precision: arithmetic of the VGG16 3x3 convs with Cin % 32 == 0 — "fp32" (f32 MFMA),
        "bf16x6" (exact 3-piece bf16 split, fp32-level products), "bf16x3" (2-piece split) or "bf16" (bf16
        operands, fp32 accumulation: Keras mixed_bfloat16). None: from the global policy
        (``mixed_precision.set_global_policy``, train_network.py:26) — "fp32" by default, "bf16" under
        'mixed_bfloat16'."""
        if precision is None:
            from .mixed_precision import loss_network_precision
            precision = loss_network_precision()
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {list(_lib.PRECISIONS)}")
        self.precision = precision
        self.style_layers = ['block1_conv2', 'block2_conv2', 'block3_conv3', 'block4_conv3']
        self.content_layers = ['block5_conv3']
        self.num_style_layers = len(self.style_layers)
        self.content_loss_factor = 1e4
        self.style_loss_factor = 1e-3
        self.total_variation_loss_factor = 1e-1
        self.depth_loss_factor = 1e-2
        self.trainable = False
        self.input_shape = tuple(int(v) for v in input_shape)
        self.max_batch = int(max_batch)
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.weights = [np.ascontiguousarray(w, np.float32) for w in (weights if weights is not None
                                                                       else init_vgg16_weights(seed))]
        lib = _lib.load()
        flat = np.concatenate([w.reshape(-1) for w in self.weights])
        if flat.size != lib.rst_loss_num_weights():
            raise ValueError(f"VGG16 trunk expects {lib.rst_loss_num_weights()} weights, got {flat.size}")
        shape = _lib.RstLossShape(self.input_shape[0], self.input_shape[1], self.max_batch,
                                  self.content_loss_factor, self.style_loss_factor, self.total_variation_loss_factor,
                                  _lib.PRECISIONS[self.precision])
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.rst_loss_create(ctypes.byref(shape), flat.ctypes.data, flat.size, ctypes.byref(h)))
        self._handle = h

    def __del__(self):
        try:
            if getattr(self, '_handle', None) is not None:
                _lib.load().rst_loss_destroy(self._handle)
                self._handle = None
        except Exception:
            pass

    def losses(self, prediction: torch.Tensor, gt_content: torch.Tensor, gt_style: torch.Tensor) -> torch.Tensor:
        """-> (B, 4) [loss, feature_loss, style_loss, total_variation_loss]."""
        if gt_style.dim() == 5:
            if gt_style.shape[1] != 1:   # styleLoss.py:311-312
                raise ValueError(f"Loss model does not support multiple styles. Found {gt_style.shape[1]}")
            gt_style = gt_style[:, 0]
        B = prediction.shape[0]
        for t in (prediction, gt_content, gt_style):
            if tuple(t.shape) != (B,) + self.input_shape:
                raise ValueError(f"expected (B,{self.input_shape}) images, got {tuple(t.shape)}")
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch={self.max_batch}")
        prediction, gt_content, gt_style = (t.contiguous() for t in (prediction, gt_content, gt_style))
        out = torch.empty((B, 4), dtype=torch.float32, device=prediction.device)
        _lib.check(_lib.load().rst_loss_forward(self._handle, _lib.dev_ptr(prediction), _lib.dev_ptr(gt_content),
                                                _lib.dev_ptr(gt_style), B, _lib.dev_ptr(out), _lib.stream_ptr()))
        return out

    def feature(self, layer: str, batch: int) -> torch.Tensor:
        """Debug: a VGG16 conv output of the most recent prediction run."""
        idx = VGG16_LAYER_NAMES.index(layer)
        H, W = self.input_shape[:2]
        div = 2 ** sum(1 for i in (1, 3, 6, 9) if i < idx)
        t = torch.empty((batch, H // div, W // div, VGG16_CHANNELS[idx]), dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().rst_loss_copy_feature(self._handle, idx, _lib.dev_ptr(t), t.numel(), batch,
                                                     _lib.stream_ptr()))
        return t


class StyleLossModelMobileNet:
    """styleLoss.py:155-193: constructible with the reference's layer names and factors; not evaluable."""

    def __init__(self, input_shape, name: str = "StyleLossModelMobileNet"):
        self.name = name
        self.input_shape = tuple(int(v) for v in input_shape)
        self.style_layers = ['expanded_conv_2/Add', 'expanded_conv_4/Add', 'expanded_conv_5/Add',
                             'expanded_conv_7/Add']
        self.content_layers = ['expanded_conv_9/Add', 'expanded_conv_10/Add']
        self.num_style_layers = len(self.style_layers)
        self.content_loss_factor = 1e-3
        self.style_loss_factor = 1
        self.total_variation_loss_factor = 1e-3
        self.depth_loss_factor = 1e-4
        self.trainable = False

    def _unavailable(self, *args, **kwargs):
        raise NotImplementedError(
            "StyleLossModelMobileNet is construct-only on MI355X: the MobileNetV3Small loss trunk (ImageNet weights, a "
            "network download) is not built; train with StyleLossModelVGG as train_network.py:85 does")

    __call__ = _unavailable
    losses = _unavailable


def gram_matrix(input_tensor: torch.Tensor) -> torch.Tensor:
    """styleLoss.py:21-37: einsum('bijc,bijd->bcd') / (H*W) on the device (channels % 64 == 0)."""
    lib = _lib.load()
    B, H, W, C = input_tensor.shape
    x = input_tensor.contiguous()
    out = torch.empty((B, C, C), dtype=torch.float32, device=x.device)
    ws = torch.empty(lib.rst_gram_workspace_size(B, H * W, C), dtype=torch.uint8, device=x.device)
    _lib.check(lib.rst_gram(_lib.dev_ptr(x), B, H * W, C, _lib.dev_ptr(out), int(ws.data_ptr()), _lib.stream_ptr()))
    return out


DEPTH_LOSS_UNAVAILABLE = ("the depth loss term needs the TF-Hub MiDaS model (styleLoss.py:250-288), a network "
                          "download that is not available here; build the loss with with_depth_loss=False")


class StyleLoss:
    """The Keras ``StyleLoss`` model make_style_loss_function returns (styleLoss.py:360-361): called with
    ``(inputs, ground_truth)`` or ``{'prediction', 'ground_truth'}`` it returns the per-image loss dict."""

    def __init__(self, feature_model, with_depth_loss: bool):
        self.feature_model = feature_model
        self.with_depth_loss = bool(with_depth_loss)
        self.trainable = False
        self.name = "StyleLoss"

    def compute(self, y_pred: torch.Tensor, y_true: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        if self.with_depth_loss:
            raise NotImplementedError(DEPTH_LOSS_UNAVAILABLE)
        t = self.feature_model.losses(y_pred, y_true['content'], y_true['style'])
        return {"loss": t[:, 0], "feature_loss": t[:, 1], "style_loss": t[:, 2], "total_variation_loss": t[:, 3]}

    def __call__(self, inputs):
        if isinstance(inputs, dict):
            return self.compute(inputs['prediction'], inputs['ground_truth'])
        raise NotImplementedError("StyleLoss takes {'prediction', 'ground_truth'}; the (inputs, ground_truth) form of "
                                  "StyleTransferModels.loss_model runs the inference model first — use "
                                  "StyleTransferTrainingModel.train_step")


def make_style_loss_function(loss_feature_extractor_model, output_shape, num_styles, with_depth_loss=True):
    """styleLoss.py:295-369 -> (compute_loss, model). The MiDaS depth term is not available: a loss built with
    ``with_depth_loss=True`` constructs, and raises NotImplementedError when it is computed."""
    if tuple(output_shape) != tuple(loss_feature_extractor_model.input_shape):
        raise ValueError(f"output_shape {output_shape} != loss model input {loss_feature_extractor_model.input_shape}")
    model = StyleLoss(loss_feature_extractor_model, with_depth_loss)

    def compute_loss(y_pred: torch.Tensor, y_true: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        return model.compute(y_pred, y_true)

    compute_loss.with_depth_loss = model.with_depth_loss
    return compute_loss, model
