"""Host mirror of ``realtime_style_transfer/models/styleTransferInferenceModel.py`` on librst.

``make_style_transfer_inference_model(num_styles, style_predictor_factory_func,
style_transfer_factory_func, name)`` keeps the reference signature (:9-12) and return value: an
object with ``.inputs``, ``.inference``, ``.transfer`` and ``.style_predictor`` (:41-48).

``inference(inputs)`` runs, on the GPU and asynchronously on the current stream:
the style predictor once per style image (:23-26; the (B, S, H, W, 3) stack goes to the predictor
as B*S images, so its (B*S, P) output already is the stacked (B, S, P) style-parameter tensor of
:28) and then the transfer network on ``{'content', 'style_params'[, 'style_weights']}`` (:30-37).
"""
from __future__ import annotations

import logging
from typing import Callable, Dict, Optional

import torch

from . import _lib

log = logging.getLogger(__name__)


class StyleTransferInference:
    """``tf.keras.Model(inputs={'content', 'style'[, 'style_weights']}, outputs=stylized_image)``."""

    def __init__(self, transfer, style_predictor, num_styles: int, name: str):
        self.transfer = transfer
        self.style_predictor = style_predictor
        self.num_styles = int(num_styles)
        self.name = name
        if tuple(style_predictor.output_shape[1:]) != (transfer.num_style_parameters,):
            raise ValueError(f"style predictor emits {style_predictor.output_shape[1:]} parameters, the transfer "
                             f"network takes {transfer.num_style_parameters}")

    @property
    def input(self) -> Dict[str, tuple]:
        spec = {'content': (None,) + self.transfer.input_shape,
                'style': (None, self.num_styles) + self.style_predictor.input_shape}
        if self.num_styles > 1:
            spec['style_weights'] = self.transfer.input['style_weights']
        return spec

    @property
    def output_shape(self):
        return (None,) + self.transfer.output_shape

    def predict_style_params(self, style: torch.Tensor) -> torch.Tensor:
        """(B, S, H, W, 3) style images -> (B, S, P) style parameters (:23-28)."""
        if style.dim() != 5 or style.shape[1] != self.num_styles:
            raise ValueError(f"style must be (B,{self.num_styles},H,W,C), got {tuple(style.shape)}")
        B, S = style.shape[:2]
        flat = style.reshape((B * S,) + tuple(style.shape[2:]))
        return self.style_predictor(flat).view(B, S, -1)

    def compile(self, run_eagerly=False, **kwargs):
        """Keras Model.compile: nothing to compile (kernels built ahead of time)."""

    trainable = False

    def __call__(self, inputs: Dict[str, torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
        sp = self.predict_style_params(_lib.as_device(inputs['style'], self.transfer.device))
        transfer_input = {'content': inputs['content'], 'style_params': sp}
        if 'style_weights' in inputs:
            transfer_input['style_weights'] = inputs['style_weights']
        return self.transfer(transfer_input, out=out)

    def predict(self, inputs: Dict[str, torch.Tensor], batch_size=None, verbose=0):
        """Keras Model.predict: the output as a host numpy array (predict_using_checkpoint.py:99)."""
        return self(inputs).cpu().numpy()

    # ------------------------------------------------------------------ checkpoints
    # The functional model's weighted layers are the two sub-models: the style predictor first
    # (layer_with_weights-0; its output feeds the stack, :23-26) and the transfer network (layer_with_weights-1,
    # :37), each keyed by its own layer tree below that prefix (tf_checkpoint.LayerTree).
    def _checkpoint_parts(self):
        return self.style_predictor._checkpoint_parts("layer_with_weights-0/") + \
            self.transfer._checkpoint_parts("layer_with_weights-1/")

    def _checkpoint_tensors(self):
        from .tf_checkpoint import parts_tensors
        return parts_tensors(self._checkpoint_parts())

    def _restore_tensors(self, tensors):
        from .tf_checkpoint import restore_parts
        return restore_parts(self._checkpoint_parts(), tensors)

    def load_weights(self, filepath):
        """``inference.load_weights(filepath)`` (predict_using_checkpoint.py:84-85) -> CheckpointLoadStatus
        (``assert_nontrivial_match()``): a checkpoint of this model, or of the training model (same layers;
        its optimizer state is left unused)."""
        from .tf_checkpoint import load_weights
        return load_weights(self, filepath)

    def save_weights(self, filepath) -> None:
        from .tf_checkpoint import save_weights
        save_weights(self, filepath)


def make_style_transfer_inference_model(num_styles, style_predictor_factory_func: Callable[[int], object],
                                        style_transfer_factory_func: Callable[[], tuple],
                                        name="StyleTransferInferenceModel"):
    """Drop-in for styleTransferInferenceModel.make_style_transfer_inference_model (:9-48)."""
    style_transfer_model, num_style_parameters = style_transfer_factory_func()
    style_predictor = style_predictor_factory_func(num_style_parameters)
    model = StyleTransferInference(style_transfer_model, style_predictor, num_styles, name)

    class StyleTransferModels:
        def __init__(self):
            self.inputs = model.input
            self.inference = model
            self.transfer = style_transfer_model
            self.style_predictor = style_predictor

    return StyleTransferModels()
