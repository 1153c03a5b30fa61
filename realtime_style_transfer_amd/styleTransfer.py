"""Host mirror of ``realtime_style_transfer/models/styleTransfer.py`` on librst (MI355X).

``create_style_transfer_model(input_shape, output_shape, bottleneck_res_y,
bottleneck_num_filters, num_styles, name)`` keeps the reference signature
(styleTransfer.py:213-214) and return value ``(model, num_style_parameters)`` (:332).
The model is called like the Keras model: ``model({'content': (B,H,W,C),
'style_params': (B,S,P)[, 'style_weights': ...]})`` -> ``(B,Ho,Wo,3)`` float32 in (0, 1),
NHWC, on the GPU. All compute runs in hand-written gfx950 kernels behind the C ABI
(include/rst.h); there is no CPU fallback.

Weights: ``get_weights()/set_weights()`` use the Keras ``model.get_weights()`` order of the
reference graph (see plan.py); the default is the seeded initialisation that mirrors the
reference initialisers (styleTransfer.py:97,146,190).
"""
from __future__ import annotations

import ctypes
import logging
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .plan import CIN_EPS, Plan, init_weights, network_plan

log = logging.getLogger(__name__)

# precision modes whose inference output misses the fp32 parity bar (opt-in only)
REDUCED_PRECISIONS = ("bf16",)


class StyleTransferModel:
    """A built transfer network resident on one GPU (one librst handle)."""

    def __init__(self, input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters, num_styles=1,
                 name="StyleTransferModel", weights: Optional[Sequence[np.ndarray]] = None, seed: int = 2,
                 max_batch: int = 8, device=None, precision: str = "winograd_bf16x6",
                 allow_reduced_precision: bool = False):
        self.name = name
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {list(_lib.PRECISIONS)}, got {precision!r}")
        if precision in REDUCED_PRECISIONS and not allow_reduced_precision:
            raise ValueError(f"precision {precision!r} computes the residual convs with bf16 operands (8 significant "
                             f"bits; ~0.1 max-abs output deviation, above the 1e-3 parity bar of an fp32 model); pass "
                             f"allow_reduced_precision=True to use it for inference")
        self.precision = precision
        self.plan: Plan = network_plan(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters,
                                       num_styles)
        self.input_shape = tuple(int(v) for v in input_shape)
        self.output_shape = tuple(int(v) for v in output_shape)
        self.num_styles = int(num_styles)
        self.num_style_parameters = self.plan.num_style_params
        self.max_batch = int(max_batch)
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self._handle = None
        self._weights = [np.ascontiguousarray(w, np.float32) for w in
                         (weights if weights is not None else init_weights(self.plan, seed))]
        self._build()

    # ------------------------------------------------------------------ lifecycle
    def _shape_struct(self) -> _lib.RstShape:
        H, W, C = self.input_shape
        return _lib.RstShape(H, W, C, self.output_shape[0], self.output_shape[1], self.plan.bottleneck_res_y,
                             self.plan.bottleneck_num_filters, self.num_styles, self.max_batch)

    def _build(self):
        lib = _lib.load()
        shapes = self.plan.weight_shapes()
        if len(self._weights) != len(shapes) or any(tuple(w.shape) != tuple(s) for w, s in zip(self._weights, shapes)):
            raise ValueError("weights do not match the network plan: expected shapes "
                             f"{shapes}, got {[w.shape for w in self._weights]}")
        flat = np.concatenate([w.reshape(-1) for w in self._weights]).astype(np.float32)
        shape = self._shape_struct()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.rst_create_ex(ctypes.byref(shape), flat.ctypes.data, flat.size,
                                         _lib.PRECISIONS[self.precision], ctypes.byref(h)))
        self._release()
        self._handle = h
        P = lib.rst_num_style_params(h)
        if P != self.num_style_parameters:
            raise RuntimeError(f"librst plan P={P} disagrees with host plan P={self.num_style_parameters}")

    def _release(self):
        if self._handle is not None:
            _lib.load().rst_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    # ------------------------------------------------------------------ Keras-like API
    def get_weights(self) -> List[np.ndarray]:
        return [w.copy() for w in self._weights]

    def set_weights(self, weights: Sequence[np.ndarray]):
        self._weights = [np.ascontiguousarray(w, np.float32) for w in weights]
        self._build()

    def compile(self, run_eagerly=False, **kwargs):
        """Keras Model.compile (predict_*_using_checkpoint.py setup_model): nothing to compile — the kernels are
        built ahead of time and the forward is graph-capturable."""

    trainable = False

    def keras_layer_attributes(self) -> List[List[str]]:
        return transfer_layer_attributes(self.plan)

    def _checkpoint_parts(self, prefix: str = ""):
        from .tf_checkpoint import LayerTree, _Part
        return [_Part(prefix, LayerTree(self.keras_layer_attributes()), self.get_weights, self.set_weights,
                      [tuple(w.shape) for w in self._weights])]

    def _checkpoint_tensors(self):
        from .tf_checkpoint import parts_tensors
        return parts_tensors(self._checkpoint_parts())

    def _restore_tensors(self, tensors):
        from .tf_checkpoint import restore_parts
        return restore_parts(self._checkpoint_parts(), tensors)

    def save_weights(self, filepath) -> None:
        """Model.save_weights(filepath) in TF checkpoint format (tracing/checkpoint.py:37)."""
        from .tf_checkpoint import save_weights
        save_weights(self, filepath)

    def load_weights(self, filepath, model_path: str = ""):
        """Model.load_weights(filepath) (predict_using_checkpoint.py:84) from a TF checkpoint prefix or
        directory -> a CheckpointLoadStatus (``assert_nontrivial_match()``, ``assert_consumed()``).
        ``model_path`` selects this model's subtree inside a larger model's checkpoint (the inference model
        keeps it under ``"layer_with_weights-1"``)."""
        from .tf_checkpoint import read_checkpoint, restore_parts
        pre = model_path.rstrip('/') + '/' if model_path else ''
        return restore_parts(self._checkpoint_parts(pre), read_checkpoint(filepath))

    @property
    def input(self) -> Dict[str, tuple]:
        spec = {'content': (None,) + self.input_shape, 'style_params': (None, self.num_styles,
                                                                           self.num_style_parameters)}
        if self.num_styles > 1:
            spec['style_weights'] = (None, self.output_shape[0], self.output_shape[1], self.num_styles - 1)
        return spec

    def _check_inputs(self, content: torch.Tensor, style_params: torch.Tensor):
        if content.dim() != 4 or tuple(content.shape[1:]) != self.input_shape:
            raise ValueError(f"content must be (B,{','.join(map(str, self.input_shape))}), got {tuple(content.shape)}")
        B = content.shape[0]
        if style_params.dim() == 2:
            style_params = style_params.unsqueeze(1)
        if tuple(style_params.shape) != (B, self.num_styles, self.num_style_parameters):
            raise ValueError(f"style_params must be (B,{self.num_styles},{self.num_style_parameters}), "
                             f"got {tuple(style_params.shape)}")
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch={self.max_batch} chosen at build time")
        return style_params

    def __call__(self, inputs: Dict[str, torch.Tensor], out: Optional[torch.Tensor] = None,
                 stream=None) -> torch.Tensor:
        content = _lib.as_device(inputs['content'], self.device)
        style_params = self._check_inputs(content, _lib.as_device(inputs['style_params'], self.device))
        B = content.shape[0]
        sw = inputs.get('style_weights')
        if sw is not None:
            sw = _lib.as_device(sw, self.device)
        if sw is not None and self.num_styles == 1:
            raise ValueError("style_weights given but num_styles == 1")
        if self.num_styles > 1:
            # styleTransfer.py:290-296: (B, out_h, out_w, S-1), the first style's weight is 1 - sum
            want = (B, self.output_shape[0], self.output_shape[1], self.num_styles - 1)
            if sw is None or tuple(sw.shape) != want:
                raise ValueError(f"style_weights must be {want} for num_styles={self.num_styles}, got "
                                 f"{None if sw is None else tuple(sw.shape)}")
            sw = sw.contiguous()
        content = content.contiguous()
        style_params = style_params.contiguous()
        if out is None:
            out = torch.empty((B,) + self.output_shape, dtype=torch.float32, device=content.device)
        _lib.check(_lib.load().rst_forward(self._handle, _lib.dev_ptr(content), _lib.dev_ptr(style_params),
                                           None if sw is None else _lib.dev_ptr(sw), _lib.dev_ptr(out), B,
                                           _lib.stream_ptr(stream)))
        return out

    def predict(self, inputs: Dict[str, torch.Tensor], batch_size=None, verbose=0) -> np.ndarray:
        """Keras Model.predict: the output as a host numpy array (predict_video_using_checkpoint.py:96-98)."""
        return self(inputs).cpu().numpy()

    # ------------------------------------------------------------------ profiling
    def profile_begin(self, max_steps: int):
        _lib.check(_lib.load().rst_profile_begin(self._handle, int(max_steps)))

    def profile_end(self):
        """-> (conv_ms[L], layer_ms[L], steps): summed per-layer HIP-event times."""
        lib = _lib.load()
        L = self.num_layers()
        conv = (ctypes.c_float * L)()
        lay = (ctypes.c_float * L)()
        steps = ctypes.c_int()
        _lib.check(lib.rst_profile_end(self._handle, conv, lay, ctypes.byref(steps)))
        return list(conv), list(lay), steps.value

    def timeline_begin(self):
        """Per-layer kernel end stamps for the forwards issued afterwards, eager or captured into a hipGraph
        (rst_timeline_begin: the residual convs and the narrow convs stamp; a measurement aid)."""
        _lib.check(_lib.load().rst_timeline_begin(self._handle))

    def timeline_read(self) -> np.ndarray:
        """-> end[L] in us after the first stamped layer's end (NaN where the layer's kernel does not stamp) of the
        most recent forward; end[k] - end[k-1] is layer k's share of a back-to-back graph replay."""
        L = self.num_layers()
        buf = (ctypes.c_double * L)()
        _lib.check(_lib.load().rst_timeline_read(self._handle, buf, L))
        a = np.array(list(buf))
        a[a < 0] = np.nan
        return a

    def timeline_end(self):
        _lib.check(_lib.load().rst_timeline_end(self._handle))

    def layer_kernel_id(self, idx: int) -> int:
        return _lib.load().rst_layer_kernel_id(self._handle, idx)

    # ------------------------------------------------------------------ debugging
    def num_layers(self) -> int:
        return _lib.load().rst_num_layers(self._handle)

    def layer_output(self, idx: int, batch: int) -> torch.Tensor:
        """Most recent output of conv layer ``idx`` as its reference block emits it."""
        lib = _lib.load()
        hwc = (ctypes.c_int * 3)()
        _lib.check(lib.rst_layer_output_shape(self._handle, idx, batch, hwc))
        t = torch.empty((batch, hwc[0], hwc[1], hwc[2]), dtype=torch.float32, device=self.device)
        _lib.check(lib.rst_copy_activation(self._handle, idx, _lib.dev_ptr(t), t.numel(), batch, _lib.stream_ptr()))
        return t


def transfer_layer_attributes(plan: Plan) -> List[List[str]]:
    """Variables per weighted Keras layer of the transfer network, in model order: each Conv2D /
    Conv2DTranspose owns (kernel, bias); the BatchNormalization after a contract conv (styleTransfer.py:194-203)
    is its own layer (gamma, beta, moving_mean, moving_variance); CIN owns none (its affine is an input)."""
    out = []
    for layer in plan.layers:
        out.append(["kernel", "bias"])
        if layer.norm == 'bn':
            out.append(["gamma", "beta", "moving_mean", "moving_variance"])
    return out


def create_style_transfer_model(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters, num_styles,
                                name="StyleTransferModel", **kwargs):
    """Drop-in for styleTransfer.create_style_transfer_model (styleTransfer.py:213-332)."""
    log.info(f"Using {num_styles} styles")
    model = StyleTransferModel(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters, num_styles,
                               name=name, **kwargs)
    return model, model.num_style_parameters


def apply_style_weights(style_weights: torch.Tensor, style_params: torch.Tensor) -> torch.Tensor:
    """``_apply_style_weights`` (styleTransfer.py:36-44) on librst: style_weights (B,H,W,S) already completed
    as ``[1 - sum(w), w]`` (:297-302), style_params (B,1,S,n) -> per-pixel params (B,H,W,n) for S == 2; for any
    other S the params come back unblended, as in the reference (:38-44). The blend is the device formula the
    conv prologues apply to the CIN affine (``rst_style_param_map``), which takes w0 as 1 - w1."""
    B, H, W, S = style_weights.shape
    if tuple(style_params.shape[:3]) != (B, 1, S):
        raise ValueError(f"style_params must be (B,1,S,n) = ({B},1,{S},n), got {tuple(style_params.shape)}")
    if S != 2:
        return style_params
    # the device blend takes w0 as 1 - w1 (the model always completes the weights so, :297-302); refuse weights
    # that are not completed rather than return w0*p0 + w1*p1 computed with a different w0
    w1 = style_weights[..., 1].contiguous()
    if not torch.allclose(style_weights[..., 0], 1.0 - w1, rtol=0.0, atol=1e-6):
        raise ValueError("style_weights[..., 0] must equal 1 - style_weights[..., 1] (the completed [1 - sum(w), w] "
                         "form of styleTransfer.py:297-302)")
    n = style_params.shape[-1]
    p = style_params.reshape(B, 2, n).contiguous()
    out = torch.empty((B, H, W, n), dtype=torch.float32, device=style_weights.device)
    _lib.check(_lib.load().rst_style_param_map(_lib.dev_ptr(w1), _lib.dev_ptr(p), B, H * W, S, n, _lib.dev_ptr(out),
                                               _lib.stream_ptr()))
    return out


def instance_norm(x: torch.Tensor, scale: torch.Tensor, bias: torch.Tensor, eps: float = CIN_EPS,
                  relu: bool = False) -> torch.Tensor:
    """ConditionalInstanceNormalization.call (styleTransfer.py:57-71) for S=1 on librst.

    x (B,H,W,C); scale/bias (B,C)."""
    lib = _lib.load()
    B, H, W, C = x.shape
    x = x.contiguous()
    scale = scale.reshape(B, C).contiguous()
    bias = bias.reshape(B, C).contiguous()
    ws = torch.empty(lib.rst_instance_norm_workspace_size(B, H * W, C), dtype=torch.uint8, device=x.device)
    y = torch.empty_like(x)
    _lib.check(lib.rst_instance_norm(_lib.dev_ptr(x), B, H * W, C, _lib.dev_ptr(scale), _lib.dev_ptr(bias),
                                     float(eps), int(relu), _lib.dev_ptr(y), int(ws.data_ptr()), _lib.stream_ptr()))
    return y

