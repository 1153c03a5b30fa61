"""Host mirror of ``realtime_style_transfer/models/stylePrediction.py`` on librst (MI355X).

``create_style_prediction_model(input_shape, feature_extractor, num_top_parameters,
num_style_parameters=100, name)`` keeps the reference signature (stylePrediction.py:25-26) and
returns a model called like the Keras one: ``model(style)`` with ``style`` (B, H, W, 3) float32 in
[0, 1] on the GPU -> ``(B, num_top_parameters)`` float32 (:73-75). All compute runs in hand-written
gfx950 kernels behind the C ABI (include/rst.h ``rst_predictor_*``); there is no CPU fallback.

Feature extractors (:19-22): ``DUMMY`` (Conv2D(1, 9, s5, same), :31-32) and ``MOBILE_NET``
(Rescaling(2,-1) + MobileNetV3Small(include_top=False, include_preprocessing=False), :33-38).
``EFFICIENT_NET`` (EfficientNetV2S, :39-43) is not built: it raises ``NotImplementedError``.

Weights use the Keras ``get_weights()`` order (:50-71 and keras.applications.mobilenet_v3). The
reference loads ImageNet weights for MobileNetV3Small, which are not available offline; the
default here is a seeded initialisation with the Keras default initialisers (glorot_uniform
kernels, BN gamma=1/beta=0/mean=0/var=1, the heads' VarianceScaling(1/3, fan_out, uniform) with
bias 0.5, :9-16,62-63,69-70); ``perturb=True`` moves BN statistics and biases off their defaults
so tests exercise every term.
"""
from __future__ import annotations

import ctypes
import logging
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

log = logging.getLogger(__name__)


class StyleFeatureExtractor:
    DUMMY = 'DUMMY'
    EFFICIENT_NET = 'EFFICIENT_NET'
    MOBILE_NET = 'MOBILE_NET'


# keras mobilenet_v3.MobileNetV3Small stack_fn: (expansion, filters, kernel, stride, se, activation)
_MOBILENET_V3_SMALL = [
    (1.0, 16, 3, 2, True, 'relu'), (72.0 / 16, 24, 3, 2, False, 'relu'), (88.0 / 24, 24, 3, 1, False, 'relu'),
    (4.0, 40, 5, 2, True, 'hard_swish'), (6.0, 40, 5, 1, True, 'hard_swish'), (6.0, 40, 5, 1, True, 'hard_swish'),
    (3.0, 48, 5, 1, True, 'hard_swish'), (3.0, 48, 5, 1, True, 'hard_swish'), (6.0, 96, 5, 2, True, 'hard_swish'),
    (6.0, 96, 5, 1, True, 'hard_swish'), (6.0, 96, 5, 1, True, 'hard_swish'),
]


def _depth(v: float, divisor: int = 8) -> int:
    """keras mobilenet_v3._depth."""
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def predictor_weight_spec(input_shape, feature_extractor: str, num_top_parameters: int,
                          num_style_parameters: int = 100) -> List[Tuple[str, Tuple[int, ...], str]]:
    """[(name, shape, initialiser kind)] in Keras get_weights() order."""
    spec: List[Tuple[str, Tuple[int, ...], str]] = []

    def bn(prefix, c):
        spec.extend([(prefix + '/gamma', (c,), 'gamma'), (prefix + '/beta', (c,), 'beta'),
                     (prefix + '/moving_mean', (c,), 'mean'), (prefix + '/moving_variance', (c,), 'var')])

    if feature_extractor == StyleFeatureExtractor.DUMMY:
        spec += [('dummy_conv/kernel', (9, 9, int(input_shape[2]), 1), 'glorot'), ('dummy_conv/bias', (1,), 'zero')]
        c = 1
    elif feature_extractor == StyleFeatureExtractor.MOBILE_NET:
        spec.append(('Conv/kernel', (3, 3, 3, 16), 'glorot'))
        bn('Conv/BatchNorm', 16)
        cin = 16
        for i, (e, f, k, s, se, _) in enumerate(_MOBILENET_V3_SMALL):
            p = 'expanded_conv/' if i == 0 else f'expanded_conv_{i}/'
            ce = _depth(cin * e)
            if i:
                spec.append((p + 'expand/kernel', (1, 1, cin, ce), 'glorot'))
                bn(p + 'expand/BatchNorm', ce)
            spec.append((p + 'depthwise/depthwise_kernel', (k, k, ce, 1), 'glorot'))
            bn(p + 'depthwise/BatchNorm', ce)
            if se:
                r = _depth(ce * 0.25)
                spec += [(p + 'squeeze_excite/Conv/kernel', (1, 1, ce, r), 'glorot'),
                         (p + 'squeeze_excite/Conv/bias', (r,), 'zero'),
                         (p + 'squeeze_excite/Conv_1/kernel', (1, 1, r, ce), 'glorot'),
                         (p + 'squeeze_excite/Conv_1/bias', (ce,), 'zero')]
            spec.append((p + 'project/kernel', (1, 1, ce, f), 'glorot'))
            bn(p + 'project/BatchNorm', f)
            cin = f
        c = _depth(cin * 6)
        spec.append(('Conv_1/kernel', (1, 1, cin, c), 'glorot'))
        bn('Conv_1/BatchNorm', c)
    elif feature_extractor == StyleFeatureExtractor.EFFICIENT_NET:
        raise NotImplementedError("EFFICIENT_NET (EfficientNetV2S) feature extractor is not built on librst")
    else:
        raise ValueError(f"{feature_extractor} is not a valid value for feature_extractor. "
                         f"Must be a StyleFeatureExtractor")
    spec += [('StylePredictor/kernel', (1, 1, c, num_style_parameters), 'head'),
             ('StylePredictor/bias', (num_style_parameters,), 'half'),
             ('StyleNormPredictor/kernel', (1, 1, num_style_parameters, num_top_parameters), 'head'),
             ('StyleNormPredictor/bias', (num_top_parameters,), 'half')]
    return spec


def predictor_layer_tree(spec):
    """The predictor's weighted Keras layers (stylePrediction.py:25-75) as a checkpoint LayerTree: the feature
    extractor first — MobileNetV3Small is a functional model used as a layer (:33-36,52), so its layers nest
    under ``layer_with_weights-0``; DUMMY's ``dummy_conv`` (:31) is a plain layer — then the two 1x1 heads
    ``StylePredictor`` (:59-63) and ``StyleNormPredictor`` (:66-70)."""
    from .tf_checkpoint import LayerTree, layer_tree_from_names
    names = [n for n, _, _ in spec]
    heads = [n for n in names if n.split('/')[0] in ('StylePredictor', 'StyleNormPredictor')]
    trunk = [n for n in names if n not in heads]
    head_layers = layer_tree_from_names(heads).entries
    if all(n.startswith('dummy_conv/') for n in trunk):
        return LayerTree(layer_tree_from_names(trunk).entries + head_layers)
    return LayerTree([layer_tree_from_names(trunk)] + head_layers)


def trainable_mask(spec) -> List[bool]:
    """Which weights are trainable variables (everything but the BatchNormalization moving statistics)."""
    return [not (n.endswith('/moving_mean') or n.endswith('/moving_variance')) for n, _, _ in spec]


def init_predictor_weights(spec, seed: int = 3, perturb: bool = False) -> List[np.ndarray]:
    rng = np.random.default_rng(seed)
    out = []
    for name, shape, kind in spec:
        if kind == 'glorot':
            rf = int(np.prod(shape[:-2]))
            fan_in, fan_out = rf * shape[-2], rf * shape[-1]
            lim = np.sqrt(6.0 / (fan_in + fan_out))
            w = rng.uniform(-lim, lim, shape)
        elif kind == 'head':
            lim = np.sqrt(3.0 * (1.0 / 3.0) / shape[-1])        # VarianceScaling(1/3, fan_out, uniform)
            w = rng.uniform(-lim, lim, shape)
        elif kind == 'half':
            w = np.full(shape, 0.5) + (rng.normal(0.0, 0.05, shape) if perturb else 0.0)
        elif kind == 'zero':
            w = rng.normal(0.0, 0.1, shape) if perturb else np.zeros(shape)
        elif kind == 'gamma':
            w = rng.uniform(0.8, 1.2, shape) if perturb else np.ones(shape)
        elif kind == 'beta':
            w = rng.normal(0.0, 0.1, shape) if perturb else np.zeros(shape)
        elif kind == 'mean':
            w = rng.normal(0.0, 0.1, shape) if perturb else np.zeros(shape)
        elif kind == 'var':
            w = rng.uniform(0.5, 1.5, shape) if perturb else np.ones(shape)
        else:
            raise AssertionError(kind)
        out.append(np.asarray(w, np.float32))
    return out


class StylePredictionModel:
    """A built style predictor resident on one GPU (one librst ``rst_predictor`` handle)."""

    def __init__(self, input_shape, feature_extractor: str, num_top_parameters: int, num_style_parameters: int = 100,
                 name: str = "StylePredictionModel", weights: Optional[Sequence[np.ndarray]] = None, seed: int = 3,
                 max_batch: int = 8, device=None):
        self.name = name
        self.input_shape = tuple(int(v) for v in input_shape)
        if len(self.input_shape) != 3:
            raise ValueError(f"input_shape must be (H, W, C), got {input_shape}")
        self.feature_extractor = feature_extractor
        self.num_top_parameters = int(num_top_parameters)
        self.num_style_parameters = int(num_style_parameters)
        self.max_batch = int(max_batch)
        self.spec = predictor_weight_spec(self.input_shape, feature_extractor, self.num_top_parameters,
                                          self.num_style_parameters)
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self._handle = None
        self._weights = [np.ascontiguousarray(w, np.float32) for w in
                         (weights if weights is not None else init_predictor_weights(self.spec, seed))]
        self._build()

    def _shape_struct(self) -> _lib.RstPredictorShape:
        H, W, C = self.input_shape
        return _lib.RstPredictorShape(H, W, C, _lib.EXTRACTORS[self.feature_extractor], self.num_top_parameters,
                                      self.num_style_parameters, self.max_batch)

    def _build(self):
        lib = _lib.load()
        shapes = [s for _, s, _ in self.spec]
        if len(self._weights) != len(shapes) or any(tuple(w.shape) != s for w, s in zip(self._weights, shapes)):
            raise ValueError(f"weights do not match the predictor: expected {shapes}, "
                             f"got {[w.shape for w in self._weights]}")
        flat = np.concatenate([w.reshape(-1) for w in self._weights]).astype(np.float32)
        shape = self._shape_struct()
        if lib.rst_predictor_num_weights(ctypes.byref(shape)) != flat.size:
            raise RuntimeError("librst predictor plan disagrees with the host weight list")
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.rst_predictor_create(ctypes.byref(shape), flat.ctypes.data, flat.size, ctypes.byref(h)))
        self._release()
        self._handle = h

    def _release(self):
        if self._handle is not None:
            _lib.load().rst_predictor_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    # ------------------------------------------------------------------ Keras-like API
    @property
    def input(self):
        class _Spec:
            shape = (None,) + self.input_shape
        return _Spec()

    @property
    def output_shape(self):
        return (None, self.num_top_parameters)

    def get_weights(self) -> List[np.ndarray]:
        return [w.copy() for w in self._weights]

    def set_weights(self, weights: Sequence[np.ndarray]):
        self._weights = [np.ascontiguousarray(w, np.float32) for w in weights]
        self._build()

    def compile(self, run_eagerly=False, **kwargs):
        """Keras Model.compile: nothing to compile (kernels built ahead of time)."""

    trainable = False

    # ------------------------------------------------------------------ checkpoints (tracing/checkpoint.py:21-37)
    def _checkpoint_parts(self, prefix: str = ""):
        from .tf_checkpoint import _Part
        return [_Part(prefix, predictor_layer_tree(self.spec), self.get_weights, self.set_weights,
                      [s for _, s, _ in self.spec])]

    def _checkpoint_tensors(self):
        from .tf_checkpoint import parts_tensors
        return parts_tensors(self._checkpoint_parts())

    def _restore_tensors(self, tensors):
        from .tf_checkpoint import restore_parts
        return restore_parts(self._checkpoint_parts(), tensors)

    def save_weights(self, filepath) -> None:
        from .tf_checkpoint import save_weights
        save_weights(self, filepath)

    def load_weights(self, filepath, model_path: str = ""):
        """Model.load_weights -> CheckpointLoadStatus; ``model_path`` selects the predictor's subtree of a larger
        model's checkpoint (``"layer_with_weights-0"`` in the inference / training models)."""
        from .tf_checkpoint import read_checkpoint, restore_parts
        pre = model_path.rstrip('/') + '/' if model_path else ''
        return restore_parts(self._checkpoint_parts(pre), read_checkpoint(filepath))

    def __call__(self, style: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        style = _lib.as_device(style, self.device)
        if style.dim() != 4 or tuple(style.shape[1:]) != self.input_shape:
            raise ValueError(f"style must be (B,{','.join(map(str, self.input_shape))}), got {tuple(style.shape)}")
        B = style.shape[0]
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch={self.max_batch} chosen at build time")
        style = style.contiguous()
        if out is None:
            out = torch.empty((B, self.num_top_parameters), dtype=torch.float32, device=style.device)
        elif tuple(out.shape) != (B, self.num_top_parameters) or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous ({B}, {self.num_top_parameters}) tensor")
        _lib.check(_lib.load().rst_predictor_forward(self._handle, _lib.dev_ptr(style), B, _lib.dev_ptr(out),
                                                     _lib.stream_ptr(stream)))
        return out

    def predict(self, style, batch_size=None, verbose=0) -> np.ndarray:
        """Keras Model.predict: the style parameters as a host numpy array."""
        return self(style).cpu().numpy()

    # ------------------------------------------------------------------ debugging
    def num_stages(self) -> int:
        return _lib.load().rst_predictor_num_stages(self._handle)

    def stage_output(self, idx: int, batch: int) -> torch.Tensor:
        """MOBILE_NET: 0 stem, 1..11 inverted-residual blocks, 12 Conv_1 features; DUMMY: 0 conv."""
        lib = _lib.load()
        hwc = (ctypes.c_int * 3)()
        _lib.check(lib.rst_predictor_stage_shape(self._handle, idx, hwc))
        t = torch.empty((batch, hwc[0], hwc[1], hwc[2]), dtype=torch.float32, device=self.device)
        _lib.check(lib.rst_predictor_copy_stage(self._handle, idx, _lib.dev_ptr(t), t.numel(), batch,
                                                _lib.stream_ptr()))
        return t


def create_style_prediction_model(input_shape, feature_extractor: str, num_top_parameters: int,
                                  num_style_parameters: int = 100, name: str = "StylePredictionModel", **kwargs):
    """Drop-in for stylePrediction.create_style_prediction_model (stylePrediction.py:25-75)."""
    log.info(f"Bottlenecking to {num_style_parameters} parameters for {num_top_parameters} norm parameters")
    return StylePredictionModel(input_shape, feature_extractor, num_top_parameters, num_style_parameters, name=name,
                                **kwargs)


class StylePredictionTrainer:
    """The style predictor in Keras training mode on one GPU (one ``rst_predictor_trainer``).

    ``forward(style)`` runs with BatchNormalization on the batch statistics (and updates the moving
    statistics, momentum 0.999); ``backward(d_style_params)`` returns the gradient of
    ``sum(style_params * d_style_params)`` for every weight (Keras order, zeros for moving
    statistics); ``apply_gradients`` is RMSprop on the device-resident weights. train_network.py
    fits this model jointly with the transfer network (stylePrediction.py:25-75 is trainable,
    styleTransferTrainingModel.py:39-70)."""

    def __init__(self, input_shape, feature_extractor: str, num_top_parameters: int, num_style_parameters: int = 100,
                 weights: Optional[Sequence[np.ndarray]] = None, seed: int = 3, max_batch: int = 4, device=None):
        self.input_shape = tuple(int(v) for v in input_shape)
        self.feature_extractor = feature_extractor
        self.num_top_parameters = int(num_top_parameters)
        self.num_style_parameters = int(num_style_parameters)
        self.max_batch = int(max_batch)
        self.spec = predictor_weight_spec(self.input_shape, feature_extractor, self.num_top_parameters,
                                          self.num_style_parameters)
        self._shapes = [s for _, s, _ in self.spec]
        self._sizes = [int(np.prod(s)) for s in self._shapes]
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        w = weights if weights is not None else init_predictor_weights(self.spec, seed)
        if len(w) != len(self._shapes) or any(tuple(np.shape(a)) != s for a, s in zip(w, self._shapes)):
            raise ValueError(f"weights do not match the predictor: expected {self._shapes}")
        flat = np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in w])
        lib = _lib.load()
        H, W, C = self.input_shape
        shape = _lib.RstPredictorShape(H, W, C, _lib.EXTRACTORS[feature_extractor], self.num_top_parameters,
                                       self.num_style_parameters, self.max_batch)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.rst_predictor_trainer_create(ctypes.byref(shape), flat.ctypes.data, flat.size,
                                                        ctypes.byref(h)))
        self._handle = h
        self.num_weights = int(lib.rst_predictor_trainer_num_weights(h))
        if self.num_weights != flat.size:
            raise RuntimeError("librst predictor trainer plan disagrees with the host weight list")
        self._style = None
        self._version = 0          # bumped by every weight change (keys the training model's inference cache)
        self.iterations = 0

    def __del__(self):
        try:
            if getattr(self, '_handle', None) is not None:
                _lib.load().rst_predictor_trainer_destroy(self._handle)
                self._handle = None
        except Exception:
            pass

    def _unflatten(self, flat: np.ndarray) -> List[np.ndarray]:
        out, o = [], 0
        for s, n in zip(self._shapes, self._sizes):
            out.append(flat[o:o + n].reshape(s).copy())
            o += n
        return out

    def forward(self, style: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if style.dim() != 4 or tuple(style.shape[1:]) != self.input_shape:
            raise ValueError(f"style must be (B,{','.join(map(str, self.input_shape))}), got {tuple(style.shape)}")
        B = style.shape[0]
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch={self.max_batch}")
        self._style = style.contiguous()          # must outlive the matching backward
        if out is None:
            out = torch.empty((B, self.num_top_parameters), dtype=torch.float32, device=style.device)
        _lib.check(_lib.load().rst_predictor_trainer_forward(self._handle, _lib.dev_ptr(self._style), B,
                                                             _lib.dev_ptr(out), _lib.stream_ptr()))
        return out

    def backward(self, d_style_params: torch.Tensor, grad: Optional[torch.Tensor] = None) -> torch.Tensor:
        if grad is None:
            grad = torch.empty(self.num_weights, dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().rst_predictor_trainer_backward(self._handle, _lib.dev_ptr(d_style_params.contiguous()),
                                                              _lib.dev_ptr(grad), _lib.stream_ptr()))
        return grad

    def apply_gradients(self, grad: torch.Tensor, learning_rate: float = 1e-3, rho: float = 0.9,
                        epsilon: float = 1e-7):
        self._version += 1
        self.iterations += 1
        _lib.check(_lib.load().rst_predictor_trainer_apply_gradients(self._handle, _lib.dev_ptr(grad),
                                                                     float(learning_rate), float(rho), float(epsilon),
                                                                     _lib.stream_ptr()))

    def weights_tensor(self) -> torch.Tensor:
        """Device copy of the flat weights (Keras get_weights() order)."""
        t = torch.empty(self.num_weights, dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().rst_predictor_trainer_copy_weights(self._handle, _lib.dev_ptr(t), t.numel(),
                                                                  _lib.stream_ptr()))
        return t

    def set_weights_tensor(self, t: torch.Tensor):
        self._version += 1
        _lib.check(_lib.load().rst_predictor_trainer_set_weights(self._handle, _lib.dev_ptr(t.contiguous()), t.numel(),
                                                                 _lib.stream_ptr()))

    @property
    def moving_statistics_index(self) -> torch.Tensor:
        """Flat indices of the BN moving_mean / moving_variance entries (averaged across data-parallel ranks)."""
        if getattr(self, '_ms_index', None) is None:
            from .styleTransferTrainingModel import moving_statistics_index
            self._ms_index = torch.from_numpy(moving_statistics_index([(n, s) for n, s, _ in self.spec])).to(self.device)
        return self._ms_index

    def get_weights(self) -> List[np.ndarray]:
        return self._unflatten(self.weights_tensor().cpu().numpy())

    def set_weights(self, weights: Sequence[np.ndarray]):
        if len(weights) != len(self._shapes) or any(tuple(np.shape(a)) != s for a, s in zip(weights, self._shapes)):
            raise ValueError(f"weights do not match the predictor: expected {self._shapes}")
        flat = np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in weights])
        self.set_weights_tensor(torch.from_numpy(flat).to(self.device))
        torch.cuda.current_stream(self.device).synchronize()

    def optimizer_slots(self) -> List[np.ndarray]:
        t = torch.empty(self.num_weights, dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().rst_predictor_trainer_copy_slots(self._handle, _lib.dev_ptr(t), t.numel(),
                                                                _lib.stream_ptr()))
        return self._unflatten(t.cpu().numpy())

    def set_optimizer_slots(self, slots: Sequence[np.ndarray]):
        """Restore the RMSprop ``rms`` slots (Keras order; a checkpoint restore)."""
        flat = np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in slots])
        if flat.size != self.num_weights:
            raise ValueError("optimizer slots do not match the predictor")
        t = torch.from_numpy(flat).to(self.device)
        _lib.check(_lib.load().rst_predictor_trainer_set_slots(self._handle, _lib.dev_ptr(t), t.numel(),
                                                               _lib.stream_ptr()))
        torch.cuda.current_stream(self.device).synchronize()

    def _checkpoint_parts(self, prefix: str = ""):
        from .tf_checkpoint import _Part
        return [_Part(prefix, predictor_layer_tree(self.spec), self.get_weights, self.set_weights, self._shapes)]

    def unflatten(self, grad: torch.Tensor) -> List[np.ndarray]:
        return self._unflatten(grad.detach().cpu().numpy())

    def inference_model(self, max_batch: Optional[int] = None) -> StylePredictionModel:
        """An inference StylePredictionModel with the current weights (BN on the moving statistics)."""
        return StylePredictionModel(self.input_shape, self.feature_extractor, self.num_top_parameters,
                                    self.num_style_parameters, weights=self.get_weights(),
                                    max_batch=max_batch or self.max_batch, device=self.device)
