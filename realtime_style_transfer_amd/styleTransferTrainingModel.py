"""Host mirror of ``realtime_style_transfer/models/styleTransferTrainingModel.py`` and of the
training loop body of ``train_network.py:102-138`` on librst (MI355X).

``StyleTransferTrainingModel`` owns one ``rst_trainer`` (include/rst.h): the transfer network's
weights and RMSprop slots live on the GPU; one ``train_step`` runs the training-mode forward,
the VGG16/Gram loss (``StyleLossModelVGG`` factors), the backward and the RMSprop update
entirely in hand-written gfx950 kernels. There is no CPU fallback.

With a style predictor (``StylePredictionTrainer``, stylePrediction.py:25-75 in training mode) the
step is the reference's joint one: ``x = {'content', 'style'}``, the predictor's output feeds the
transfer network as its style parameters, their gradient flows back into the predictor, and both
weight sets take an RMSprop step. Without one, ``style_params`` are an input (``x = {'content',
'style_params'}``) and their gradient is returned.

* ``compute_loss`` returns the per-image ``(B,)`` loss; Keras minimises its sum, and so does this.
* Data parallel: under an initialised process group, ONE all-reduce per step (SUM, RCCL over xGMI)
  carries the flat bucket [transfer gradient | predictor gradient | BN moving statistics]. Summing the
  gradients equals one step on the concatenated global batch except that each rank normalises with its
  own BatchNorm batch statistics (TF without SyncBatchNorm does the same). The BN *moving* statistics,
  which each rank's forward updated from its own batch, come back divided by the world size and are
  written straight into the canonical weights (``rst_*trainer_set_moving_statistics``, no re-pack):
  TF MirroredStrategy's MEAN aggregation of the moving-average assignments. The update is linear, so
  the mean of the per-rank updates equals the update with the mean of the per-rank batch statistics,
  and every rank keeps bitwise identical weights.
"""
from __future__ import annotations

import ctypes
import logging
import os
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .plan import Plan, init_weights, network_plan
from .styleLoss import DEPTH_LOSS_UNAVAILABLE, StyleLossModelVGG, make_style_loss_function
from .styleTransfer import StyleTransferModel
from .styleTransferInferenceModel import StyleTransferInference, make_style_transfer_inference_model

log = logging.getLogger(__name__)

LOSS_NAMES = ('loss', 'feature_loss', 'style_loss', 'total_variation_loss')


class RMSprop:
    """Keras ``tf.keras.optimizers.RMSprop()`` defaults (train_network.py:102)."""

    def __init__(self, learning_rate: float = 1e-3, rho: float = 0.9, momentum: float = 0.0, epsilon: float = 1e-7,
                 centered: bool = False):
        if momentum != 0.0 or centered:
            raise NotImplementedError("RMSprop with momentum or centered=True is not used by the reference")
        self.learning_rate, self.rho, self.epsilon = float(learning_rate), float(rho), float(epsilon)


def _all_reduce_sum(t: torch.Tensor, group=None):
    """SUM over the group in place; gloo gets a host copy of a device tensor (RCCL reduces in HBM)."""
    dist = torch.distributed
    if t.is_cuda and dist.get_backend(group) != "nccl":
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


def allreduce_gradients(grad: torch.Tensor, group=None) -> bool:
    """Data-parallel gradient exchange: one flat bucket (the whole ~5.9 MB fp32 gradient of
    rst-960-120-128-17) summed in place across the process group — RCCL over xGMI with the
    "nccl" backend on MI355X, gloo on CPU. SUM, not mean: the reference minimises the per-image
    loss vector's sum, so the global step equals one step on the concatenated batch. Returns
    whether a collective ran (no-op for world size 1 / no process group)."""
    dist = torch.distributed
    if not (dist.is_available() and dist.is_initialized()):
        return False
    if dist.get_world_size(group) == 1:
        return False
    _all_reduce_sum(grad, group)
    return True


def average_over_ranks(values: torch.Tensor, group=None) -> bool:
    """values <- mean over the ranks (in place); False when there is nothing to average with."""
    dist = torch.distributed
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return False
    _all_reduce_sum(values, group)
    values /= dist.get_world_size(group)
    return True


def moving_statistics_index(weight_names_or_layers) -> np.ndarray:
    """Flat indices (Keras get_weights() order, concatenated) of every BatchNormalization moving_mean /
    moving_variance entry, from [(name, shape)] pairs."""
    idx, o = [], 0
    for name, shape in weight_names_or_layers:
        n = int(np.prod(shape))
        if name.endswith('moving_mean') or name.endswith('moving_variance'):
            idx.append(np.arange(o, o + n))
        o += n
    return np.concatenate(idx) if idx else np.zeros(0, np.int64)


class StyleTransferTrainingModel:
    """styleTransferTrainingModel.py:11-36 + Keras train_step, one GPU (one librst trainer)."""

    def __init__(self, input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters,
                 loss_model: Optional[StyleLossModelVGG] = None, weights: Optional[Sequence[np.ndarray]] = None,
                 seed: int = 2, max_batch: int = 4, optimizer: Optional[RMSprop] = None, process_group=None,
                 device=None, name: str = "StyleTransferTrainingModel", style_predictor=None,
                 precision: str = "winograd_bf16x6", with_depth_loss: bool = False):
        """``loss_model``: a StyleLossModelVGG (trainable), or a construct-only loss model such as
        StyleLossModelMobileNet, with which the model is built (weights, inference ``__call__``) but
        ``train_step`` raises — what the reference's inference and export scripts need
        (predict_video_using_checkpoint.py:43-58, save_using_checkpoint.py:39-53). ``with_depth_loss``: the
        loss asked for the MiDaS depth term (unavailable): construction works, ``train_step`` raises.
        ``precision``: the transfer network's arithmetic — "winograd_bf16x6" (default; fp32-level, the benchmarked
        config-4 line), "fp32_winograd" or "fp32"; the VGG16 loss network's comes from ``loss_model.precision``."""
        if precision not in ("fp32", "fp32_winograd", "winograd_bf16x6"):
            raise ValueError("transfer-network training precision must be 'fp32', 'fp32_winograd' or "
                             f"'winograd_bf16x6', got {precision!r}")
        self.name = name
        self.precision = precision
        self.plan: Plan = network_plan(input_shape, output_shape, bottleneck_res_y, bottleneck_num_filters, 1)
        self.input_shape = tuple(int(v) for v in input_shape)
        self.output_shape = tuple(int(v) for v in output_shape)
        self.max_batch = int(max_batch)
        self.num_style_parameters = self.plan.num_style_params
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.optimizer = optimizer or RMSprop()
        self.process_group = process_group
        # the style predictor's backward beside the transfer network's tail of the backward (_predictor_backward)
        self._overlap_pbwd = os.environ.get("RST_SERIAL_PREDICTOR_BWD", "0") != "1"
        self._pbwd_stream = None
        self.loss_model = loss_model or StyleLossModelVGG(self.output_shape, max_batch=self.max_batch,
                                                          device=self.device)
        if tuple(self.loss_model.input_shape) != self.output_shape:
            raise ValueError(f"loss model input {self.loss_model.input_shape} != output shape {self.output_shape}")
        self.with_depth_loss = bool(with_depth_loss)
        self._shapes = [tuple(s) for s in self.plan.weight_shapes()]
        self._sizes = [int(np.prod(s)) for s in self._shapes]
        w = weights if weights is not None else init_weights(self.plan, seed)
        flat = self._flatten(w)
        self.style_predictor = style_predictor      # StylePredictionTrainer or None
        self.style_losses: Dict[str, torch.Tensor] = {}
        self._version, self._inference = 0, None
        self.iterations = 0                         # optimizer steps taken (Keras OptimizerV2.iterations)
        self._handle = None
        if not isinstance(self.loss_model, StyleLossModelVGG):
            # construct-only: weights on the host, no trainer (train_step raises)
            self._host_weights = flat.copy()
            self.num_weights = flat.size
            return
        lib = _lib.load()
        H, W, C = self.input_shape
        shape = _lib.RstShape(H, W, C, self.output_shape[0], self.output_shape[1], self.plan.bottleneck_res_y,
                              self.plan.bottleneck_num_filters, 1, self.max_batch)
        lm = self.loss_model
        lshape = _lib.RstLossShape(self.output_shape[0], self.output_shape[1], self.max_batch,
                                   lm.content_loss_factor, lm.style_loss_factor, lm.total_variation_loss_factor,
                                   _lib.PRECISIONS[lm.precision])
        vgg = np.concatenate([a.reshape(-1) for a in lm.weights]).astype(np.float32)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.rst_trainer_create_ex(ctypes.byref(shape), flat.ctypes.data, flat.size,
                                                 ctypes.byref(lshape), vgg.ctypes.data, vgg.size,
                                                 _lib.PRECISIONS[precision], ctypes.byref(h)))
        self._handle = h
        self.num_weights = int(lib.rst_trainer_num_weights(h))
        if self.num_weights != flat.size or lib.rst_trainer_num_style_params(h) != self.num_style_parameters:
            raise RuntimeError("librst trainer plan disagrees with the host plan")
        n_pred = 0
        if style_predictor is not None:
            if style_predictor.num_top_parameters != self.num_style_parameters:
                raise ValueError(f"style predictor emits {style_predictor.num_top_parameters} parameters, the "
                                 f"transfer network takes {self.num_style_parameters}")
            if style_predictor.max_batch < self.max_batch:
                raise ValueError("style predictor max_batch is smaller than the training batch")
            n_pred = style_predictor.num_weights
        # one flat bucket, one all-reduce per step: [transfer gradient | predictor gradient | transfer BN moving
        # statistics | predictor BN moving statistics]
        self._n_stat = int(lib.rst_trainer_num_moving_statistics(h))
        self._n_pstat = int(_lib.load().rst_predictor_trainer_num_moving_statistics(style_predictor._handle)) \
            if style_predictor is not None else 0
        nb = self.num_weights + n_pred
        self._bucket = torch.zeros(nb + self._n_stat + self._n_pstat, dtype=torch.float32, device=self.device)
        self._grad_bucket = self._bucket[:nb]
        self._stat = self._bucket[nb:nb + self._n_stat]
        self._pstat = self._bucket[nb + self._n_stat:]
        # BN moving statistics (contract blocks: layer weights kernel, bias, gamma, beta, moving_mean,
        # moving_variance — styleTransfer.py:190-203) for the cross-rank average after each step
        named = []
        for layer in self.plan.layers:
            attrs = ['kernel', 'bias'] + (['gamma', 'beta', 'moving_mean', 'moving_variance'] if layer.norm == 'bn' else [])
            named += list(zip(attrs, layer.weight_shapes))
        self._bn_index = torch.from_numpy(moving_statistics_index(named)).to(self.device)
        self._grad = self._bucket[:self.num_weights]
        self._pgrad = self._bucket[self.num_weights:nb] if n_pred else None

    # ------------------------------------------------------------------ lifecycle
    def _flatten(self, weights: Sequence[np.ndarray]) -> np.ndarray:
        if len(weights) != len(self._shapes) or any(tuple(np.shape(w)) != s for w, s in zip(weights, self._shapes)):
            raise ValueError(f"weights do not match the network plan: expected {self._shapes}")
        return np.concatenate([np.asarray(w, np.float32).reshape(-1) for w in weights])

    def _unflatten(self, flat: np.ndarray) -> List[np.ndarray]:
        out, o = [], 0
        for s, n in zip(self._shapes, self._sizes):
            out.append(flat[o:o + n].reshape(s).copy())
            o += n
        return out

    def __del__(self):
        try:
            if getattr(self, '_handle', None) is not None:
                _lib.load().rst_trainer_destroy(self._handle)
                self._handle = None
        except Exception:
            pass

    # ------------------------------------------------------------------ Keras-like API
    @property
    def trainable_on_device(self) -> bool:
        return self._handle is not None

    def _require_trainer(self):
        if self.with_depth_loss:
            raise NotImplementedError(DEPTH_LOSS_UNAVAILABLE)
        if self._handle is None:
            raise NotImplementedError(f"{type(self.loss_model).__name__} is construct-only: training needs "
                                      "StyleLossModelVGG (train_network.py:85)")

    def get_weights(self) -> List[np.ndarray]:
        if self._handle is None:
            return self._unflatten(self._host_weights)
        t = torch.empty(self.num_weights, dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().rst_trainer_copy_weights(self._handle, _lib.dev_ptr(t), t.numel(), _lib.stream_ptr()))
        return self._unflatten(t.cpu().numpy())

    def set_weights(self, weights: Sequence[np.ndarray]):
        self._version += 1
        if self._handle is None:
            self._host_weights = self._flatten(weights)
            return
        t = torch.from_numpy(self._flatten(weights)).to(self.device)
        _lib.check(_lib.load().rst_trainer_set_weights(self._handle, _lib.dev_ptr(t), t.numel(), _lib.stream_ptr()))
        torch.cuda.current_stream(self.device).synchronize()

    def _weights_version(self):
        pr = self.style_predictor
        return (self._version, getattr(pr, '_version', 0) if pr is not None else 0)

    def inference_model(self):
        """The Keras model this training model wraps (styleTransferTrainingModel.py:19: inference_model.input ->
        output), in inference mode with the current weights: predictor -> transfer, or the transfer alone. Rebuilt
        whenever the transfer or the predictor weights (BN moving statistics included) changed."""
        v = self._weights_version()
        if self._inference is None or self._inference[0] != v:
            transfer = self.transfer_model()
            model = StyleTransferInference(transfer, self.style_predictor.inference_model(), 1, self.name) \
                if self.style_predictor is not None else transfer
            self._inference = (v, model)
        return self._inference[1]

    def __call__(self, inputs: Dict[str, torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``training(element)`` (save_using_checkpoint.py:63, predict_video_using_checkpoint.py:71): the forward
        with BatchNormalization in inference mode (Keras' default training=False)."""
        return self.inference_model()(inputs, out=out)

    def predict(self, inputs, batch_size=None, verbose=0) -> np.ndarray:
        return self(inputs).cpu().numpy()

    trainable = True

    def compile(self, run_eagerly=False, optimizer=None, **kwargs):
        """Keras Model.compile (train_network.py:103-106): takes the optimizer (an RMSprop of this module)."""
        if optimizer is not None:
            if not isinstance(optimizer, RMSprop):
                raise TypeError("optimizer must be styleTransferTrainingModel.RMSprop (the reference's only optimizer, "
                                "train_network.py:102)")
            self.optimizer = optimizer

    def optimizer_slots(self) -> List[np.ndarray]:
        """RMSprop ``rms`` slots in weight order."""
        t = torch.empty(self.num_weights, dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().rst_trainer_copy_slots(self._handle, _lib.dev_ptr(t), t.numel(), _lib.stream_ptr()))
        return self._unflatten(t.cpu().numpy())

    def set_optimizer_slots(self, slots: Sequence[np.ndarray]):
        """Restore the RMSprop ``rms`` slots (weight order; a checkpoint restore)."""
        self._require_live()
        t = torch.from_numpy(self._flatten(slots)).to(self.device)
        _lib.check(_lib.load().rst_trainer_set_slots(self._handle, _lib.dev_ptr(t), t.numel(), _lib.stream_ptr()))
        torch.cuda.current_stream(self.device).synchronize()

    def _require_live(self):
        if self._handle is None:
            raise NotImplementedError(f"{type(self.loss_model).__name__} is construct-only: no optimizer state")

    # ------------------------------------------------------------------ checkpoints
    # The training model is the functional inference graph (styleTransferTrainingModel.py:19, 44-52), so its
    # weighted layers are the style predictor (layer_with_weights-0: it runs first, styleTransferInferenceModel.py:
    # 23-26) and the transfer network (layer_with_weights-1, :37); after compile(optimizer) the RMSprop state
    # follows: slot ``rms`` of every trainable variable under ``<variable>/.OPTIMIZER_SLOT/optimizer/rms``, and
    # ``optimizer/{iter, learning_rate, rho, decay, momentum}``. Without a predictor (style_params fed directly)
    # the model is the transfer network alone, at the root.
    def _checkpoint_parts(self):
        from .tf_checkpoint import LayerTree, _Part
        from .styleTransfer import transfer_layer_attributes
        tree = LayerTree(transfer_layer_attributes(self.plan))
        pr = self.style_predictor
        if pr is None:
            return [_Part("", tree, self.get_weights, self.set_weights, self._shapes)]
        return pr._checkpoint_parts("layer_with_weights-0/") + \
            [_Part("layer_with_weights-1/", tree, self.get_weights, self.set_weights, self._shapes)]

    def _slot_groups(self):
        """[(part, trainable mask, get slots, set slots)] for the optimizer state."""
        from .stylePrediction import trainable_mask
        parts = self._checkpoint_parts()
        tmask = [not (p.endswith('/moving_mean') or p.endswith('/moving_variance')) for p in parts[-1].tree.paths()]
        groups = [(parts[-1], tmask, self.optimizer_slots, self.set_optimizer_slots)]
        if self.style_predictor is not None:
            pr = self.style_predictor
            groups.insert(0, (parts[0], trainable_mask(pr.spec), pr.optimizer_slots, pr.set_optimizer_slots))
        return groups

    def _checkpoint_tensors(self):
        from .tf_checkpoint import SLOT_MARK, VAR_SUFFIX, parts_tensors
        out = parts_tensors(self._checkpoint_parts())
        if self._handle is None:
            return out
        for part, mask, get, _ in self._slot_groups():
            for path, slot, trainable in zip(part.tree.paths(part.prefix), get(), mask):
                if trainable:
                    out[f"{path}{SLOT_MARK}optimizer/rms{VAR_SUFFIX}"] = np.asarray(slot, np.float32)
        o = self.optimizer
        out["optimizer/iter" + VAR_SUFFIX] = np.array(self.iterations, np.int64)
        for name, v in (("learning_rate", o.learning_rate), ("rho", o.rho), ("decay", 0.0), ("momentum", 0.0)):
            out[f"optimizer/{name}{VAR_SUFFIX}"] = np.array(v, np.float32)
        return out

    def _restore_tensors(self, tensors):
        from .tf_checkpoint import SLOT_MARK, VAR_SUFFIX, restore_parts
        used, slot_sets = [], []
        if self._handle is not None:
            for part, mask, get, set_ in self._slot_groups():
                keys = [f"{p}{SLOT_MARK}optimizer/rms{VAR_SUFFIX}" if t else None
                        for p, t in zip(part.tree.paths(part.prefix), mask)]
                have = [k in tensors for k in keys if k is not None]
                if have and all(have):
                    slot_sets.append((keys, get, set_))
                    used += [k for k in keys if k is not None]
            used += [f"optimizer/{n}{VAR_SUFFIX}" for n in ("iter", "learning_rate", "rho", "decay", "momentum")
                     if f"optimizer/{n}{VAR_SUFFIX}" in tensors]
        status = restore_parts(self._checkpoint_parts(), tensors, extra_keys=used)   # validates, then sets weights
        for keys, get, set_ in slot_sets:
            set_([np.asarray(tensors[k], np.float32).reshape(c.shape) if k is not None else np.zeros_like(c)
                  for k, c in zip(keys, get())])
        if self._handle is not None:
            it = tensors.get("optimizer/iter" + VAR_SUFFIX)
            if it is not None:
                self.iterations = int(it)
                if self.style_predictor is not None:
                    self.style_predictor.iterations = int(it)
            for name in ("learning_rate", "rho"):
                if f"optimizer/{name}{VAR_SUFFIX}" in tensors:
                    setattr(self.optimizer, name, float(tensors[f"optimizer/{name}{VAR_SUFFIX}"]))
        return status

    def load_weights(self, filepath):
        """``training.load_weights(path)`` (predict_video_using_checkpoint.py:74) -> CheckpointLoadStatus: the
        predictor and transfer weights and, when the checkpoint holds them, the RMSprop state."""
        from .tf_checkpoint import load_weights
        return load_weights(self, filepath)

    def save_weights(self, filepath) -> None:
        """``Model.save_weights`` of the training model (tracing/checkpoint.py:37, TF format): weights + optimizer."""
        from .tf_checkpoint import save_weights
        save_weights(self, filepath)

    def output_gradient(self, idx: int, batch: int) -> torch.Tensor:
        """Debug: d loss / d (activated output of conv layer idx) of the most recent step."""
        layer = self.plan.layers[idx]
        t = torch.empty((batch,) + tuple(layer.out_hw) + (layer.cout,), dtype=torch.float32, device=self.device)
        _lib.check(_lib.load().rst_trainer_copy_output_gradient(self._handle, idx, _lib.dev_ptr(t), t.numel(), batch,
                                                                _lib.stream_ptr()))
        return t

    def vgg_feature(self, layer: str, batch: int) -> torch.Tensor:
        """Debug: a VGG16 conv output of the most recent prediction (the trainer's loss model)."""
        from .styleLoss import VGG16_CHANNELS, VGG16_LAYER_NAMES
        idx = VGG16_LAYER_NAMES.index(layer)
        H, W = self.output_shape[:2]
        div = 2 ** sum(1 for i in (1, 3, 6, 9) if i < idx)
        t = torch.empty((batch, H // div, W // div, VGG16_CHANNELS[idx]), dtype=torch.float32, device=self.device)
        lib = _lib.load()
        _lib.check(lib.rst_loss_copy_feature(lib.rst_trainer_loss(self._handle), idx, _lib.dev_ptr(t), t.numel(),
                                             batch, _lib.stream_ptr()))
        return t

    def _check(self, content, style_params, gt_content, gt_style):
        B = content.shape[0]
        if tuple(content.shape) != (B,) + self.input_shape:
            raise ValueError(f"content must be (B,{self.input_shape}), got {tuple(content.shape)}")
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch={self.max_batch}")
        sp = style_params.reshape(B, -1) if style_params.dim() == 3 and style_params.shape[1] == 1 else style_params
        if tuple(sp.shape) != (B, self.num_style_parameters):
            raise ValueError(f"style_params must be (B,1,{self.num_style_parameters}), got {tuple(style_params.shape)}")
        if gt_style.dim() == 5:
            if gt_style.shape[1] != 1:   # styleLoss.py:311-312
                raise ValueError(f"Loss model does not support multiple styles. Found {gt_style.shape[1]}")
            gt_style = gt_style[:, 0]
        for t in (gt_content, gt_style):
            if tuple(t.shape) != (B,) + self.output_shape:
                raise ValueError(f"ground truth must be (B,{self.output_shape}), got {tuple(t.shape)}")
        return B, content.contiguous(), sp.contiguous(), gt_content.contiguous(), gt_style.contiguous()

    def compute_targets(self, gt_content: torch.Tensor, gt_style: torch.Tensor):
        """Start the loss targets of the next ``compute_gradients`` (the style image's Grams and the content image's
        block5_conv3 features, rst_trainer_compute_targets) on the trainer's side stream, so that they run beside
        the work queued after this call (the style predictor's forward in ``train_step``). The next
        ``compute_gradients`` must get these same ground-truth tensors; results are bitwise those without."""
        self._require_trainer()
        gs = gt_style[:, 0] if gt_style.dim() == 5 and gt_style.shape[1] == 1 else gt_style
        B = gt_content.shape[0]
        for t in (gt_content, gs):
            if tuple(t.shape) != (B,) + self.output_shape:
                raise ValueError(f"ground truth must be (B,{self.output_shape}), got {tuple(t.shape)}")
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch={self.max_batch}")
        gc, gs = gt_content.contiguous(), gs.contiguous()
        _lib.check(_lib.load().rst_trainer_compute_targets(self._handle, _lib.dev_ptr(gc), _lib.dev_ptr(gs), B,
                                                           _lib.stream_ptr()))
        self._pending_targets = (gt_content, gt_style, gc, gs)   # keeps the buffers alive until the join

    def cancel_targets(self):
        """Drop the loss targets ``compute_targets`` started (the step failed before ``compute_gradients``)."""
        if self._handle is not None:
            self._pending_targets = None
            _lib.check(_lib.load().rst_trainer_cancel_targets(self._handle, _lib.stream_ptr()))

    def compute_gradients(self, content: torch.Tensor, style_params: torch.Tensor, gt_content: torch.Tensor,
                          gt_style: torch.Tensor, grad: Optional[torch.Tensor] = None,
                          grad_style_params: Optional[torch.Tensor] = None):
        """Training-mode forward + loss + backward -> (prediction, losses (B,4), grad, grad_style_params)."""
        self._require_trainer()
        pending = getattr(self, "_pending_targets", None)
        self._pending_targets = None
        gt_in = (gt_content, gt_style)
        B, content, sp, gt_content, gt_style = self._check(content, style_params, gt_content, gt_style)
        if pending is not None and pending[0] is gt_in[0] and pending[1] is gt_in[1]:
            gt_content, gt_style = pending[2], pending[3]   # the buffers the targets were started on
        dev = content.device
        pred = torch.empty((B,) + self.output_shape, dtype=torch.float32, device=dev)
        losses = torch.empty((B, 4), dtype=torch.float32, device=dev)
        grad = self._grad if grad is None else grad
        if grad_style_params is None:
            grad_style_params = torch.empty((B, self.num_style_parameters), dtype=torch.float32, device=dev)
        _lib.check(_lib.load().rst_trainer_compute_gradients(
            self._handle, _lib.dev_ptr(content), _lib.dev_ptr(sp), _lib.dev_ptr(gt_content), _lib.dev_ptr(gt_style),
            B, _lib.dev_ptr(pred), _lib.dev_ptr(losses), _lib.dev_ptr(grad), _lib.dev_ptr(grad_style_params),
            _lib.stream_ptr()))
        return pred, losses, grad, grad_style_params

    def apply_gradients(self, grad: torch.Tensor):
        self._require_trainer()
        self._version += 1
        o = self.optimizer
        _lib.check(_lib.load().rst_trainer_apply_gradients(self._handle, _lib.dev_ptr(grad), o.learning_rate, o.rho,
                                                           o.epsilon, _lib.stream_ptr()))
        self.iterations += 1

    def _world(self) -> int:
        dist = torch.distributed
        if not (dist.is_available() and dist.is_initialized()):
            return 1
        return dist.get_world_size(self.process_group)

    def _get_moving_statistics(self):
        """BN moving statistics (transfer net, then the jointly trained predictor) -> the bucket's tail."""
        lib = _lib.load()
        if self._n_stat:
            _lib.check(lib.rst_trainer_get_moving_statistics(self._handle, _lib.dev_ptr(self._stat), self._n_stat,
                                                             _lib.stream_ptr()))
        if self._n_pstat:
            _lib.check(lib.rst_predictor_trainer_get_moving_statistics(
                self.style_predictor._handle, _lib.dev_ptr(self._pstat), self._n_pstat, _lib.stream_ptr()))

    def _set_moving_statistics(self, divisor: float):
        lib = _lib.load()
        self._version += 1
        if self.style_predictor is not None:
            self.style_predictor._version += 1
        if self._n_stat:
            _lib.check(lib.rst_trainer_set_moving_statistics(self._handle, _lib.dev_ptr(self._stat), self._n_stat,
                                                             float(divisor), _lib.stream_ptr()))
        if self._n_pstat:
            _lib.check(lib.rst_predictor_trainer_set_moving_statistics(
                self.style_predictor._handle, _lib.dev_ptr(self._pstat), self._n_pstat, float(divisor),
                _lib.stream_ptr()))

    def exchange(self) -> bool:
        """The data-parallel step exchange: ONE all-reduce (SUM) of [gradients | BN moving statistics], then the
        moving statistics divided by the world size go straight back into the weights (no re-pack). No-op
        without a multi-rank process group."""
        world = self._world()
        if world == 1:
            return False
        self._get_moving_statistics()
        _all_reduce_sum(self._bucket, self.process_group)
        self._set_moving_statistics(world)
        return True

    def sync_moving_statistics(self) -> bool:
        """Average only the BatchNorm moving statistics over the ranks (a separate small all-reduce; train_step
        folds this into the gradient all-reduce instead). No-op without a multi-rank process group."""
        world = self._world()
        if world == 1:
            return False
        self._get_moving_statistics()
        tail = self._bucket[self._grad_bucket.numel():]
        _all_reduce_sum(tail, self.process_group)
        self._set_moving_statistics(world)
        return True

    def compute_loss(self, x=None, y=None, y_pred=None, sample_weight=None):
        """styleTransferTrainingModel.py:26-29: the (B,) 'loss' of the most recent step."""
        return self.style_losses['loss']

    def compute_metrics(self, x=None, y=None, y_pred=None, sample_weight=None) -> Dict[str, torch.Tensor]:
        """styleTransferTrainingModel.py:31-33: batch means of every loss term."""
        return {n: l.mean() for n, l in self.style_losses.items()}

    def reset_metrics(self):
        self.style_losses = {}

    def _predictor_backward(self, pr, gsp: torch.Tensor):
        """The style predictor's backward from d loss / d style_params. On the GPU it runs on a side stream that starts
        where the transfer network's backward has made gsp final (after its last conditional instance norm,
        rst_trainer_wait_style_gradient) and so overlaps the rest of that backward — the contract layers and the start
        conv's weight gradient — instead of following it; the caller's stream joins it before either gradient is used.
        Same kernels on the same inputs: the gradients are bitwise those of the serial order (RST_SERIAL_PREDICTOR_BWD=1)."""
        # Under hipGraph capture the backward stays on the caller's stream: a capture whose fork is two levels deep
        # (caller -> this side stream -> the predictor trainer's weight-gradient stream) segfaulted at capture end on
        # this HIP runtime (tools/train_graph_check.py, profiles/r06/r06e); one level (the weight-gradient stream
        # forked from the caller's) captures and replays bitwise. Same kernels, same bits either way.
        if not (gsp.is_cuda and getattr(self, "_overlap_pbwd", True)) or torch.cuda.is_current_stream_capturing():
            pr.backward(gsp, grad=self._pgrad)
            return
        main = torch.cuda.current_stream(gsp.device)
        if getattr(self, "_pbwd_stream", None) is None:
            self._pbwd_stream = torch.cuda.Stream(device=gsp.device)
        side = self._pbwd_stream
        _lib.check(_lib.load().rst_trainer_wait_style_gradient(self._handle, _lib.stream_ptr(side)))
        gsp.record_stream(side)       # the allocator must not hand gsp's memory to the caller's stream before the join
        with torch.cuda.stream(side):
            pr.backward(gsp, grad=self._pgrad)
        main.wait_stream(side)

    def train_step(self, x: Dict[str, torch.Tensor], y: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """One Keras fit step. With a style predictor: x = {'content', 'style' (B,1,H,W,3)}; without:
        x = {'content', 'style_params'}. y = {'content', 'style'}."""
        self._require_trainer()
        pr = self.style_predictor
        if pr is not None:
            style = x['style']
            if style.dim() == 5:
                if style.shape[1] != 1:
                    raise ValueError("the training model takes one style (num_styles=1, styleTransferTrainingModel.py:46)")
                style = style[:, 0]
            self.compute_targets(y['content'], y['style'])            # loss targets beside the predictor forward
            try:
                sp = pr.forward(style)                                 # styleTransferInferenceModel.py:23-28
            except BaseException:
                self.cancel_targets()
                raise
        else:
            sp = x['style_params']
        pred, losses, grad, gsp = self.compute_gradients(x['content'], sp, y['content'], y['style'])
        if pr is not None:
            self._predictor_backward(pr, gsp)
        self.exchange()                       # one collective: gradients + BN moving statistics
        self.apply_gradients(grad)
        if pr is not None:
            o = self.optimizer
            pr.apply_gradients(self._pgrad, o.learning_rate, o.rho, o.epsilon)
        self.style_losses = {n: losses[:, i] for i, n in enumerate(LOSS_NAMES)}
        self.last_prediction = pred
        self.last_style_params = sp
        self.last_grad_style_params = gsp
        return self.compute_metrics()

    def transfer_model(self, max_batch: Optional[int] = None) -> StyleTransferModel:
        """An inference ``StyleTransferModel`` holding the current weights (BN in inference mode)."""
        return StyleTransferModel(self.input_shape, self.output_shape, self.plan.bottleneck_res_y,
                                  self.plan.bottleneck_num_filters, 1, weights=self.get_weights(),
                                  max_batch=max_batch or self.max_batch, device=self.device)


class StyleTransferModels:
    """The object make_style_transfer_training_model returns (styleTransferTrainingModel.py:60-68).
    ``transfer`` / ``style_predictor`` / ``inference`` share the training model's variables, as the Keras models
    do: every access sees the trainers' current weights (a train step, a restore through any of them, moving
    statistics), rebuilt lazily from the trainers when their weight versions changed. ``refresh()`` forces it."""

    def __init__(self, training: StyleTransferTrainingModel, loss_model):
        self.training = training
        self.style_loss = loss_model

        def end_to_end_loss(inputs):
            """loss_model((x, y_true)) (styleTransferTrainingModel.py:59,64): the losses of the inference output."""
            x, y_true = inputs
            if hasattr(loss_model, 'compute'):
                return loss_model.compute(training(x), y_true)
            from .styleLoss import StyleLoss
            return StyleLoss(loss_model, training.with_depth_loss).compute(training(x), y_true)

        self.loss_model = end_to_end_loss
        self._views = None
        self._inference = (_SharedInference(self) if training.style_predictor is not None
                           else _SharedTransfer(self))
        self.refresh()

    def _current(self):
        """(transfer, style_predictor) inference models holding the trainers' current weights."""
        tr = self.training
        v = tr._weights_version()
        if self._views is None or self._views[0] != v:
            transfer = tr.transfer_model()
            sp = tr.style_predictor.inference_model() if tr.style_predictor is not None else None
            self._views = (v, transfer, sp)
        return self._views[1], self._views[2]

    @property
    def transfer(self):
        return self._current()[0]

    @property
    def style_predictor(self):
        return self._current()[1]

    @property
    def inference(self):
        return self._inference

    def refresh(self):
        self._views = None
        self._current()


class _SharedInference(StyleTransferInference):
    """``models.inference``: the inference graph of the training model, sharing its variables as the Keras
    models do (styleTransferTrainingModel.py:52,66): it runs the trainers' current weights, and a checkpoint
    restored through it (``load_weights``, ``Checkpoint(models.inference).restore``, train_network.py:112-113)
    lands in the trainers."""

    def __init__(self, models):
        self._models = models
        self.num_styles = 1
        self.name = models.training.name

    @property
    def transfer(self):
        return self._models.transfer

    @property
    def style_predictor(self):
        return self._models.style_predictor

    def _restore_tensors(self, tensors):
        return _restore_weights_only(self._models, tensors)

    def _checkpoint_tensors(self):
        from .tf_checkpoint import parts_tensors
        return parts_tensors(self._models.training._checkpoint_parts())


def _restore_weights_only(models, tensors):
    """A restore through the inference view (``Checkpoint(models.inference).restore``, train_network.py:112-113;
    ``inference.load_weights``): as in TF, the optimizer is not reachable from the inference model, so only the
    predictor and transfer weights are bound — the RMSprop slots, ``iter`` and the hyperparameters stay untouched and
    are reported unused (``assert_consumed()`` fails on a training checkpoint, as TF's does)."""
    from .tf_checkpoint import restore_parts
    st = restore_parts(models.training._checkpoint_parts(), tensors)
    models.refresh()
    return st


class _SharedTransfer:
    """``models.inference`` without a style predictor: the transfer network (style_params are an input)."""

    def __init__(self, models):
        self._models = models

    def __call__(self, inputs, out=None):
        return self._models.transfer(inputs, out=out)

    def predict(self, inputs, batch_size=None, verbose=0):
        return self._models.transfer.predict(inputs)

    def _restore_tensors(self, tensors):
        return _restore_weights_only(self._models, tensors)

    def _checkpoint_tensors(self):
        from .tf_checkpoint import parts_tensors
        return parts_tensors(self._models.training._checkpoint_parts())

    def load_weights(self, filepath):
        from .tf_checkpoint import load_weights
        return load_weights(self, filepath)

    def save_weights(self, filepath):
        from .tf_checkpoint import save_weights
        save_weights(self, filepath)


def make_style_transfer_training_model(style_predictor_factory_func: Optional[Callable],
                                       style_transfer_factory_func: Callable,
                                       style_loss_func_factory_func: Callable,
                                       name="StyleTransferTrainingModel", max_batch: int = 4,
                                       optimizer: Optional[RMSprop] = None, process_group=None,
                                       precision: str = "winograd_bf16x6"):
    """styleTransferTrainingModel.py:39-70 on librst.

    ``style_transfer_factory_func() -> (StyleTransferModel, P)`` supplies the architecture and
    initial weights; ``style_predictor_factory_func(P) -> StylePredictionModel`` (or None: feed
    ``style_params`` directly) the predictor trained jointly with it (stylePrediction.py:25-75);
    ``style_loss_func_factory_func() -> (compute_loss, StyleLoss)`` the loss (make_style_loss_function). A
    construct-only loss (StyleLossModelMobileNet, or the MiDaS depth term) builds a model whose train_step
    raises — enough for the inference / export scripts, which never train. ``precision``: the transfer network's
    training arithmetic (default "winograd_bf16x6", the benchmarked config-4 line); the VGG16 loss network's is
    the loss model's own (``StyleLossModelVGG(..., precision="bf16")`` for BASELINE config 4)."""
    from .stylePrediction import StylePredictionTrainer
    transfer, P = style_transfer_factory_func()
    predictor = None
    if style_predictor_factory_func is not None:
        pm = style_predictor_factory_func(P)
        predictor = StylePredictionTrainer(pm.input_shape, pm.feature_extractor, pm.num_top_parameters,
                                           pm.num_style_parameters, weights=pm.get_weights(), max_batch=max_batch,
                                           device=transfer.device)
    compute_loss, loss = style_loss_func_factory_func()
    feature_model = getattr(loss, 'feature_model', loss)
    training = StyleTransferTrainingModel(transfer.input_shape, transfer.output_shape, transfer.plan.bottleneck_res_y,
                                          transfer.plan.bottleneck_num_filters, loss_model=feature_model,
                                          weights=transfer.get_weights(), max_batch=max_batch, optimizer=optimizer,
                                          process_group=process_group, device=transfer.device, name=name,
                                          style_predictor=predictor, precision=precision,
                                          with_depth_loss=getattr(compute_loss, 'with_depth_loss', False))
    return StyleTransferModels(training, loss)


__all__ = ['allreduce_gradients', 'RMSprop', 'StyleTransferTrainingModel', 'StyleTransferModels', 'make_style_transfer_training_model',
           'make_style_loss_function', 'make_style_transfer_inference_model']
