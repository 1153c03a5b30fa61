"""ctypes binding of librst.so (the C ABI in include/rst.h).

The product path has no fallback: if librst.so is missing or cannot be loaded, every
entry point raises. ``torch`` is imported first so that librst resolves
``libamdhip64.so.7`` to the HIP runtime torch already loaded (one runtime per process,
so torch's hipStream_t handles are valid inside librst).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np
import torch  # noqa: F401  (must precede loading librst, see module docstring)

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "librst.so"

RST_OK, RST_ERR_INVALID, RST_ERR_UNSUPPORTED, RST_ERR_HIP, RST_ERR_ALLOC = range(5)
PRECISIONS = {"fp32": 0, "bf16x3": 1, "bf16x6": 2, "fp32_winograd": 3, "bf16": 4, "winograd_bf16x6": 5}   # include/rst.h RST_PRECISION_*

# Symbols declared in include/rst.h — tests check that the library exports all of them.
EXPORTED_SYMBOLS = [
    "rst_create", "rst_create_ex", "rst_precision", "rst_destroy", "rst_num_style_params", "rst_num_weights_for_shape", "rst_forward",
    "rst_num_layers", "rst_layer_output_shape", "rst_copy_activation", "rst_gram_workspace_size", "rst_gram",
    "rst_instance_norm_workspace_size", "rst_instance_norm", "rst_style_param_map", "rst_last_error", "rst_version",
    "rst_profile_begin", "rst_profile_end", "rst_timeline_begin", "rst_timeline_read", "rst_timeline_end",
    "rst_layer_kernel_id",
    "rst_loss_num_weights", "rst_loss_create", "rst_loss_destroy", "rst_loss_forward", "rst_loss_copy_feature",
    "rst_trainer_create", "rst_trainer_create_ex", "rst_trainer_destroy", "rst_trainer_num_style_params", "rst_trainer_num_weights",
    "rst_trainer_compute_gradients", "rst_trainer_compute_targets", "rst_trainer_apply_gradients",
    "rst_trainer_copy_weights",
    "rst_trainer_copy_slots", "rst_trainer_set_weights", "rst_trainer_set_slots", "rst_trainer_cancel_targets", "rst_trainer_wait_style_gradient",
    "rst_trainer_copy_output_gradient",
    "rst_trainer_debug_vgg_gradient", "rst_trainer_loss", "rst_trainer_num_moving_statistics",
    "rst_trainer_get_moving_statistics", "rst_trainer_set_moving_statistics",
    "rst_predictor_num_weights", "rst_predictor_create", "rst_predictor_destroy", "rst_predictor_forward",
    "rst_predictor_num_stages", "rst_predictor_stage_shape", "rst_predictor_copy_stage",
    "rst_predictor_trainer_create", "rst_predictor_trainer_destroy", "rst_predictor_trainer_num_weights",
    "rst_predictor_trainer_forward", "rst_predictor_trainer_backward", "rst_predictor_trainer_apply_gradients",
    "rst_predictor_trainer_copy_weights", "rst_predictor_trainer_set_weights", "rst_predictor_trainer_copy_slots",
    "rst_predictor_trainer_set_slots", "rst_predictor_trainer_num_moving_statistics", "rst_predictor_trainer_get_moving_statistics",
    "rst_predictor_trainer_set_moving_statistics",
    "rst_gbuffer_resized_size", "rst_gbuffer_preprocess", "rst_crc32c_extend",
]
EXTRACTORS = {"DUMMY": 0, "MOBILE_NET": 1}   # include/rst.h RST_EXTRACTOR_*


class RstShape(ctypes.Structure):
    _fields_ = [("in_h", ctypes.c_int), ("in_w", ctypes.c_int), ("in_c", ctypes.c_int),
                ("out_h", ctypes.c_int), ("out_w", ctypes.c_int),
                ("bottleneck_res_y", ctypes.c_int), ("bottleneck_num_filters", ctypes.c_int),
                ("num_styles", ctypes.c_int), ("max_batch", ctypes.c_int)]


class RstLossShape(ctypes.Structure):
    _fields_ = [("h", ctypes.c_int), ("w", ctypes.c_int), ("max_batch", ctypes.c_int),
                ("content_factor", ctypes.c_float), ("style_factor", ctypes.c_float), ("tv_factor", ctypes.c_float),
                ("precision", ctypes.c_int)]


class RstPredictorShape(ctypes.Structure):
    _fields_ = [("h", ctypes.c_int), ("w", ctypes.c_int), ("c", ctypes.c_int), ("feature_extractor", ctypes.c_int),
                ("num_top_parameters", ctypes.c_int), ("num_style_parameters", ctypes.c_int),
                ("max_batch", ctypes.c_int)]


class RstError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"librst error {code}: {msg}")
        self.code = code


_lib = None


class _MissingSymbol:
    def __init__(self, name):
        self.name = name

    def __call__(self, *args):
        raise RuntimeError(f"{self.name} is not exported by the library RST_LIB names")


class _OlderLib:
    """An explicitly selected librst (RST_LIB, same-box A/B runs of an older build) may lack newer entry points."""

    def __init__(self, lib):
        self._lib = lib
        self._missing = {}

    def __getattr__(self, name):
        try:
            return getattr(self._lib, name)
        except AttributeError:
            return self._missing.setdefault(name, _MissingSymbol(name))


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("RST_LIB", str(LIB_PATH))
    if not Path(path).exists():
        raise RuntimeError(f"librst.so not found at {path}: build it with "
                           f"`python -m realtime_style_transfer_amd.build` (there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    if "RST_LIB" in os.environ:
        lib = _OlderLib(lib)        # A/B against an older build: entry points it lacks raise when called
    vp, i, sz, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_float
    lib.rst_create.argtypes = [ctypes.POINTER(RstShape), vp, sz, ctypes.POINTER(vp)]
    lib.rst_create.restype = i
    lib.rst_create_ex.argtypes = [ctypes.POINTER(RstShape), vp, sz, i, ctypes.POINTER(vp)]
    lib.rst_create_ex.restype = i
    lib.rst_precision.argtypes = [vp]
    lib.rst_precision.restype = i
    lib.rst_destroy.argtypes = [vp]
    lib.rst_destroy.restype = None
    lib.rst_num_style_params.argtypes = [vp]
    lib.rst_num_style_params.restype = i
    lib.rst_num_weights_for_shape.argtypes = [ctypes.POINTER(RstShape)]
    lib.rst_num_weights_for_shape.restype = sz
    lib.rst_forward.argtypes = [vp, vp, vp, vp, vp, i, vp]
    lib.rst_forward.restype = i
    lib.rst_num_layers.argtypes = [vp]
    lib.rst_num_layers.restype = i
    lib.rst_layer_output_shape.argtypes = [vp, i, i, ctypes.POINTER(ctypes.c_int)]
    lib.rst_layer_output_shape.restype = i
    lib.rst_copy_activation.argtypes = [vp, i, vp, sz, i, vp]
    lib.rst_copy_activation.restype = i
    lib.rst_gram_workspace_size.argtypes = [i, i, i]
    lib.rst_gram_workspace_size.restype = sz
    lib.rst_gram.argtypes = [vp, i, i, i, vp, vp, vp]
    lib.rst_gram.restype = i
    lib.rst_instance_norm_workspace_size.argtypes = [i, i, i]
    lib.rst_instance_norm_workspace_size.restype = sz
    lib.rst_instance_norm.argtypes = [vp, i, i, i, vp, vp, fp, i, vp, vp, vp]
    lib.rst_instance_norm.restype = i
    lib.rst_style_param_map.argtypes = [vp, vp, i, i, i, i, vp, vp]
    lib.rst_style_param_map.restype = i
    lib.rst_profile_begin.argtypes = [vp, i]
    lib.rst_profile_begin.restype = i
    lib.rst_profile_end.argtypes = [vp, ctypes.POINTER(fp), ctypes.POINTER(fp), ctypes.POINTER(i)]
    lib.rst_profile_end.restype = i
    lib.rst_timeline_begin.argtypes = [vp]
    lib.rst_timeline_begin.restype = i
    lib.rst_timeline_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i]
    lib.rst_timeline_read.restype = i
    lib.rst_timeline_end.argtypes = [vp]
    lib.rst_timeline_end.restype = i
    lib.rst_layer_kernel_id.argtypes = [vp, i]
    lib.rst_layer_kernel_id.restype = i
    lib.rst_loss_num_weights.argtypes = []
    lib.rst_loss_num_weights.restype = sz
    lib.rst_loss_create.argtypes = [ctypes.POINTER(RstLossShape), vp, sz, ctypes.POINTER(vp)]
    lib.rst_loss_create.restype = i
    lib.rst_loss_destroy.argtypes = [vp]
    lib.rst_loss_destroy.restype = None
    lib.rst_loss_forward.argtypes = [vp, vp, vp, vp, i, vp, vp]
    lib.rst_loss_forward.restype = i
    lib.rst_loss_copy_feature.argtypes = [vp, i, vp, sz, i, vp]
    lib.rst_loss_copy_feature.restype = i
    lib.rst_trainer_create.argtypes = [ctypes.POINTER(RstShape), vp, sz, ctypes.POINTER(RstLossShape), vp, sz,
                                       ctypes.POINTER(vp)]
    lib.rst_trainer_create.restype = i
    lib.rst_trainer_create_ex.argtypes = [ctypes.POINTER(RstShape), vp, sz, ctypes.POINTER(RstLossShape), vp, sz, i,
                                          ctypes.POINTER(vp)]
    lib.rst_trainer_create_ex.restype = i
    lib.rst_trainer_destroy.argtypes = [vp]
    lib.rst_trainer_destroy.restype = None
    lib.rst_trainer_num_style_params.argtypes = [vp]
    lib.rst_trainer_num_style_params.restype = i
    lib.rst_trainer_num_weights.argtypes = [vp]
    lib.rst_trainer_num_weights.restype = sz
    lib.rst_trainer_compute_gradients.argtypes = [vp, vp, vp, vp, vp, i, vp, vp, vp, vp, vp]
    lib.rst_trainer_compute_gradients.restype = i
    lib.rst_trainer_compute_targets.argtypes = [vp, vp, vp, i, vp]
    lib.rst_trainer_compute_targets.restype = i
    lib.rst_trainer_apply_gradients.argtypes = [vp, vp, fp, fp, fp, vp]
    lib.rst_trainer_apply_gradients.restype = i
    lib.rst_trainer_cancel_targets.argtypes = [vp, vp]
    lib.rst_trainer_cancel_targets.restype = i
    lib.rst_trainer_wait_style_gradient.argtypes = [vp, vp]
    lib.rst_trainer_wait_style_gradient.restype = i
    for name in ("rst_trainer_copy_weights", "rst_trainer_copy_slots", "rst_trainer_set_weights",
                 "rst_trainer_set_slots"):
        getattr(lib, name).argtypes = [vp, vp, sz, vp]
        getattr(lib, name).restype = i
    lib.rst_trainer_copy_output_gradient.argtypes = [vp, i, vp, sz, i, vp]
    lib.rst_trainer_copy_output_gradient.restype = i
    lib.rst_trainer_debug_vgg_gradient.argtypes = [vp, i, vp, sz, i, vp]
    lib.rst_trainer_debug_vgg_gradient.restype = i
    for pre in ("rst_trainer", "rst_predictor_trainer"):
        getattr(lib, pre + "_num_moving_statistics").argtypes = [vp]
        getattr(lib, pre + "_num_moving_statistics").restype = sz
        getattr(lib, pre + "_get_moving_statistics").argtypes = [vp, vp, sz, vp]
        getattr(lib, pre + "_get_moving_statistics").restype = i
        getattr(lib, pre + "_set_moving_statistics").argtypes = [vp, vp, sz, fp, vp]
        getattr(lib, pre + "_set_moving_statistics").restype = i
    lib.rst_trainer_loss.argtypes = [vp]
    lib.rst_trainer_loss.restype = vp
    lib.rst_predictor_num_weights.argtypes = [ctypes.POINTER(RstPredictorShape)]
    lib.rst_predictor_num_weights.restype = sz
    lib.rst_predictor_create.argtypes = [ctypes.POINTER(RstPredictorShape), vp, sz, ctypes.POINTER(vp)]
    lib.rst_predictor_create.restype = i
    lib.rst_predictor_destroy.argtypes = [vp]
    lib.rst_predictor_destroy.restype = None
    lib.rst_predictor_forward.argtypes = [vp, vp, i, vp, vp]
    lib.rst_predictor_forward.restype = i
    lib.rst_predictor_num_stages.argtypes = [vp]
    lib.rst_predictor_num_stages.restype = i
    lib.rst_predictor_stage_shape.argtypes = [vp, i, ctypes.POINTER(ctypes.c_int)]
    lib.rst_predictor_stage_shape.restype = i
    lib.rst_predictor_copy_stage.argtypes = [vp, i, vp, sz, i, vp]
    lib.rst_predictor_copy_stage.restype = i
    lib.rst_predictor_trainer_create.argtypes = [ctypes.POINTER(RstPredictorShape), vp, sz, ctypes.POINTER(vp)]
    lib.rst_predictor_trainer_create.restype = i
    lib.rst_predictor_trainer_destroy.argtypes = [vp]
    lib.rst_predictor_trainer_destroy.restype = None
    lib.rst_predictor_trainer_num_weights.argtypes = [vp]
    lib.rst_predictor_trainer_num_weights.restype = sz
    lib.rst_predictor_trainer_forward.argtypes = [vp, vp, i, vp, vp]
    lib.rst_predictor_trainer_forward.restype = i
    lib.rst_predictor_trainer_backward.argtypes = [vp, vp, vp, vp]
    lib.rst_predictor_trainer_backward.restype = i
    lib.rst_predictor_trainer_apply_gradients.argtypes = [vp, vp, fp, fp, fp, vp]
    lib.rst_predictor_trainer_apply_gradients.restype = i
    for name in ("rst_predictor_trainer_copy_weights", "rst_predictor_trainer_set_weights",
                 "rst_predictor_trainer_copy_slots", "rst_predictor_trainer_set_slots"):
        getattr(lib, name).argtypes = [vp, vp, sz, vp]
        getattr(lib, name).restype = i
    lib.rst_gbuffer_resized_size.argtypes = [i, i, i, i, ctypes.POINTER(ctypes.c_int)]
    lib.rst_gbuffer_resized_size.restype = i
    lib.rst_gbuffer_preprocess.argtypes = [ctypes.POINTER(vp), i, i, i, ctypes.c_longlong, ctypes.c_longlong, vp, i,
                                           i, vp]
    lib.rst_gbuffer_preprocess.restype = i
    lib.rst_crc32c_extend.argtypes = [ctypes.c_uint, ctypes.c_char_p, sz]
    lib.rst_crc32c_extend.restype = ctypes.c_uint
    lib.rst_last_error.argtypes = []
    lib.rst_last_error.restype = ctypes.c_char_p
    lib.rst_version.argtypes = []
    lib.rst_version.restype = ctypes.c_char_p
    _lib = lib
    return lib


def check(code: int):
    if code != RST_OK:
        msg = load().rst_last_error().decode(errors="replace")
        if code == RST_ERR_INVALID:
            raise ValueError(f"librst: {msg}")
        raise RstError(code, msg)


def stream_ptr(stream=None) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return int(s.cuda_stream)


def as_device(x, device) -> torch.Tensor:
    """Keras-call input convenience: numpy arrays and host tensors are copied to ``device`` as float32 (the
    H2D copy Keras does for host inputs); device tensors pass through untouched."""
    if not isinstance(x, torch.Tensor):
        x = torch.from_numpy(np.ascontiguousarray(x, np.float32))
    if not x.is_cuda:
        x = x.to(device=device, dtype=torch.float32)
    return x


def dev_ptr(t: torch.Tensor) -> int:
    if not t.is_cuda:
        raise ValueError("librst operates on device tensors; got a CPU tensor")
    if t.dtype != torch.float32:
        raise ValueError(f"librst expects float32 tensors, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("librst expects contiguous (NHWC) tensors")
    return int(t.data_ptr())
