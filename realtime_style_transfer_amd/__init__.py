"""MI355X-native realtime style transfer (hot path of singinwhale/realtime-style-transfer).

Host-side mirror of the reference interface (ShapeConfig, create_style_transfer_model,
make_style_loss_function, ...) over librst.so — hand-written gfx950 HIP kernels behind
the C ABI in include/rst.h. See DESIGN.md.
"""
from .shape_config import ShapeConfig, StyleFeatureExtractor  # noqa: F401
from .plan import network_plan, init_weights, synthetic_style_params  # noqa: F401

__all__ = ["ShapeConfig", "StyleFeatureExtractor", "network_plan", "init_weights", "synthetic_style_params"]
