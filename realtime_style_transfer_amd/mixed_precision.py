"""Mirror of ``tf.keras.mixed_precision``'s global policy for this path.

The reference's ``train_network.py:26`` selects Keras mixed precision with one global call
(``tf.keras.mixed_precision.set_global_policy(...)``, commented out there, so its default run is float32).
BASELINE config 4 trains in bf16: ``set_global_policy('mixed_bfloat16')`` before the loss model is built makes
``StyleLossModelVGG()`` run the VGG16 convs with bf16 operands and fp32 accumulation (Keras ``mixed_bfloat16``
arithmetic, ``RST_PRECISION_BF16``), i.e. the benchmarked config-4 line through the reference-signature
construction sequence. The transfer network keeps its own (fp32-level) arithmetic under every policy, as
``make_style_transfer_training_model(precision=...)`` documents.
"""
from __future__ import annotations

_POLICIES = {"float32": "fp32", "mixed_bfloat16": "bf16"}
_global = "float32"


class Policy:
    """``tf.keras.mixed_precision.Policy`` (name, compute and variable dtypes) for the supported names."""

    def __init__(self, name: str):
        if name == "mixed_float16":
            raise NotImplementedError("mixed_float16 (fp16 operands with loss scaling) is not implemented on this "
                                      "path; use 'mixed_bfloat16' (BASELINE config 4) or 'float32'")
        if name not in _POLICIES:
            raise ValueError(f"unknown policy {name!r}; supported: {sorted(_POLICIES)}")
        self.name = name
        self.compute_dtype = "bfloat16" if name == "mixed_bfloat16" else "float32"
        self.variable_dtype = "float32"

    def __repr__(self):
        return f'<Policy "{self.name}">'


def set_global_policy(policy) -> None:
    global _global
    _global = Policy(policy.name if isinstance(policy, Policy) else str(policy)).name


def global_policy() -> Policy:
    return Policy(_global)


def loss_network_precision() -> str:
    """The VGG16 loss network's librst precision under the global policy ("fp32" or "bf16")."""
    return _POLICIES[_global]
