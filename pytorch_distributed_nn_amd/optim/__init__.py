"""Fused flat-buffer optimizers (single-launch SGD / Adam / AdamW) and the parameter arena."""
from .flat import FlatParams, flatten_module  # noqa: F401
from .fused import SGD, Adam, AdamW  # noqa: F401
