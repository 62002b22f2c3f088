"""Ops layer: HIP/CDNA4 kernels (``kernels``) and autograd-level functions (``functional``)."""
from . import functional  # noqa: F401
from ._backend import available as native_available  # noqa: F401
