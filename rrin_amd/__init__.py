"""rrin_amd — MI355X-native RRIN inference hot path (Net.forward) on HIP/CDNA4.

``from rrin_amd import Net`` gives the drop-in replacement of the reference
``model.Net`` (`/root/reference/model.py:24-65`).
"""
from .model import Net  # noqa: F401
from .unet import UNet  # noqa: F401

__all__ = ["Net", "UNet"]
