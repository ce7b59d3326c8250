"""Server-side dequantization of quantized client results on the device."""

from .dequantizer import ModelDequantizer  # noqa: F401
