"""PyTorch-side server components of the FedOpt path."""

from .fedopt import DeviceServerOptimizer, PTFedOptModelShareableGenerator  # noqa: F401
