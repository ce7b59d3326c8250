"""Drop-in FOBS tensor decomposer whose recompose returns views over the received bytes (row f2).

Reference: ``nvflare/app_opt/pt/decomposers.py:38-132`` (safetensors payloads).  ``native_recompose``
parses the safetensors header and returns a tensor VIEW of the payload (``nvflare_amd.ingest.
recompose_safetensors``) instead of ``safetensors.torch.load``'s copy.  Disk-offloaded tensors
(``lazy_tensor_dict._LazyRef``) need no decomposer change: the aggregation helper stages them from an mmap
of their file (``nvflare_amd.ingest.MappedTensor``).  Register after NVFlare's own decomposers::

    from nvflare_amd.app_opt.pt import decomposers
    decomposers.register()
"""

from __future__ import annotations

from typing import Any

import torch

from ...ingest import recompose_safetensors

try:
    from nvflare.app_opt.pt.decomposers import TensorDecomposer as _RefTensorDecomposer
except Exception:  # pragma: no cover - exercised where nvflare is absent
    _RefTensorDecomposer = None


class _ZeroCopyRecompose:
    def native_decompose(self, target: torch.Tensor, manager: Any = None) -> bytes:
        from safetensors.torch import save

        return save({"t": target})

    def native_recompose(self, data: bytes, manager: Any = None) -> torch.Tensor:
        tensors = recompose_safetensors(data)
        if "t" not in tensors:
            raise ValueError(f"failed to load data: no tensor 't' in payload (keys {list(tensors)})")
        return tensors["t"]


if _RefTensorDecomposer is not None:

    class TensorDecomposer(_ZeroCopyRecompose, _RefTensorDecomposer):
        pass

else:

    class TensorDecomposer(_ZeroCopyRecompose):
        """Stand-in with the reference's native encode / decode methods (no FOBS streaming without NVFlare)."""

        def supported_type(self):
            return torch.Tensor


def register():
    """Replace NVFlare's tensor decomposer with the zero-copy one (no-op without NVFlare)."""
    if _RefTensorDecomposer is None:
        return
    from nvflare.fuel.utils import fobs

    fobs.register(TensorDecomposer)
