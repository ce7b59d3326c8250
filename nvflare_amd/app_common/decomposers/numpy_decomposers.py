"""Drop-in FOBS numpy decomposer whose recompose returns a view over the received bytes (row f2).

Reference: ``nvflare/app_common/decomposers/numpy_decomposers.py:63-107``.  ``native_decompose`` is the
reference's (``np.save``); ``native_recompose`` parses the ``.npy`` header and returns an array VIEW of the
payload (``nvflare_amd.ingest.recompose_npy``) instead of ``np.load``'s copy, so the aggregator stages the
client's bytes straight from the message buffer into the pinned H2D ring.  Register it after NVFlare's own
decomposers (it claims the same type)::

    from nvflare_amd.app_common.decomposers import numpy_decomposers
    numpy_decomposers.register()

Arrays recomposed from ``bytes`` are read-only (see nvflare_amd/ingest.py).
"""

from __future__ import annotations

from io import BytesIO
from typing import Any

import numpy as np

from ...ingest import recompose_npy

try:  # the reference decomposer (download / streaming support) when NVFlare is installed
    from nvflare.app_common.decomposers.numpy_decomposers import NumpyArrayDecomposer as _RefNumpyArrayDecomposer
except Exception:  # pragma: no cover - exercised where nvflare is absent
    _RefNumpyArrayDecomposer = None


class _ZeroCopyRecompose:
    def native_decompose(self, target: np.ndarray, manager: Any = None) -> bytes:
        stream = BytesIO()
        np.save(stream, target, allow_pickle=False)
        return stream.getvalue()

    def native_recompose(self, data: bytes, manager: Any = None) -> np.ndarray:
        return recompose_npy(data)


if _RefNumpyArrayDecomposer is not None:

    class NumpyArrayDecomposer(_ZeroCopyRecompose, _RefNumpyArrayDecomposer):
        pass

else:

    class NumpyArrayDecomposer(_ZeroCopyRecompose):
        """Stand-in with the reference's native encode / decode methods (no FOBS streaming without NVFlare)."""

        def supported_type(self):
            return np.ndarray


def register():
    """Replace NVFlare's numpy array decomposer with the zero-copy one (no-op without NVFlare)."""
    if _RefNumpyArrayDecomposer is None:
        return
    from nvflare.fuel.utils import fobs

    fobs.register(NumpyArrayDecomposer)
