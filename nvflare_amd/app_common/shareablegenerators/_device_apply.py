"""WEIGHT_DIFF apply ``w = base + d`` on the GPU for a batch of fp32 host arrays.

``full_model_shareable_generator.py:58-67`` and ``fedopt.py:247-263`` add each aggregated difference to
its base weight with one fp32 add per element (numpy ``+`` / torch ``+``, a new array).  Here the pairs
are packed into one flat staging layout, moved to HBM, added by the fused-epilogue kernel
(``fedavg_accumulate_tiled_epi`` with no clients, the differences as ``acc_in`` and
``FEDAVG_EPI_ADD_BASE``) and returned with one D2H -- the same single rounding, so the bits match.
"""

from __future__ import annotations

import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ... import _native as N
from ...device import DeviceContext

_ALIGN = 64  # elements: 256-byte aligned pieces, as in the aggregation engine's flat key layout


class DeviceAdder:
    """Reusable staging for ``base + diff`` batches on one HIP device."""

    def __init__(self, device: Optional[int] = None):
        self._device = device
        self._ctx = None
        self._bufs = None
        self._cap = 0
        self._lock = threading.Lock()

    @property
    def ctx(self) -> DeviceContext:
        if self._ctx is None:
            self._ctx = DeviceContext.get(self._device)
        return self._ctx

    def _ensure(self, n: int) -> None:
        if self._cap >= n:
            return
        cap = max(n, 2 * self._cap, 1 << 16)
        self._bufs = [self.ctx.alloc(cap * 4) for _ in range(3)]  # base, diff, out
        self._cap = cap

    def add(self, pairs: Sequence[Tuple[np.ndarray, np.ndarray]]) -> List[np.ndarray]:
        """pairs of same-shape float32 numpy arrays -> list of new float32 arrays base + diff."""
        if not pairs:
            return []
        offs, total = [], 0
        for b, d in pairs:
            if b.dtype != np.float32 or d.dtype != np.float32 or b.shape != d.shape:
                raise TypeError("DeviceAdder: pairs must be float32 arrays of equal shape")
            offs.append(total)
            total += (b.size + _ALIGN - 1) // _ALIGN * _ALIGN
        total = max(total, _ALIGN)
        with self._lock, self.ctx.lock:
            self._ensure(total)
            base_buf, diff_buf, out_buf = self._bufs
            keep = []
            for (b, d), off in zip(pairs, offs):
                for arr, buf in ((b, base_buf), (d, diff_buf)):
                    a = np.ascontiguousarray(arr)
                    keep.append(a)
                    if a.size:
                        self.ctx.h2d_ptr(buf.ptr + off * 4, a.ctypes.data, a.nbytes)
            e = N.Epilogue()
            e.kind = N.FEDAVG_EPI_ADD_BASE
            e.base = base_buf.ptr
            self.ctx.accumulate_tiled_epi([], [], 4096, 4096, 0, total, out_buf.ptr, N.FEDAVG_OP_TORCH,
                                          N.FEDAVG_FIN_NONE, 1.0, e, acc_in_ptr=diff_buf.ptr)
            host = np.empty(total, np.float32)
            self.ctx.d2h(host, out_buf.ptr)
            del keep
        return [host[off:off + b.size].reshape(b.shape) for (b, _), off in zip(pairs, offs)]
