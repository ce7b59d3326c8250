"""Quantized client payloads that are dequantized ON THE DEVICE.

A ``QuantizedPayload`` stands in for one dequantized array: it keeps the compressed payload and its
quantization state on the host until the HIP library dequantizes it --

* straight into the client's slot of an aggregation slab (``engine.DeviceFedAvg.add``), so staging moves
  the compressed bytes over PCIe (1/4 of fp32 for blockwise8, 1/8 for 4-bit), or
* into a flat device buffer followed by one D2H (``materialize()``), which is what any other consumer
  gets: NVFlare's own ``WeightedAggregationHelper`` calls ``materialize()`` on such values
  (``weighted_aggregation_helper.py:170-175``).

The arithmetic per format is ``fedavg_dequantize`` (include/nvflare_amd_fedavg.h); the Python side only
moves bytes and applies the reference's final dtype cast (``dequantizer.py:162-176``).
"""

from __future__ import annotations

import threading
from typing import Optional, Tuple

import numpy as np

from . import _native as N
from .device import DeviceContext

try:
    import torch
except ImportError:  # pragma: no cover - torch is a hard dependency of the device path
    torch = None

_ALIGN = 256


def _as_numpy(a) -> np.ndarray:
    if torch is not None and isinstance(a, torch.Tensor):
        t = a.detach().cpu().contiguous()
        if t.dtype == torch.bfloat16:
            return t.view(torch.int16).numpy().view(np.uint16)
        return t.numpy()
    return np.ascontiguousarray(a)


class QuantizedPayload:
    """One quantized tensor awaiting device dequantization (see module docstring).

    Args:
        qtype: ``N.FEDAVG_Q_*``.
        payload: the quantized values (any integer / fp16 array or tensor; its bytes are what moves).
        shape: shape of the dequantized tensor.
        container: "numpy" or "torch" -- the type the reference would return.
        out_dtype: numpy dtype of the dequantized result (the parameter's source dtype).
        absmax, code, blocksize: blockwise8 / fp4 / nf4 state.
        norm, level, offset, has_norm: adaquant state.
        device: HIP device for ``materialize()`` (default $NVFLARE_AMD_DEVICE or 0).
    """

    def __init__(self, qtype: int, payload, shape: Tuple[int, ...], container: str, out_dtype=np.float32,
                 absmax=None, code=None, blocksize: int = 0, norm: float = 0.0, level: float = 1.0,
                 offset: float = 0.0, has_norm: bool = True, device: Optional[int] = None):
        self.qtype = int(qtype)
        self.payload = _as_numpy(payload)
        self.shape = tuple(int(s) for s in shape)
        self.n = int(np.prod(self.shape, dtype=np.int64)) if self.shape else 1
        self.container = container
        self.out_dtype = np.dtype(out_dtype)
        self.absmax = None if absmax is None else np.ascontiguousarray(_as_numpy(absmax), dtype=np.float32)
        self.code = None if code is None else np.ascontiguousarray(_as_numpy(code), dtype=np.float32)
        self.blocksize = int(blocksize)
        self.norm, self.level, self.offset, self.has_norm = float(norm), float(level), float(offset), bool(has_norm)
        self.device = device
        self._check()

    # array-like metadata, so the aggregation bookkeeping treats it as the array it stands for
    @property
    def dtype(self):
        if self.container == "torch":
            return {np.dtype(np.float32): torch.float32, np.dtype(np.float16): torch.float16,
                    np.dtype(np.float64): torch.float64}.get(self.out_dtype, torch.bfloat16)
        return self.out_dtype

    @property
    def nbytes(self) -> int:
        return self.payload.nbytes

    def _check(self) -> None:
        need = {N.FEDAVG_Q_F16: 2 * self.n, N.FEDAVG_Q_BF16: 2 * self.n, N.FEDAVG_Q_BLOCKWISE8: self.n,
                N.FEDAVG_Q_FP4: (self.n + 1) // 2, N.FEDAVG_Q_NF4: (self.n + 1) // 2, N.FEDAVG_Q_ADA_U8: self.n,
                N.FEDAVG_Q_ADA_U16: 2 * self.n}.get(self.qtype)
        if need is None:
            raise ValueError(f"nvflare_amd: unknown quantization type {self.qtype}")
        if self.qtype in (N.FEDAVG_Q_ADA_U8, N.FEDAVG_Q_ADA_U16) and not self.has_norm:
            need = 0
        if self.payload.nbytes < need:
            raise ValueError(f"nvflare_amd: quantized payload holds {self.payload.nbytes} bytes, {need} needed")
        if self.qtype in (N.FEDAVG_Q_BLOCKWISE8, N.FEDAVG_Q_FP4, N.FEDAVG_Q_NF4):
            if self.absmax is None or self.blocksize <= 0 or self.blocksize % 4:
                raise ValueError("nvflare_amd: blocked quantization needs absmax and a blocksize multiple of 4")
            if self.absmax.size < (self.n + self.blocksize - 1) // self.blocksize:
                raise ValueError("nvflare_amd: absmax has fewer entries than blocks")
            if self.qtype == N.FEDAVG_Q_BLOCKWISE8 and (self.code is None or self.code.size < 256):
                raise ValueError("nvflare_amd: blockwise8 needs a 256-entry code")

    def pieces(self):
        """Host byte arrays to upload: (payload, absmax, code) -- absent ones omitted."""
        out = [self.payload.reshape(-1).view(np.uint8)]
        for a in (self.absmax, self.code):
            if a is not None:
                out.append(a.reshape(-1).view(np.uint8))
        return out

    def quant_struct(self, absmax_ptr: int = 0, code_ptr: int = 0) -> "N.Quant":
        q = N.Quant()
        q.qtype = self.qtype
        q.has_norm = int(self.has_norm)
        q.blocksize = self.blocksize
        q.absmax = absmax_ptr or None
        q.code = code_ptr or None
        q.norm, q.level, q.offset = self.norm, self.level, self.offset
        return q

    def materialize(self):
        """Dequantize on the device and return the host array / tensor the reference would produce."""
        flat = _STAGER.dequantize_to_host(self)
        return finish_host_result(flat, self)


def finish_host_result(flat_f32: np.ndarray, p: QuantizedPayload):
    """fp32 dequantized values -> the reference's container and source dtype (dequantizer.py:162-176;
    fp32 -> fp16 / bf16 is one round-to-nearest-even, as numpy ``astype`` / torch ``.half()``)."""
    arr = flat_f32.reshape(p.shape)
    if p.container == "torch":
        t = torch.from_numpy(arr)
        if p.out_dtype == np.dtype(np.float16):
            t = t.half()
        elif p.out_dtype.name == "bfloat16" or p.dtype == torch.bfloat16:
            t = t.bfloat16()
        return t
    if p.out_dtype != np.dtype(np.float32):
        arr = arr.astype(p.out_dtype)
    return arr


class DeviceStager:
    """Uploads quantized payloads into a reusable device scratch and dequantizes them (one HIP device)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._scratch = {}  # device -> (DeviceBuffer, capacity)

    def _upload(self, ctx: DeviceContext, device_key, p: QuantizedPayload):
        pieces = p.pieces()
        offs, total = [], 0
        for a in pieces:
            offs.append(total)
            total += (a.nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
        buf, cap = self._scratch.get(device_key, (None, 0))
        if cap < total:
            if buf is not None:
                ctx.sync()
                buf.close()
            cap = max(total, 2 * cap, 1 << 20)
            buf = ctx.alloc(cap)
            self._scratch[device_key] = (buf, cap)
        for a, off in zip(pieces, offs):
            if a.nbytes:
                ctx.h2d_ptr(buf.ptr + off, a.ctypes.data, a.nbytes)
        ptrs = [buf.ptr + off for off in offs]
        q_ptr = ptrs[0]
        absmax_ptr = ptrs[1] if p.absmax is not None else 0
        code_ptr = ptrs[2] if p.code is not None else 0
        return q_ptr, p.quant_struct(absmax_ptr, code_ptr)

    def dequantize_into(self, ctx: DeviceContext, p: QuantizedPayload, out_ptr: int, tile: int, tile_stride: int,
                        logical_offset: int) -> None:
        """Dequantize p into a tiled fp32 destination (an aggregation slot); returns after completion."""
        with self._lock, ctx.lock:
            q_ptr, qs = self._upload(ctx, ctx.device, p)
            ctx.dequantize(qs, q_ptr, p.n, out_ptr, tile, tile_stride, logical_offset)
            ctx.sync()  # the scratch is reused by the next upload

    def dequantize_to_host(self, p: QuantizedPayload) -> np.ndarray:
        ctx = DeviceContext.get(p.device)
        n_pad = (p.n + 3) // 4 * 4
        with self._lock, ctx.lock:
            q_ptr, qs = self._upload(ctx, ctx.device, p)
            out = ctx.alloc(max(n_pad, 4) * 4)
            try:
                ctx.dequantize(qs, q_ptr, p.n, out.ptr)
                host = np.empty(p.n, np.float32)
                ctx.d2h(host, out.ptr)
            finally:
                ctx.sync()
                out.close()
        return host


_STAGER = DeviceStager()


def stager() -> DeviceStager:
    return _STAGER
