"""Device handle and device buffers over the C-ABI (one handle per HIP device, shared per process)."""

from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import Dict, Optional, Sequence

import numpy as np

from . import _native as N

# numpy has no bfloat16: the engine carries torch.bfloat16 keys as 2-byte raw values of this dtype
BF16_NP = np.dtype("V2")

_NP_TO_DT = {
    np.dtype(np.float32): N.FEDAVG_F32,
    np.dtype(np.float64): N.FEDAVG_F64,
    np.dtype(np.int32): N.FEDAVG_I32,
    np.dtype(np.int64): N.FEDAVG_I64,
    np.dtype(np.float16): N.FEDAVG_F16,
    BF16_NP: N.FEDAVG_BF16,
    np.dtype(np.uint8): N.FEDAVG_U8,
    np.dtype(np.int8): N.FEDAVG_I8,
    np.dtype(np.int16): N.FEDAVG_I16,
    np.dtype(np.bool_): N.FEDAVG_BOOL,
    np.dtype(np.uint16): N.FEDAVG_U16,
    np.dtype(np.uint32): N.FEDAVG_U32,
    np.dtype(np.uint64): N.FEDAVG_U64,
}


def fedavg_dtype(dt) -> int:
    dt = np.dtype(dt)
    if dt not in _NP_TO_DT:
        raise TypeError(f"nvflare_amd: dtype {dt} has no device kernel")
    return _NP_TO_DT[dt]


class TiledLayout:
    """Geometry of a tiled client slab (fedavg_accumulate_tiled in include/nvflare_amd_fedavg.h).

    A slab holds `slots` clients; element i of the client in slot s is at
        s * tile + (i // tile) * tile_stride + i % tile,   tile_stride = slots * tile
    so each tile's client segments are contiguous in HBM."""

    __slots__ = ("tile", "slots", "tile_stride")

    def __init__(self, tile: int, slots: int):
        self.tile = int(tile)
        self.slots = int(slots)
        self.tile_stride = self.slots * self.tile

    def n_tiles(self, n: int) -> int:
        return (int(n) + self.tile - 1) // self.tile

    def slab_elems(self, n: int) -> int:
        return self.n_tiles(n) * self.tile_stride

    def slot_offset_elems(self, slot: int) -> int:
        return int(slot) * self.tile

    def __repr__(self):
        return f"TiledLayout(tile={self.tile}, slots={self.slots}, tile_stride={self.tile_stride})"


class _Lease:
    """Buffer owner of one ``HostArenaPool.take``: the handed-out array is made over this non-array object,
    so numpy's collapse of a view's ``base`` chain stops at that array (it never skips to the pooled
    storage).  Every slice, reshape and ``torch.from_numpy`` of it therefore references the handed-out
    array, which dies exactly when the last of them does."""

    __slots__ = ("storage", "__array_interface__")

    def __init__(self, storage: np.ndarray):
        self.storage = storage
        self.__array_interface__ = storage.__array_interface__


class HostArenaPool:
    """Host result arrays reused across rounds once nothing else references them.

    Each round returns its results as views of one fresh host array (numpy results of the reference are
    new arrays).  A fresh array costs a page fault per 4 KiB page during the D2H (≈150 ms single-threaded
    for 500 MB); the pool keeps the last ``depth`` arrays and hands one out again only when no view of it
    is alive.  In scatter-and-gather the previous round's result is still referenced while the next one is
    computed, so ``depth`` = 3 lets round r reuse the array of round r - 2.

    Liveness is tracked explicitly, not by reference-count arithmetic: every take() hands out a fresh
    array over the pooled storage (through a ``_Lease``), and the storage is free again once that array's
    weak reference is dead."""

    PIN_MIN_BYTES = 16 << 20  # smaller results are cheaper through the pinned ring than to register

    def __init__(self, depth: int = 3):
        self._arrs: list = []  # [storage ndarray, weakref to the array last handed out over it]
        self._depth = depth
        self._lock = threading.Lock()

    def take(self, n: int, dtype=np.float32, pin: Optional["DeviceContext"] = None) -> np.ndarray:
        """A host array of n elements.  With ``pin``, a new array of at least PIN_MIN_BYTES is page-locked
        through that context (once; it stays registered while the pool reuses it), so D2H copies into it
        run at the PCIe rate without the pinned ring's extra host copy; it is unregistered just before
        its memory is freed (when the pool has dropped it and no view of it is left)."""
        dtype = np.dtype(dtype)
        with self._lock:
            for i in range(len(self._arrs)):
                storage, ref = self._arrs[i]
                if storage.size == n and storage.dtype == dtype and ref() is None:
                    self._arrs.pop(i)
                    return self._lease(storage)  # most recently used last
            storage = np.empty(n, dtype=dtype)
            if pin is not None and storage.nbytes >= self.PIN_MIN_BYTES:
                try:
                    pin.host_register(storage)
                except N.FedAvgError:  # e.g. a locked-memory limit: the copies go through the pinned ring
                    pass
            out = self._lease(storage)
            if len(self._arrs) > self._depth:
                self._arrs.pop(0)
            return out

    def _lease(self, storage: np.ndarray) -> np.ndarray:
        arr = np.asarray(_Lease(storage))
        assert isinstance(arr.base, _Lease) and arr.ctypes.data == storage.ctypes.data
        self._arrs.append([storage, weakref.ref(arr)])
        return arr


class DeviceBuffer:
    """Device memory owned through a DeviceContext; freed on close() or garbage collection."""

    __slots__ = ("ctx", "ptr", "nbytes", "_fin", "__weakref__")

    def __init__(self, ctx: "DeviceContext", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p(0)
        N.call("fedavg_malloc", ctx.handle, ctypes.c_size_t(self.nbytes), ctypes.byref(p))
        self.ptr = p.value or 0
        self._fin = weakref.finalize(self, DeviceContext._free_ptr, ctx, self.ptr)

    def close(self) -> None:
        if self._fin.alive:
            self._fin()
        self.ptr = 0

    def __repr__(self) -> str:
        return f"DeviceBuffer(ptr=0x{self.ptr:x}, nbytes={self.nbytes}, device={self.ctx.device})"


class DeviceContext:
    """Python view of a fedavg_ctx (C-ABI handle) bound to one device."""

    _instances: Dict[int, "DeviceContext"] = {}
    _instances_lock = threading.Lock()

    def __init__(self, device: int = 0):
        self.device = int(device)
        h = ctypes.c_void_p(0)
        N.call("fedavg_create", ctypes.c_int(self.device), ctypes.byref(h))
        self.handle = h.value
        self.lock = threading.RLock()
        ncu = ctypes.c_int(0)
        free = ctypes.c_size_t(0)
        total = ctypes.c_size_t(0)
        N.call("fedavg_device_info", self.handle, ctypes.byref(ncu), ctypes.byref(free), ctypes.byref(total))
        self.num_cus = ncu.value
        self.total_bytes = total.value

    # -- shared per-process handles ------------------------------------------------------------
    @classmethod
    def get(cls, device: Optional[int] = None) -> "DeviceContext":
        """The process-wide context of a HIP device (None: $NVFLARE_AMD_DEVICE, default 0)."""
        if device is None:
            device = int(os.environ.get("NVFLARE_AMD_DEVICE", "0"))
        device = int(device)
        with cls._instances_lock:
            ctx = cls._instances.get(device)
            if ctx is None:
                ctx = cls(device)
                cls._instances[device] = ctx
            return ctx

    @staticmethod
    def _free_ptr(ctx: "DeviceContext", ptr: int) -> None:
        if ptr and ctx.handle:
            try:
                N.call("fedavg_free", ctx.handle, ctypes.c_void_p(ptr))
            except Exception:
                pass

    def close(self) -> None:
        if self.handle:
            N.call("fedavg_destroy", self.handle)
            self.handle = None

    # -- memory / copies -------------------------------------------------------------------------
    def mem_info(self):
        free = ctypes.c_size_t(0)
        total = ctypes.c_size_t(0)
        N.call("fedavg_device_info", self.handle, None, ctypes.byref(free), ctypes.byref(total))
        return free.value, total.value

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def h2d(self, dst_ptr: int, host: np.ndarray) -> None:
        host = np.ascontiguousarray(host)
        if host.nbytes:
            N.call("fedavg_h2d", self.handle, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(host.ctypes.data),
                   ctypes.c_size_t(host.nbytes))

    def h2d_ptr(self, dst_ptr: int, src_ptr: int, nbytes: int) -> None:
        if nbytes:
            N.call("fedavg_h2d", self.handle, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), ctypes.c_size_t(nbytes))

    def d2h(self, host: np.ndarray, src_ptr: int) -> None:
        if not host.flags.c_contiguous:
            raise ValueError("d2h destination must be C-contiguous")
        if host.nbytes:
            N.call("fedavg_d2h", self.handle, ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(src_ptr),
                   ctypes.c_size_t(host.nbytes))

    def host_register(self, arr: np.ndarray) -> None:
        """Page-lock ``arr``'s memory until it is garbage-collected (unregistered first: numpy clears an
        array's weak references before it frees the data)."""
        ptr = arr.ctypes.data
        N.call("fedavg_host_register", self.handle, ctypes.c_void_p(ptr), ctypes.c_size_t(arr.nbytes))
        fin = weakref.finalize(arr, DeviceContext._unregister_ptr, self, ptr)
        fin.atexit = False  # at exit the process's memory goes with it

    @staticmethod
    def _unregister_ptr(ctx: "DeviceContext", ptr: int) -> None:
        try:
            N.call("fedavg_host_unregister", ctx.handle, ctypes.c_void_p(ptr))
        except Exception:  # pragma: no cover - nothing useful to do while an array is being freed
            pass

    def mark(self, ready_bytes: int) -> None:
        """Record that bytes [0, ready_bytes) of the next d2h_marked source are final after the work so far."""
        N.call("fedavg_mark", self.handle, ctypes.c_size_t(int(ready_bytes)))

    def marks_reset(self) -> None:
        """Drop recorded marks (start of a new marked sequence, or a copy that will not happen)."""
        N.call("fedavg_marks_reset", self.handle)

    def d2h_multi(self, host: np.ndarray, dev_ptr: int, pieces) -> None:
        """Device -> host copies in one call: ``pieces`` = [(host byte offset, device byte offset, nbytes)]
        from ``dev_ptr`` into ``host`` (C-contiguous); returns when the host holds them (fedavg_d2h_multi)."""
        if not host.flags.c_contiguous:
            raise ValueError("d2h destination must be C-contiguous")
        pieces = [p for p in pieces if p[2]]
        for ho, _, nb in pieces:
            if ho < 0 or ho + nb > host.nbytes:
                raise ValueError("d2h_multi piece outside the host array")
        n = len(pieces)
        if not n:
            return
        arr = (ctypes.c_size_t * n)
        N.call("fedavg_d2h_multi", self.handle, ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(dev_ptr),
               ctypes.c_int(n), arr(*[p[0] for p in pieces]), arr(*[p[1] for p in pieces]), arr(*[p[2] for p in pieces]))

    def d2h_marked(self, host: np.ndarray, src_ptr: int) -> None:
        """D2H overlapping the launches still producing src (see mark); returns when host is filled."""
        if not host.flags.c_contiguous:
            raise ValueError("d2h_marked needs a C-contiguous host array")
        N.call("fedavg_d2h_marked", self.handle, ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(src_ptr),
               ctypes.c_size_t(host.nbytes))

    def d2h_ptr(self, dst_ptr: int, src_ptr: int, nbytes: int) -> None:
        if nbytes:
            N.call("fedavg_d2h", self.handle, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), ctypes.c_size_t(nbytes))

    def d2d(self, dst_ptr: int, src_ptr: int, nbytes: int) -> None:
        if nbytes:
            N.call("fedavg_d2d", self.handle, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), ctypes.c_size_t(nbytes))

    def memset(self, dst_ptr: int, value: int, nbytes: int) -> None:
        if nbytes:
            N.call("fedavg_memset", self.handle, ctypes.c_void_p(dst_ptr), ctypes.c_int(value), ctypes.c_size_t(nbytes))

    def sync(self) -> None:
        N.call("fedavg_sync", self.handle)

    def set_stream(self, stream_ptr: Optional[int]) -> None:
        N.call("fedavg_set_stream", self.handle, ctypes.c_void_p(stream_ptr or 0))

    def stream(self) -> int:
        s = ctypes.c_void_p(0)
        N.call("fedavg_get_stream", self.handle, ctypes.byref(s))
        return s.value or 0

    # -- compute ---------------------------------------------------------------------------------
    def accumulate(
        self,
        rows: Sequence[int],
        weights: Sequence[float],
        n: int,
        out_ptr: int,
        in_dtype: int,
        acc_dtype: int,
        op: int,
        fin: int,
        count: float = 1.0,
        acc_in_ptr: Optional[int] = None,
    ) -> None:
        k = len(rows)
        rows_arr = (ctypes.c_void_p * max(k, 1))(*rows)
        w_arr = (ctypes.c_double * max(k, 1))(*[float(w) for w in weights])
        N.call(
            "fedavg_accumulate",
            self.handle,
            rows_arr,
            w_arr,
            ctypes.c_int(k),
            ctypes.c_void_p(acc_in_ptr or 0),
            ctypes.c_void_p(out_ptr),
            ctypes.c_size_t(n),
            ctypes.c_int(in_dtype),
            ctypes.c_int(acc_dtype),
            ctypes.c_int(op),
            ctypes.c_int(fin),
            ctypes.c_double(float(count)),
        )

    def accumulate_tiled(self, bases: Sequence[int], weights: Sequence[float], tile: int, tile_stride: int,
                         begin: int, end: int, out_ptr: int, op: int, fin: int, count: float = 1.0,
                         acc_in_ptr: Optional[int] = None) -> None:
        k = len(bases)
        b_arr = (ctypes.c_void_p * max(k, 1))(*bases)
        w_arr = (ctypes.c_double * max(k, 1))(*[float(w) for w in weights])
        N.call("fedavg_accumulate_tiled", self.handle, b_arr, w_arr, ctypes.c_int(k), ctypes.c_size_t(tile),
               ctypes.c_size_t(tile_stride), ctypes.c_size_t(begin), ctypes.c_size_t(end),
               ctypes.c_void_p(acc_in_ptr or 0), ctypes.c_void_p(out_ptr), ctypes.c_int(op), ctypes.c_int(fin),
               ctypes.c_double(float(count)))

    def accumulate_tiled16(self, fmt: int, bases: Sequence[int], weights: Sequence[float], tile: int, tile_stride: int,
                           begin: int, end: int, out_ptr: int, op: int, fin: int, count: float = 1.0,
                           acc_in_ptr: Optional[int] = None, tails: Optional[np.ndarray] = None) -> None:
        """fedavg_accumulate_tiled16(_tails): ``tails`` = sorted int64 flat indices taking torch's scalar-remainder
        step (torch16.scalar_tail_indices), or None."""
        k = len(bases)
        b_arr = (ctypes.c_void_p * max(k, 1))(*bases)
        w_arr = (ctypes.c_double * max(k, 1))(*[float(w) for w in weights])
        args = (self.handle, ctypes.c_int(fmt), b_arr, w_arr, ctypes.c_int(k), ctypes.c_size_t(tile),
                ctypes.c_size_t(tile_stride), ctypes.c_size_t(begin), ctypes.c_size_t(end),
                ctypes.c_void_p(acc_in_ptr or 0), ctypes.c_void_p(out_ptr), ctypes.c_int(op), ctypes.c_int(fin),
                ctypes.c_double(float(count)))
        if tails is None or len(tails) == 0:
            N.call("fedavg_accumulate_tiled16", *args)
            return
        t = np.ascontiguousarray(tails, dtype=np.int64)
        N.call("fedavg_accumulate_tiled16_tails", *args, ctypes.c_void_p(t.ctypes.data), ctypes.c_size_t(t.size))

    def accumulate_tiled64(self, bases: Sequence[int], weights: Sequence[float], tile: int, tile_stride: int,
                           begin: int, end: int, out_ptr: int, op: int, fin: int, count: float = 1.0,
                           acc_in_ptr: Optional[int] = None) -> None:
        k = len(bases)
        b_arr = (ctypes.c_void_p * max(k, 1))(*bases)
        w_arr = (ctypes.c_double * max(k, 1))(*[float(w) for w in weights])
        N.call("fedavg_accumulate_tiled64", self.handle, b_arr, w_arr, ctypes.c_int(k), ctypes.c_size_t(tile),
               ctypes.c_size_t(tile_stride), ctypes.c_size_t(begin), ctypes.c_size_t(end),
               ctypes.c_void_p(acc_in_ptr or 0), ctypes.c_void_p(out_ptr), ctypes.c_int(op), ctypes.c_int(fin),
               ctypes.c_double(float(count)))

    def accumulate_tiled_epi(self, bases: Sequence[int], weights: Sequence[float], tile: int, tile_stride: int,
                             begin: int, end: int, out_ptr: Optional[int], op: int, fin: int, count: float,
                             epilogue: "N.Epilogue", acc_in_ptr: Optional[int] = None) -> None:
        if epilogue.torch_sqrt == N.FEDAVG_SQRT_TORCH_AMD:
            self.load_rsqrtps()
        k = len(bases)
        b_arr = (ctypes.c_void_p * max(k, 1))(*bases)
        w_arr = (ctypes.c_double * max(k, 1))(*[float(w) for w in weights])
        N.call("fedavg_accumulate_tiled_epi", self.handle, b_arr, w_arr, ctypes.c_int(k), ctypes.c_size_t(tile),
               ctypes.c_size_t(tile_stride), ctypes.c_size_t(begin), ctypes.c_size_t(end),
               ctypes.c_void_p(acc_in_ptr or 0), ctypes.c_void_p(out_ptr or 0), ctypes.c_int(op), ctypes.c_int(fin),
               ctypes.c_double(float(count)), ctypes.cast(ctypes.pointer(epilogue), ctypes.c_void_p))

    def h2d_tiled(self, base_ptr: int, tile_bytes: int, tile_stride_bytes: int, logical_offset: int, src_ptr: int,
                  nbytes: int) -> None:
        if nbytes:
            N.call("fedavg_h2d_tiled", self.handle, ctypes.c_void_p(base_ptr), ctypes.c_size_t(tile_bytes),
                   ctypes.c_size_t(tile_stride_bytes), ctypes.c_size_t(logical_offset), ctypes.c_void_p(src_ptr),
                   ctypes.c_size_t(nbytes))

    def h2d_tiled_multi(self, base_ptr: int, tile_bytes: int, tile_stride_bytes: int, pieces) -> None:
        """pieces: [(logical_byte_offset, src_ptr, nbytes)] sorted by offset, non-overlapping."""
        n = len(pieces)
        if not n:
            return
        offs = (ctypes.c_size_t * n)(*[p[0] for p in pieces])
        srcs = (ctypes.c_void_p * n)(*[p[1] for p in pieces])
        lens = (ctypes.c_size_t * n)(*[p[2] for p in pieces])
        N.call("fedavg_h2d_tiled_multi", self.handle, ctypes.c_void_p(base_ptr), ctypes.c_size_t(tile_bytes),
               ctypes.c_size_t(tile_stride_bytes), ctypes.c_int(n), offs, srcs, lens)

    def d2d_tiled(self, base_ptr: int, tile_bytes: int, tile_stride_bytes: int, logical_offset: int, src_ptr: int,
                  nbytes: int) -> None:
        if nbytes:
            N.call("fedavg_d2d_tiled", self.handle, ctypes.c_void_p(base_ptr), ctypes.c_size_t(tile_bytes),
                   ctypes.c_size_t(tile_stride_bytes), ctypes.c_size_t(logical_offset), ctypes.c_void_p(src_ptr),
                   ctypes.c_size_t(nbytes))

    def set_timing(self, enable: bool) -> None:
        N.call("fedavg_set_timing", self.handle, ctypes.c_int(1 if enable else 0))

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float(0.0)
        N.call("fedavg_last_kernel_ms", self.handle, ctypes.byref(ms))
        return float(ms.value)

    def timing_begin(self) -> None:
        N.call("fedavg_timing_begin", self.handle)

    def timing_end(self) -> float:
        ms = ctypes.c_float(0.0)
        N.call("fedavg_timing_end", self.handle, ctypes.byref(ms))
        return float(ms.value)

    def launch_count(self) -> int:
        """Kernel launches issued on this context's compute stream so far (fedavg_launch_count)."""
        n = ctypes.c_uint64(0)
        N.call("fedavg_launch_count", self.handle, ctypes.byref(n))
        return int(n.value)

    def set_launch(self, blocks_per_cu: int = 0, unroll: int = 0) -> None:
        N.call("fedavg_set_launch", self.handle, ctypes.c_int(blocks_per_cu), ctypes.c_int(unroll))

    def set_variant(self, variant: int = 0) -> None:
        N.call("fedavg_set_variant", self.handle, ctypes.c_int(variant))
        self._variant = int(variant)  # what ab_build() restores

    def ab_build(self) -> bool:
        """Whether the loaded library is an A/B build (tools/build_rev_lib.py, -DFEDAVG_AB): it accepts the A/B-only
        launch variants, tile widths and unrolls, which a product library refuses (round 5).  Probed with variant
        bit 5, then the context's variant is restored to what it was (not reset to 0)."""
        prev = getattr(self, "_variant", 0)
        try:
            N.call("fedavg_set_variant", self.handle, ctypes.c_int(32))
        except N.FedAvgError:
            return False
        finally:
            N.call("fedavg_set_variant", self.handle, ctypes.c_int(prev))
        return True

    def dequantize(self, quant: "N.Quant", q_ptr: int, n: int, out_ptr: int, tile: int = 0, tile_stride: int = 0,
                   logical_offset: int = 0) -> None:
        """Dequantize n elements of the device payload at q_ptr into fp32 (fedavg_dequantize)."""
        if n:
            N.call("fedavg_dequantize", self.handle, ctypes.cast(ctypes.pointer(quant), ctypes.c_void_p),
                   ctypes.c_void_p(q_ptr), ctypes.c_size_t(n), ctypes.c_void_p(out_ptr), ctypes.c_size_t(tile),
                   ctypes.c_size_t(tile_stride), ctypes.c_size_t(logical_offset))

    def fill_synthetic_f32(self, dst_ptr: int, n: int, seed: int, row: int, col0: int = 0, tile: int = 0,
                           tile_stride: int = 0) -> None:
        N.call("fedavg_fill_synthetic_f32", self.handle, ctypes.c_void_p(dst_ptr), ctypes.c_size_t(n),
               ctypes.c_size_t(tile), ctypes.c_size_t(tile_stride), ctypes.c_uint64(seed), ctypes.c_uint64(row),
               ctypes.c_uint64(col0))

    def set_tile(self, tile: int = 0) -> None:
        N.call("fedavg_set_tile", self.handle, ctypes.c_int(tile))

    def sqrt_f32(self, x_ptr: int, out_ptr: int, n: int, torch_sqrt=False) -> None:
        """out[i] = the epilogues' sqrt of x[i] (device pointers).  ``torch_sqrt``: a FEDAVG_SQRT_* value, or a bool
        (True: torch CPU's AVX-512 vsSqrt, False: the correctly rounded sqrt).  Test entry."""
        if int(torch_sqrt) == N.FEDAVG_SQRT_TORCH_AMD:
            self.load_rsqrtps()
        N.call("fedavg_sqrt_f32", self.handle, ctypes.c_void_p(x_ptr), ctypes.c_void_p(out_ptr), ctypes.c_size_t(n),
               ctypes.c_int(int(torch_sqrt)))

    def load_rsqrtps(self, table: Optional[np.ndarray] = None) -> None:
        """Upload the RSQRTPS table FEDAVG_SQRT_TORCH_AMD reads (fedavg_set_rsqrtps_table): ``table`` (kept until the
        next upload), or -- when the context has none yet -- THIS host CPU's estimates captured at run time
        (torch_sqrt.host_rsqrtps_table)."""
        if table is None and getattr(self, "_rsqrtps_loaded", False):
            return
        from . import torch_sqrt

        t = np.ascontiguousarray(torch_sqrt.host_rsqrtps_table() if table is None else table, dtype=np.uint16)
        with self.lock:
            N.call("fedavg_set_rsqrtps_table", self.handle, ctypes.c_void_p(t.ctypes.data), ctypes.c_size_t(t.size))
            self._rsqrtps_loaded = True

    def gather_f32(self, src_ptr: int, idx: np.ndarray) -> np.ndarray:
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        out = np.empty(idx.size, dtype=np.float32)
        N.call("fedavg_gather_f32", self.handle, ctypes.c_void_p(src_ptr), ctypes.c_void_p(idx.ctypes.data),
               ctypes.c_size_t(idx.size), ctypes.c_void_p(out.ctypes.data))
        return out
