"""Device engine behind the drop-in WeightedAggregationHelper.

Reference semantics: nvflare/app_common/aggregators/weighted_aggregation_helper.py:153-240.
Design:

* Every ``add`` STAGES the contributor's arrays into HBM (H2D for host arrays, D2D for device
  tensors): nothing is computed on the host and the caller's arrays are never aliased
  (``:181-199``).  fp32 keys of one contribution share one *slot*: a device buffer laid out by a
  process-wide per-helper key layout (each key at a 256-byte aligned element offset), so the K slots of
  a round form the stacked ``[K][P]`` client matrix the kernel streams.  Other dtypes (fp64, int32,
  int64) get a buffer per key per contribution and go through the generic kernel.
* ``get_result`` launches the arrival-ordered K-way accumulate-and-finalise kernel over every run of
  keys that share the same contributor list (one launch for the usual all-keys-from-all-clients case),
  then copies the results back in one D2H.
* If the resident slots would exceed the budget (``max_resident_bytes``, default 85 % of HBM), the
  pending slots are FOLDED into a device accumulator (same kernel, ``FIN_NONE``) and recycled; the
  per-element operation sequence is unchanged, so the bits are too.

Numerics are the reference's, per container type (finding 2):
numpy -> ``FEDAVG_OP_NUMPY`` + ``FEDAVG_FIN_SCALE``; torch -> ``FEDAVG_OP_TORCH`` + ``FEDAVG_FIN_DIV``;
``weigh_by_local_iter=False`` -> ``FEDAVG_OP_UNWEIGHTED``.
"""

from __future__ import annotations

import os
import threading
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import _native as N
from .device import DeviceBuffer, DeviceContext, fedavg_dtype

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

ALIGN_ELEMS = 64  # 256 B for fp32: every key starts on a 256-byte boundary inside a slot

_TORCH_TO_NP = {}
if torch is not None:
    _TORCH_TO_NP = {
        torch.float32: np.dtype(np.float32),
        torch.float64: np.dtype(np.float64),
        torch.int32: np.dtype(np.int32),
        torch.int64: np.dtype(np.int64),
    }
    _NP_TO_TORCH = {v: k for k, v in _TORCH_TO_NP.items()}


def is_torch_tensor(v) -> bool:
    return torch is not None and isinstance(v, torch.Tensor)


def is_device_array(v) -> bool:
    """Arrays/tensors that take the HIP path; everything else (python numbers, opaque objects such as
    HE ciphertexts) follows the reference's object protocol on the host."""
    return isinstance(v, np.ndarray) or is_torch_tensor(v)


class _Staged:
    """One contribution's device copy of one key (or its place inside a slot)."""

    __slots__ = ("ptr", "weight", "owner")

    def __init__(self, ptr: int, weight: float, owner):
        self.ptr = ptr
        self.weight = weight
        self.owner = owner  # _Slot or DeviceBuffer keeping the memory alive


class _Slot:
    """One contribution's fp32 arena (all its fp32 keys at their layout offsets)."""

    __slots__ = ("buf", "refs")

    def __init__(self, buf: DeviceBuffer):
        self.buf = buf
        self.refs = 0


class _KeyState:
    __slots__ = (
        "name",
        "shape",
        "container",
        "torch_device",
        "in_np",
        "acc_np",
        "op",
        "fin",
        "n",
        "arena",
        "offset",
        "pending",
        "acc_valid",
        "acc_buf",
        "count",
    )

    def __init__(self):
        self.pending: List[_Staged] = []
        self.acc_valid = False
        self.acc_buf: Optional[DeviceBuffer] = None
        self.count = None

    @property
    def in_dt(self):
        return fedavg_dtype(self.in_np)

    @property
    def acc_dt(self):
        return fedavg_dtype(self.acc_np)


def _resolve_types(v, weight, weighted: bool) -> Tuple[str, np.dtype, np.dtype, int, int]:
    """(container, input dtype, accumulator/result dtype, op, fin) as the reference's numpy / torch
    arithmetic would produce them (weighted_aggregation_helper.py:181-216, :233-236)."""
    if is_torch_tensor(v):
        tdt = v.dtype
        if tdt not in _TORCH_TO_NP:
            raise TypeError(f"nvflare_amd: torch dtype {tdt} is not supported by the device kernels")
        in_np = _TORCH_TO_NP[tdt]
        if in_np.kind == "i":
            if not weighted:
                # reference: v.clone() stays integer and div_(count) raises on an integer tensor
                raise TypeError("nvflare_amd: integer tensors need weigh_by_local_iter=True (reference raises in div_)")
            acc_np = _TORCH_TO_NP[torch.get_default_dtype()]
        else:
            acc_np = in_np
        op = N.FEDAVG_OP_TORCH if weighted else N.FEDAVG_OP_UNWEIGHTED
        return "torch", in_np, acc_np, op, N.FEDAVG_FIN_DIV
    in_np = np.dtype(v.dtype)
    if in_np not in (np.dtype(np.float32), np.dtype(np.float64), np.dtype(np.int32), np.dtype(np.int64)):
        raise TypeError(f"nvflare_amd: numpy dtype {in_np} is not supported by the device kernels")
    if weighted:
        if isinstance(weight, np.generic):
            acc_np = np.result_type(in_np, np.dtype(type(weight)))
        elif isinstance(weight, (bool, int)) and in_np.kind == "i":
            raise TypeError("nvflare_amd: integer arrays with an integer weight accumulate in integers; unsupported")
        else:
            acc_np = np.result_type(in_np, 1.0)  # NEP 50: python float is weak
        op = N.FEDAVG_OP_NUMPY
    else:
        if in_np.kind == "i":
            raise TypeError("nvflare_amd: integer arrays need weigh_by_local_iter=True")
        if isinstance(weight, np.generic):
            raise TypeError("nvflare_amd: numpy-scalar weights with weigh_by_local_iter=False change the result dtype; unsupported")
        acc_np = in_np
        op = N.FEDAVG_OP_UNWEIGHTED
    acc_np = np.dtype(acc_np)
    if acc_np not in (np.dtype(np.float32), np.dtype(np.float64)):
        raise TypeError(f"nvflare_amd: accumulator dtype {acc_np} unsupported")
    return "numpy", in_np, acc_np, op, N.FEDAVG_FIN_SCALE


def _default_budget(ctx: DeviceContext) -> int:
    env = os.environ.get("NVFLARE_AMD_MAX_RESIDENT_BYTES")
    if env:
        return int(float(env))
    return int(ctx.total_bytes * 0.85)


class DeviceFedAvg:
    """Arrival-ordered weighted accumulation of client arrays on one HIP device."""

    def __init__(self, device: Optional[int] = None, max_resident_bytes: Optional[int] = None):
        if device is None:
            device = int(os.environ.get("NVFLARE_AMD_DEVICE", "0"))
        self.device = int(device)
        self._ctx: Optional[DeviceContext] = None  # opened on first use (config checks need no GPU)
        self._max_resident_bytes = max_resident_bytes
        self.lock = threading.RLock()
        self.layout_elems = 0  # fp32 arena layout size (elements)
        self.keys: Dict[str, _KeyState] = {}
        self.arena_acc: Optional[DeviceBuffer] = None
        self._free_slots: List[DeviceBuffer] = []
        self._live_slots: List[_Slot] = []
        self._side_bufs: List[DeviceBuffer] = []
        self.stats = {"h2d_bytes": 0, "folds": 0, "launches": 0}

    @property
    def ctx(self) -> DeviceContext:
        if self._ctx is None:
            self._ctx = DeviceContext.get(self.device)
        return self._ctx

    @property
    def max_resident_bytes(self) -> int:
        if self._max_resident_bytes is None:
            self._max_resident_bytes = _default_budget(self.ctx)
        return self._max_resident_bytes

    # ------------------------------------------------------------------ memory accounting
    def _resident_bytes(self) -> int:
        live = sum(s.buf.nbytes for s in self._live_slots)
        side = sum(b.nbytes for b in self._side_bufs)
        acc = self.arena_acc.nbytes if self.arena_acc is not None else 0
        return live + side + acc + sum(b.nbytes for b in self._free_slots)

    def _acquire_slot(self, nbytes: int) -> _Slot:
        best = None
        for i, b in enumerate(self._free_slots):
            if b.nbytes >= nbytes and (best is None or b.nbytes < self._free_slots[best].nbytes):
                best = i
        if best is not None:
            return _Slot(self._free_slots.pop(best))
        if self._resident_bytes() + nbytes > self.max_resident_bytes:
            self._fold()
            while self._free_slots and self._resident_bytes() + nbytes > self.max_resident_bytes:
                self._free_slots.pop().close()
            for i, b in enumerate(self._free_slots):
                if b.nbytes >= nbytes:
                    return _Slot(self._free_slots.pop(i))
        try:
            return _Slot(self.ctx.alloc(nbytes))
        except N.FedAvgError:
            self._fold()
            for b in self._free_slots:
                b.close()
            self._free_slots.clear()
            return _Slot(self.ctx.alloc(nbytes))

    def _release_slot(self, slot: _Slot) -> None:
        if slot in self._live_slots:
            self._live_slots.remove(slot)
            self._free_slots.append(slot.buf)

    # ------------------------------------------------------------------ layout
    def _register_key(self, name: str, v, weight, weighted: bool) -> _KeyState:
        container, in_np, acc_np, op, fin = _resolve_types(v, weight, weighted)
        st = self.keys.get(name)
        shape = tuple(v.shape)
        if st is not None:
            if st.container != container or st.in_np != in_np or st.acc_np != acc_np:
                raise TypeError(
                    f"nvflare_amd: key {name!r} changed type between contributions "
                    f"({st.container}/{st.in_np} -> {container}/{in_np}); unsupported"
                )
            if st.shape != shape:
                raise ValueError(f"nvflare_amd: key {name!r} shape {shape} != first contribution's {st.shape}")
            return st
        st = _KeyState()
        st.name = name
        st.shape = shape
        st.container = container
        st.torch_device = v.device if (is_torch_tensor(v) and v.device.type != "cpu") else None
        st.in_np = in_np
        st.acc_np = acc_np
        st.op = op
        st.fin = fin
        st.n = int(np.prod(shape, dtype=np.int64)) if shape else 1
        st.arena = in_np == np.dtype(np.float32) and acc_np == np.dtype(np.float32)
        if st.arena:
            st.offset = self.layout_elems
            self.layout_elems += (st.n + ALIGN_ELEMS - 1) // ALIGN_ELEMS * ALIGN_ELEMS
        else:
            st.offset = -1
        self.keys[name] = st
        return st

    def _ensure_arena_acc(self) -> None:
        need = self.layout_elems * 4
        if self.arena_acc is not None and self.arena_acc.nbytes >= need:
            return
        new = self.ctx.alloc(max(need, 4))
        if self.arena_acc is not None:
            self.ctx.d2d(new.ptr, self.arena_acc.ptr, self.arena_acc.nbytes)
            self.ctx.sync()
            self.arena_acc.close()
        self.arena_acc = new

    # ------------------------------------------------------------------ staging
    def _stage(self, dst_ptr: int, v) -> None:
        if is_torch_tensor(v):
            t = v.detach()
            if not t.is_contiguous():
                t = t.contiguous()
            nbytes = t.numel() * t.element_size()
            if t.device.type == "cpu":
                self.ctx.h2d_ptr(dst_ptr, t.data_ptr(), nbytes)
            else:
                if t.device.index != self.ctx.device:
                    raise ValueError(f"nvflare_amd: tensor on {t.device}, engine on device {self.ctx.device}")
                # order the copy after the producer's work on torch's current stream
                torch.cuda.current_stream(t.device).synchronize()
                self.ctx.d2d(dst_ptr, t.data_ptr(), nbytes)
        else:
            a = np.ascontiguousarray(v)
            self.ctx.h2d_ptr(dst_ptr, a.ctypes.data, a.nbytes)
        self.stats["h2d_bytes"] += int(v.nbytes) if isinstance(v, np.ndarray) else int(v.numel() * v.element_size())

    def add(self, items: List[Tuple[str, Any]], weight, weighted: bool) -> None:
        """Stage one contribution's device-path arrays (already filtered by exclude_vars)."""
        with self.lock, self.ctx.lock:
            states = [(self._register_key(k, v, weight, weighted), v) for k, v in items]
            arena_items = [(st, v) for st, v in states if st.arena and st.n > 0]
            if arena_items:
                end = max(st.offset + st.n for st, _ in arena_items)
                slot = self._acquire_slot(end * 4)
                self._live_slots.append(slot)
                for st, v in arena_items:
                    ptr = slot.buf.ptr + st.offset * 4
                    self._stage(ptr, v)
                    st.pending.append(_Staged(ptr, weight, slot))
                    slot.refs += 1
            for st, v in states:
                if st.arena or st.n == 0:
                    if st.n == 0:
                        st.pending.append(_Staged(0, weight, None))
                    continue
                buf = self.ctx.alloc(st.n * st.in_np.itemsize)
                self._side_bufs.append(buf)
                self._stage(buf.ptr, v)
                st.pending.append(_Staged(buf.ptr, weight, buf))
            for st, _ in states:
                st.count = weight if st.count is None else st.count + weight

    # ------------------------------------------------------------------ compute
    def _runs(self):
        """Group arena keys (offset order) into maximal runs with identical launch parameters."""
        arena = sorted((st for st in self.keys.values() if st.arena and st.n > 0), key=lambda s: s.offset)
        runs = []
        for st in arena:
            sig = (
                tuple(p.owner.buf.ptr for p in st.pending),
                tuple(p.weight for p in st.pending),
                st.acc_valid,
                st.op,
                st.fin,
                st.count,
            )
            if runs and runs[-1][0] == sig:
                runs[-1][1].append(st)
            else:
                runs.append((sig, [st]))
        return runs

    def _launch_arena(self, final: bool) -> None:
        if not any(st.arena and st.n > 0 for st in self.keys.values()):
            return
        self._ensure_arena_acc()
        for _, group in self._runs():
            first, last = group[0], group[-1]
            n = last.offset + last.n - first.offset
            rows = [p.owner.buf.ptr + first.offset * 4 for p in first.pending]
            weights = [p.weight for p in first.pending]
            if not rows and not (final and first.acc_valid):
                continue
            if not rows and not first.acc_valid:
                continue
            out = self.arena_acc.ptr + first.offset * 4
            self.ctx.accumulate(
                rows,
                weights,
                n,
                out,
                N.FEDAVG_F32,
                N.FEDAVG_F32,
                first.op,
                first.fin if final else N.FEDAVG_FIN_NONE,
                float(first.count),
                acc_in_ptr=out if first.acc_valid else None,
            )
            self.stats["launches"] += 1
            for st in group:
                for p in st.pending:
                    if isinstance(p.owner, _Slot):
                        p.owner.refs -= 1
                        if p.owner.refs == 0:
                            self._release_slot(p.owner)
                st.pending = []
                st.acc_valid = True

    def _launch_side(self, final: bool) -> None:
        for st in self.keys.values():
            if st.arena or st.n == 0:
                continue
            if not st.pending and not (final and st.acc_valid):
                continue
            if st.acc_buf is None:
                st.acc_buf = self.ctx.alloc(st.n * st.acc_np.itemsize)
            rows = [p.ptr for p in st.pending]
            self.ctx.accumulate(
                rows,
                [p.weight for p in st.pending],
                st.n,
                st.acc_buf.ptr,
                st.in_dt,
                st.acc_dt,
                st.op,
                st.fin if final else N.FEDAVG_FIN_NONE,
                float(st.count),
                acc_in_ptr=st.acc_buf.ptr if st.acc_valid else None,
            )
            self.stats["launches"] += 1
            st.pending = []
            st.acc_valid = True

    def _fold(self) -> None:
        """Fold pending contributions into the device accumulators (bitwise-neutral) and free slots."""
        self._launch_arena(final=False)
        self._launch_side(final=False)
        self.ctx.sync()
        for b in self._side_bufs:
            b.close()
        self._side_bufs.clear()
        self.stats["folds"] += 1

    def result(self) -> Dict[str, Any]:
        """Finalise every key on the device and return host (or device-tensor) results."""
        with self.lock, self.ctx.lock:
            # device tensors from torch: make sure their producers finished before we read
            self._launch_arena(final=True)
            self._launch_side(final=True)
            out: Dict[str, Any] = {}
            host_arena = None
            if self.layout_elems and any(st.arena and st.n > 0 and st.torch_device is None for st in self.keys.values()):
                host_arena = np.empty(self.layout_elems, dtype=np.float32)
                self.ctx.d2h(host_arena, self.arena_acc.ptr)
            else:
                self.ctx.sync()
            for name, st in self.keys.items():
                out[name] = self._materialize(st, host_arena)
            return out

    def _materialize(self, st: _KeyState, host_arena):
        if st.n == 0:
            if st.container == "torch":
                return torch.empty(st.shape, dtype=_NP_TO_TORCH[st.acc_np],
                                   device=st.torch_device if st.torch_device is not None else "cpu")
            arr = np.empty(st.shape, dtype=st.acc_np)
        elif st.arena:
            if st.torch_device is not None:
                t = torch.empty(st.shape, dtype=_NP_TO_TORCH[st.acc_np], device=st.torch_device)
                self.ctx.d2d(t.data_ptr(), self.arena_acc.ptr + st.offset * 4, st.n * 4)
                self.ctx.sync()
                return t
            arr = host_arena[st.offset : st.offset + st.n].reshape(st.shape)
        else:
            if st.torch_device is not None:
                t = torch.empty(st.shape, dtype=_NP_TO_TORCH[st.acc_np], device=st.torch_device)
                self.ctx.d2d(t.data_ptr(), st.acc_buf.ptr, st.n * st.acc_np.itemsize)
                self.ctx.sync()
                return t
            arr = np.empty(st.shape, dtype=st.acc_np)
            self.ctx.d2h(arr.reshape(-1) if arr.ndim else arr.reshape(1), st.acc_buf.ptr)
        if st.container == "torch":
            return torch.from_numpy(arr)
        if arr.ndim == 0:
            return arr[()]  # numpy arithmetic on 0-d arrays returns a numpy scalar
        return arr

    # ------------------------------------------------------------------ lifetime
    def reset(self) -> None:
        """Drop the round's state; slot buffers are kept for reuse by the next round."""
        if self._ctx is None:
            self.keys.clear()
            self.layout_elems = 0
            return
        with self.lock, self.ctx.lock:
            for slot in list(self._live_slots):
                self._release_slot(slot)
            for b in self._side_bufs:
                b.close()
            self._side_bufs.clear()
            for st in self.keys.values():
                if st.acc_buf is not None:
                    st.acc_buf.close()
            self.keys.clear()
            self.layout_elems = 0

    def release(self) -> None:
        """Free every device buffer held by this engine."""
        with self.lock:
            self.reset()
            for b in self._free_slots:
                b.close()
            self._free_slots.clear()
            if self.arena_acc is not None:
                self.arena_acc.close()
                self.arena_acc = None
