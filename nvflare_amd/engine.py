"""Device engine behind the drop-in WeightedAggregationHelper.

Reference semantics: nvflare/app_common/aggregators/weighted_aggregation_helper.py:153-240.
Design:

* ``add`` STAGES a contribution's arrays into HBM (H2D for host arrays, D2D for device tensors, bytes
  straight from an mmap for disk-offloaded refs); nothing is computed on the host and the caller's arrays
  are never aliased (``:181-199``).
* Keys of one element format (fp32; float16 and bfloat16 totals) live in that format's ARENA: one flat
  layout (each key at a 256-byte aligned offset), tiled SLABS of client slots, one accumulator.  Element i
  of the client in slot s sits at ``s*T + (i // T) * S*T + i % T`` (T = 4096) of a slab of S slots, so every
  tile's S client segments are contiguous in HBM and the kernel streams them sequentially.
* ``result`` launches the arrival-ordered K-way accumulate-and-finalise kernel over every run of keys
  that share the same contributor list (one launch per arena for the usual all-keys-from-all-clients case)
  and copies the results back -- for large models in a pipelined D2H that overlaps the launches.  fp64 and
  integer / bool keys get a buffer per key per contribution and the generic kernel.
* If the staged slots would exceed the HBM budget (``max_resident_bytes``, default HBM - 8 GiB), the
  pending contributions are FOLDED into the accumulators (same kernels, ``FIN_NONE``) and their slots
  recycled; the per-element operation sequence is unchanged, so the bits are too.
* Slabs persist across rounds.  In the first round they grow geometrically (16, 32, 64, ... slots); at
  ``reset`` a round that needed several slabs is consolidated into one slab of the observed client count,
  so later rounds aggregate in a single launch.
* ``result_deferred`` leaves the fp32 results in HBM (nvflare_amd/deferred.py) for a fused server step.

Numerics are the reference's, per container type (finding 2):
numpy -> ``FEDAVG_OP_NUMPY`` + ``FEDAVG_FIN_SCALE``; torch -> ``FEDAVG_OP_TORCH`` + ``FEDAVG_FIN_DIV``;
``weigh_by_local_iter=False`` -> ``FEDAVG_OP_UNWEIGHTED``.
"""

from __future__ import annotations

import os
import math
import threading
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import _native as N
from . import torch16
from .device import BF16_NP, DeviceBuffer, DeviceContext, HostArenaPool, TiledLayout, fedavg_dtype
from .ingest import MappedTensor
from .quantized import QuantizedPayload, stager

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

ALIGN_ELEMS = 64  # 256 B: every fp32 key starts on a 256-byte boundary of the flat layout
TILE = 4096  # elements per client segment per tile (the kernel's default geometry)
# results larger than two of these leave in a pipelined D2H: the finalising launches are split at every
# EGRESS_CHUNK bytes of results and each finished chunk is copied out while the next ones compute
EGRESS_CHUNK = 256 << 20

_TORCH_TO_NP = {}
_NP_TO_TORCH = {}
if torch is not None:
    _TORCH_TO_NP = {
        torch.float32: np.dtype(np.float32),
        torch.float64: np.dtype(np.float64),
        torch.int32: np.dtype(np.int32),
        torch.int64: np.dtype(np.int64),
        torch.float16: np.dtype(np.float16),
        torch.bfloat16: BF16_NP,
        torch.uint8: np.dtype(np.uint8),
        torch.int8: np.dtype(np.int8),
        torch.int16: np.dtype(np.int16),
        torch.bool: np.dtype(np.bool_),
    }
    _NP_TO_TORCH = {v: k for k, v in _TORCH_TO_NP.items()}

_F16 = np.dtype(np.float16)
_F32 = np.dtype(np.float32)
_F64 = np.dtype(np.float64)
# numpy dtypes with a device kernel; integer and bool arrays accumulate in float64 (numpy promotion)
_NUMPY_INPUTS = {_F16, _F32, _F64} | {np.dtype(t) for t in (np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16,
                                                             np.uint32, np.uint64, np.bool_)}
# (input, accumulator) pairs the C-ABI accepts (include/nvflare_amd_fedavg.h, fedavg_accumulate)
_ACC_F32_INPUTS = {_F32, _F16} | {np.dtype(t) for t in (np.int8, np.int16, np.int32, np.int64, np.uint8, np.bool_)}


def is_torch_tensor(v) -> bool:
    return torch is not None and isinstance(v, torch.Tensor)


def is_device_array(v) -> bool:
    """Arrays/tensors take the HIP path; everything else (python numbers, opaque objects such as HE
    ciphertexts) follows the reference's object protocol on the host."""
    return isinstance(v, (np.ndarray, QuantizedPayload, MappedTensor)) or is_torch_tensor(v)


def _type_proxy(v):
    """An empty array / tensor with the container and dtype a QuantizedPayload dequantizes to."""
    if isinstance(v, QuantizedPayload):
        return torch.empty(0, dtype=v.dtype) if v.container == "torch" else np.empty(0, v.out_dtype)
    if isinstance(v, MappedTensor):  # a disk-offloaded tensor: materialises as a CPU torch tensor
        return torch.empty(0, dtype=v.dtype)
    return v


def _resolve_types(v, weight, weighted: bool) -> Tuple[str, np.dtype, np.dtype, int, int]:
    """(container, input dtype, accumulator/result dtype, op, fin) as the reference's numpy / torch
    arithmetic would produce them (weighted_aggregation_helper.py:181-216, :233-236).

    float16 / bfloat16 values keep a 16-bit total (both libraries keep the array dtype); integer and bool
    values are promoted: torch to the default dtype (float32), numpy to float64 (NEP 50: a python float
    meeting an integer array gives float64).  bfloat16 is carried as ``device.BF16_NP``."""
    v = _type_proxy(v)
    if is_torch_tensor(v):
        tdt = v.dtype
        if tdt not in _TORCH_TO_NP:
            raise TypeError(f"nvflare_amd: torch dtype {tdt} is not supported by the device kernels")
        in_np = _TORCH_TO_NP[tdt]
        # the reference's torch ops run where the tensors are: torch CPU kernels for host tensors, torch-ROCm's
        # GPU kernels for device-resident ones (alpha kept in fp32, div_ by a scalar as a reciprocal product;
        # include/nvflare_amd_fedavg.h FEDAVG_OP_TORCH_DEVICE / FEDAVG_FIN_RECIP, probed against torch on the GPU)
        on_device = v.device.type != "cpu"
        fin = N.FEDAVG_FIN_RECIP if on_device else N.FEDAVG_FIN_DIV
        if in_np.kind in "iub":
            if not weighted:
                # reference: v.clone() stays integer, add_ keeps it, and get_result's div_(count) raises
                # (weighted_aggregation_helper.py:186-187, :208-209, :233): the key is marked, not staged
                return "torch", in_np, in_np, N.FEDAVG_OP_UNWEIGHTED, fin
            acc_np = _TORCH_TO_NP[torch.get_default_dtype()]
        else:
            acc_np = in_np
        op = (N.FEDAVG_OP_TORCH_DEVICE if on_device else N.FEDAVG_OP_TORCH) if weighted else N.FEDAVG_OP_UNWEIGHTED
        return "torch", in_np, acc_np, op, fin
    in_np = np.dtype(v.dtype)
    if in_np not in _NUMPY_INPUTS:
        raise TypeError(f"nvflare_amd: numpy dtype {in_np} is not supported by the device kernels")
    if weighted:
        if isinstance(weight, np.generic):
            acc_np = np.result_type(in_np, np.dtype(type(weight)))
        elif isinstance(weight, (bool, int)) and in_np.kind in "iub":
            raise TypeError("nvflare_amd: integer arrays with an integer weight accumulate in integers; unsupported")
        else:
            acc_np = np.result_type(in_np, 1.0)  # NEP 50: python float is weak
        op = N.FEDAVG_OP_NUMPY
    else:
        if isinstance(weight, np.generic):
            raise TypeError("nvflare_amd: numpy-scalar weights with weigh_by_local_iter=False change the result dtype; unsupported")
        # integer / bool arrays: an integer (bool: OR) sum in the array's dtype, float64 after the scaling
        # (weighted_aggregation_helper.py:195-199, :214-215, :236)
        acc_np = _F64 if in_np.kind in "iub" else in_np
        op = N.FEDAVG_OP_UNWEIGHTED
    acc_np = np.dtype(acc_np)
    ok = (acc_np == _F64 or (acc_np == _F32 and in_np in _ACC_F32_INPUTS) or (acc_np == _F16 and in_np == _F16))
    if not ok:
        raise TypeError(f"nvflare_amd: ({in_np} -> {acc_np}) accumulation unsupported")
    return "numpy", in_np, acc_np, op, N.FEDAVG_FIN_SCALE


def _numpy_scale_override(st) -> Optional[float]:
    """numpy's finalisation ``T * (1.0 / count)`` (weighted_aggregation_helper.py:236) when the weight sum is a
    numpy scalar narrower than the total (np.float32 / np.float16 weights on a float64 total, np.float16 on
    float32): ``1.0 / count`` is then that scalar type's correctly rounded quotient, not the total type's.
    Returns the scale to multiply by in a separate launch, or None when the library's fin value is exact."""
    c = st.count
    if st.fin != N.FEDAVG_FIN_SCALE or not isinstance(c, np.floating):
        return None
    if np.dtype(type(c)).itemsize >= np.dtype(st.acc_np).itemsize or st.acc_np not in (_F32, _F64):
        return None
    with np.errstate(all="ignore"):
        return float(1.0 / c)


def _default_budget(ctx: DeviceContext) -> int:
    """HBM the engine may hold: everything but an 8 GiB reserve (torch, the runtime, other helpers)."""
    env = os.environ.get("NVFLARE_AMD_MAX_RESIDENT_BYTES")
    if env:
        return int(float(env))
    return max(int(ctx.total_bytes) - (8 << 30), int(ctx.total_bytes) // 2)


_ARENA_FORMATS = {  # element formats that get tiled slabs: (C-ABI code, bytes per element)
    np.dtype(np.float32): (N.FEDAVG_F32, 4),
    np.dtype(np.float16): (N.FEDAVG_F16, 2),
    BF16_NP: (N.FEDAVG_BF16, 2),
    np.dtype(np.float64): (N.FEDAVG_F64, 8),
}


class _Arena:
    """One element format's flat key layout, tiled client slabs and accumulator.

    fp32 keys (the hot path), 16-bit keys (float16 / bfloat16 totals) and fp64 keys (numpy's default dtype)
    each get one: a contribution's keys of that format occupy one slot of a slab of the arena, and a run of
    keys is aggregated by one launch of the format's tiled kernel (``fedavg_accumulate_tiled`` /
    ``fedavg_accumulate_tiled16`` / ``fedavg_accumulate_tiled64``)."""

    __slots__ = ("fmt", "esize", "np_dtype", "layout_elems", "slabs", "live", "acc", "host_pool")

    def __init__(self, np_dtype: np.dtype):
        self.np_dtype = np_dtype
        self.fmt, self.esize = _ARENA_FORMATS[np_dtype]
        self.layout_elems = 0  # flat layout size (elements)
        self.slabs: List["_Slab"] = []
        self.live: List["_Slot"] = []
        self.acc: Optional[DeviceBuffer] = None
        self.host_pool = HostArenaPool()

    def launch_end(self, st: "_KeyState") -> int:
        """End of a key's launch range: rounded up to the kernel's vector width, inside the key's 256-byte
        aligned extent."""
        q = 4 if self.esize == 4 else 8
        return (st.offset + st.n + q - 1) // q * q


class _Slab:
    """S client slots in one tiled allocation covering `capacity` elements of an arena's flat layout."""

    __slots__ = ("buf", "layout", "capacity", "free", "arena")

    def __init__(self, buf: DeviceBuffer, layout: TiledLayout, capacity: int, arena: _Arena):
        self.buf = buf
        self.layout = layout
        self.capacity = capacity
        self.arena = arena
        self.free = list(range(layout.slots - 1, -1, -1))  # pop() hands out slot 0 first


class _Slot:
    __slots__ = ("slab", "index", "refs")

    def __init__(self, slab: _Slab, index: int):
        self.slab = slab
        self.index = index
        self.refs = 0

    @property
    def base(self) -> int:
        return self.slab.buf.ptr + self.slab.layout.slot_offset_elems(self.index) * self.slab.arena.esize


class _Staged:
    """One contribution's device copy of one key: a slot of a slab (arena keys) or its own buffer."""

    __slots__ = ("weight", "slot", "buf")

    def __init__(self, weight, slot: Optional[_Slot] = None, buf: Optional[DeviceBuffer] = None):
        self.weight = weight
        self.slot = slot
        self.buf = buf


_FLT_MAX = float(np.finfo(np.float32).max)
_HALF_MAX = 65504.0
# c10 scalar type names in torch's "result type Float can't be cast to the desired output type X"
_TORCH_C10_NAMES = {np.dtype(np.int8): "Char", np.dtype(np.int16): "Short", np.dtype(np.int32): "Int",
                    np.dtype(np.int64): "Long", np.dtype(np.uint8): "Byte", np.dtype(np.bool_): "Bool"}
# torch totals whose add_ alpha c10 range-checks: (largest finite value, c10's type name in the message)
_TORCH_ALPHA_LIMITS = {np.dtype(np.float32): (_FLT_MAX, "float"), np.dtype(np.float16): (_HALF_MAX, "c10::Half"),
                       BF16_NP: (3.3895313892515355e38, "c10::BFloat16")}


class _AddTx:
    """What one ``DeviceFedAvg.add`` took (engine.py): rolled back if the add fails, kept for ``undo_add``."""

    __slots__ = ("n_keys", "layout", "slots", "bufs", "staged", "counts", "moved", "committed")

    def __init__(self, n_keys: int, layout: Dict[int, int]):
        self.n_keys = n_keys  # keys registered before this add (the ones after it are its own)
        self.layout = layout  # arena flat-layout sizes before this add
        self.slots: List[_Slot] = []
        self.bufs: List[DeviceBuffer] = []
        self.staged: List[Tuple["_KeyState", _Staged]] = []
        self.counts: List[tuple] = []  # (key state, count before, count after)
        self.moved = 0
        self.committed = False


class _KeyState:
    __slots__ = ("name", "shape", "container", "torch_device", "in_np", "acc_np", "op", "fin", "n", "arena",
                 "offset", "pending", "acc_valid", "acc_buf", "count", "done", "sig", "int_sum", "doomed")

    def __init__(self):
        self.int_sum = False  # numpy integer / bool sum (weigh_by_local_iter=False): acc_buf holds in_np values
        self.doomed = None  # torch integer total the reference's div_ rejects: c10 type name, nothing staged
        self.sig = None  # (dtype, type(weight), weighted) of plain numpy contributions already type-checked
        self.pending: List[_Staged] = []
        self.acc_valid = False
        self.done = False  # finalised in its arena accumulator (eagerly, or by a deferred round's fused step)
        self.acc_buf: Optional[DeviceBuffer] = None
        self.count = None
        self.arena: Optional[_Arena] = None

    @property
    def in_dt(self):
        return fedavg_dtype(self.in_np)

    @property
    def acc_dt(self):
        return fedavg_dtype(self.acc_np)


class DeviceFedAvg:
    """Arrival-ordered weighted accumulation of client arrays on one HIP device."""

    def __init__(self, device: Optional[int] = None, max_resident_bytes: Optional[int] = None,
                 slab_slots: Optional[int] = None):
        if device is None:
            device = int(os.environ.get("NVFLARE_AMD_DEVICE", "0"))
        self.device = int(device)
        self._ctx: Optional[DeviceContext] = None  # opened on first use (config checks need no GPU)
        self._max_resident_bytes = max_resident_bytes
        env_slots = os.environ.get("NVFLARE_AMD_SLAB_SLOTS")
        self.slab_slots = int(slab_slots or (int(env_slots) if env_slots else 0))  # 0 = adaptive
        self.lock = threading.RLock()
        self.keys: Dict[str, _KeyState] = {}
        self.arenas: Dict[int, _Arena] = {}  # by element format
        self._side_bufs: List[DeviceBuffer] = []
        self._round_clients = 0
        self.peak_clients = 0
        self._deferred = None  # DeferredRound still holding fp32 slots (result_deferred)
        self._last_add: Optional[_AddTx] = None  # the last committed add, while undo_add may take it back
        self._tails_cache: Dict[tuple, np.ndarray] = {}  # torch16 scalar-loop elements per run layout
        # key -> (first element within its whole tensor, the whole tensor's size) for keys that are a bucket of a
        # larger tensor (sharding.ShardedFedAvg); other keys are whole tensors
        self.key_spans: Dict[str, Tuple[int, int]] = {}
        self.stats = {"h2d_bytes": 0, "folds": 0, "launches": 0, "slabs_allocated": 0}

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

    def _arena(self, np_dtype: np.dtype) -> _Arena:
        a = self.arenas.get(_ARENA_FORMATS[np_dtype][0])
        if a is None:
            a = self.arenas[_ARENA_FORMATS[np_dtype][0]] = _Arena(np_dtype)
        return a

    @property
    def f32(self) -> _Arena:
        """The fp32 arena (the hot path; deferred rounds live here)."""
        return self._arena(np.dtype(np.float32))

    @property
    def layout_elems(self) -> int:
        """Elements of the fp32 flat layout (all fp32 keys of the round)."""
        a = self.arenas.get(N.FEDAVG_F32)
        return a.layout_elems if a is not None else 0

    @property
    def slabs(self) -> List[_Slab]:
        return [s for a in self.arenas.values() for s in a.slabs]

    @property
    def _live_slots(self) -> List[_Slot]:
        return [s for a in self.arenas.values() for s in a.live]

    # ------------------------------------------------------------------ memory
    def _resident_bytes(self) -> int:
        total = sum(b.nbytes for b in self._side_bufs)
        for a in self.arenas.values():
            total += sum(s.buf.nbytes for s in a.slabs)
            total += a.acc.nbytes if a.acc is not None else 0
        return total

    def _next_slab_slots(self, arena: _Arena) -> int:
        if self.slab_slots:
            return self.slab_slots
        if not arena.slabs:
            return 16 if self.peak_clients == 0 else max(8, (self.peak_clients + 7) // 8 * 8)
        return min(128, 2 * arena.slabs[-1].layout.slots)

    def _new_slab(self, arena: _Arena, capacity: int, min_slots: int = 0) -> Optional[_Slab]:
        """Allocate a slab for clients of flat extent <= capacity, sized to the remaining budget (but at
        least `min_slots` slots)."""
        n_tiles = (capacity + TILE - 1) // TILE
        per_slot = n_tiles * TILE * arena.esize
        room = self.max_resident_bytes - self._resident_bytes() - arena.esize * (arena.layout_elems + ALIGN_ELEMS)
        slots = max(min_slots, min(self._next_slab_slots(arena), room // per_slot if per_slot else 0))
        while slots >= max(1, min_slots):
            layout = TiledLayout(TILE, int(slots))
            try:
                buf = self.ctx.alloc(layout.slab_elems(capacity) * arena.esize)
            except N.FedAvgError:
                if slots == 1:
                    return None
                slots = max(1, slots // 2)
                continue
            slab = _Slab(buf, layout, n_tiles * TILE, arena)
            arena.slabs.append(slab)
            self.stats["slabs_allocated"] += 1
            return slab
        return None

    def _find_free(self, arena: _Arena, extent: int) -> Optional[_Slot]:
        for slab in arena.slabs:
            if slab.capacity >= extent and slab.free:
                slot = _Slot(slab, slab.free.pop())
                arena.live.append(slot)
                return slot
        return None

    def _acquire_slot(self, arena: _Arena, extent: int) -> _Slot:
        slot = self._find_free(arena, extent)
        if slot is None and self._new_slab(arena, max(extent, arena.layout_elems)) is not None:
            slot = self._find_free(arena, extent)
        if slot is None and self._live_slots:
            self._fold()  # over budget: fold what is staged (frees every slot, keeps the slabs)
            slot = self._find_free(arena, extent)
        if slot is None:
            # the remaining slabs cannot hold this client: drop them and make room for at least one slot
            for s in arena.slabs:
                s.buf.close()
            arena.slabs.clear()
            if self._new_slab(arena, max(extent, arena.layout_elems), min_slots=1) is not None:
                slot = self._find_free(arena, extent)
        if slot is None:
            raise N.FedAvgError(f"nvflare_amd: cannot stage a client of {extent} {arena.np_dtype} elements on "
                                f"device {self.device} (HBM budget {self.max_resident_bytes} bytes)")
        return slot

    def _release_slot(self, slot: _Slot) -> None:
        live = slot.slab.arena.live
        if slot in live:
            live.remove(slot)
            slot.slab.free.append(slot.index)

    # ------------------------------------------------------------------ layout
    def _check_torch_alpha(self, items, weight, weighted: bool) -> None:
        """torch's ``T.add_(v, alpha=w)`` (weighted_aggregation_helper.py:205-207) refuses a finite alpha
        outside the total's range (c10 ``checked_convert``: fp32, float16 65504, bfloat16).  Raise the same
        RuntimeError, before anything of this contribution is staged (the reference fails part-way through the
        keys instead)."""
        if not weighted:
            return
        w = float(weight)
        if not (math.isfinite(w) and abs(w) > _HALF_MAX):
            return
        for k, _ in items:
            st = self.keys.get(k)
            if st is None or st.container != "torch":
                continue
            # device tensors: torch-ROCm converts alpha to its fp32 opmath type whatever the tensor dtype
            limit = (_TORCH_ALPHA_LIMITS.get(st.acc_np) if st.torch_device is None
                     else (_FLT_MAX, "float") if st.acc_np != _F64 else None)
            if limit is not None and abs(w) > limit[0]:
                raise RuntimeError(f"value cannot be converted to type {limit[1]} without overflow")

    def _register_key(self, name: str, v, weight, weighted: bool) -> _KeyState:
        st = self.keys.get(name)
        plain = type(v) is np.ndarray
        if st is not None and plain and st.sig is not None and st.shape == v.shape \
                and st.sig == (v.dtype, type(weight), weighted):
            return st  # same inputs to _resolve_types as a contribution already checked: same result
        container, in_np, acc_np, op, fin = _resolve_types(v, weight, weighted)
        shape = tuple(v.shape)
        if st is not None:
            if st.container != container or st.in_np != in_np or st.acc_np != acc_np:
                raise TypeError(
                    f"nvflare_amd: key {name!r} changed type between contributions "
                    f"({st.container}/{st.in_np} -> {container}/{in_np}); unsupported"
                )
            if st.shape != shape:
                raise ValueError(f"nvflare_amd: key {name!r} shape {shape} != first contribution's {st.shape}")
            if plain:
                st.sig = (v.dtype, type(weight), weighted)
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
        if plain:
            st.sig = (v.dtype, type(weight), weighted)
        if op == N.FEDAVG_OP_UNWEIGHTED and in_np.kind in "iub":
            if container == "torch":
                st.doomed = _TORCH_C10_NAMES[in_np]
            else:
                st.int_sum = True
        if in_np == acc_np and in_np in _ARENA_FORMATS:
            st.arena = self._arena(in_np)
            st.offset = st.arena.layout_elems
            st.arena.layout_elems += (st.n + ALIGN_ELEMS - 1) // ALIGN_ELEMS * ALIGN_ELEMS
        else:
            st.offset = -1
        self.keys[name] = st
        return st

    def _ensure_acc(self, arena: _Arena) -> None:
        need = max(arena.layout_elems, ALIGN_ELEMS) * arena.esize
        if arena.acc is not None and arena.acc.nbytes >= need:
            return
        new = self.ctx.alloc(need)
        if arena.acc is not None:
            self.ctx.d2d(new.ptr, arena.acc.ptr, arena.acc.nbytes)
            self.ctx.sync()
            arena.acc.close()
        arena.acc = new

    # ------------------------------------------------------------------ staging
    @staticmethod
    def _source(v):
        """(keep-alive, pointer, nbytes, on_device) of a contiguous view of v."""
        if isinstance(v, MappedTensor):  # bytes straight from the page cache of the safetensors file
            keep, ptr, nbytes = v.host_view()
            return keep, ptr, nbytes, False
        if is_torch_tensor(v):
            t = v.detach()
            if not t.is_contiguous():
                t = t.contiguous()
            if t.device.type != "cpu":
                torch.cuda.current_stream(t.device).synchronize()  # producer's work done before we read
            return t, t.data_ptr(), t.numel() * t.element_size(), t.device.type != "cpu"
        a = np.ascontiguousarray(v)
        return a, a.ctypes.data, a.nbytes, False

    def _check_device(self, v) -> None:
        if is_torch_tensor(v) and v.device.type != "cpu" and v.device.index != self.ctx.device:
            raise ValueError(f"nvflare_amd: tensor on {v.device}, engine on device {self.ctx.device}")

    def _stage_arena(self, arena: _Arena, items, weight, tx: "_AddTx") -> None:
        """One contribution's keys of one arena into one slot (the slot base + logical offsets).  The staged
        records go to ``tx``; the keys' ``pending`` lists only see them when the whole contribution commits."""
        extent = max(st.offset + st.n for st, _ in items)
        slot = self._acquire_slot(arena, extent)
        tx.slots.append(slot)
        slot.refs += len(items)  # held by this contribution: a fold while its other arenas stage keeps it live
        lay = slot.slab.layout
        es = arena.esize
        host_pieces, keep = [], []
        quantized = []
        device_src = False
        staged = _Staged(weight, slot=slot)  # immutable: shared by every key of this contribution in this slot
        moved = 0
        for st, v in sorted(items, key=lambda x: x[0].offset):
            if type(v) is np.ndarray and v.flags.c_contiguous:  # the common case, without _source's dispatch
                nbytes = v.nbytes
                host_pieces.append((st.offset * es, v.ctypes.data, nbytes))
                keep.append(v)
            elif isinstance(v, QuantizedPayload):  # fp32 arena only (dequantizes to fp32)
                quantized.append((st, v))
                nbytes = v.nbytes
            else:
                src, ptr, nbytes, on_dev = self._source(v)
                if on_dev:
                    self.ctx.d2d_tiled(slot.base, lay.tile * es, lay.tile_stride * es, st.offset * es, ptr, nbytes)
                    keep.append(src)
                    device_src = True
                else:
                    host_pieces.append((st.offset * es, ptr, nbytes))
                    keep.append(src)
            tx.staged.append((st, staged))
            moved += nbytes
        # every host key of this client in one pass through the pinned ring (one DMA per 64 MiB)
        self.ctx.h2d_tiled_multi(slot.base, lay.tile * es, lay.tile_stride * es, host_pieces)
        for st, v in quantized:  # compressed bytes over PCIe, fp32 written into the slot by the GPU
            stager().dequantize_into(self.ctx, v, slot.base, lay.tile, lay.tile_stride, st.offset)
        tx.moved += moved
        if device_src:
            # the device-to-device copies run on the library's stream: finish them before the caller (or torch's
            # allocator, for a contiguous() temporary) may reuse the source memory -- accept must not alias
            self.ctx.sync()
        del keep

    def add(self, items: List[Tuple[str, Any]], weight, weighted: bool) -> "_AddTx":
        """Stage one contribution's device-path arrays (already filtered by exclude_vars).

        All or nothing: the contribution's slots, side buffers and keys it introduces are taken inside a
        transaction; only when every arena and side buffer is staged do its records join the keys' pending
        lists and its weight their counts (the reference's per-key ``counts[k] += w`` next to the key's sum,
        weighted_aggregation_helper.py:201,216).  On any exception (an allocation, a copy) everything is given
        back and the next aggregation is the one over the contributions accepted so far.  Returns the
        committed transaction, which ``undo_add`` can take back while it is the engine's last operation (a
        sharded contribution whose other buckets failed, sharding.ShardedFedAvg.add)."""
        # quantized payloads dequantize on the device straight into their fp32 slot; other dtypes take
        # the generic path from their (device-dequantized) host values
        items = [(k, v.materialize() if isinstance(v, QuantizedPayload) and v.out_dtype != np.float32 else v)
                 for k, v in items]
        with self.lock, self.ctx.lock:
            self._last_add = None
            self._settle()
            self._check_torch_alpha(items, weight, weighted)
            tx = _AddTx(len(self.keys), {fmt: a.layout_elems for fmt, a in self.arenas.items()})
            try:
                states = [(self._register_key(k, v, weight, weighted), v) for k, v in items]
                for _, v in states:
                    if type(v) is not np.ndarray:
                        self._check_device(v)
                by_arena: Dict[int, Tuple[_Arena, list]] = {}
                for st, v in states:
                    if st.arena is not None and st.n > 0:
                        by_arena.setdefault(st.arena.fmt, (st.arena, []))[1].append((st, v))
                for arena, arena_items in by_arena.values():
                    self._stage_arena(arena, arena_items, weight, tx)
                for st, v in states:
                    if st.arena is not None or st.n == 0 or st.doomed:
                        if st.n == 0 and not st.doomed:
                            tx.staged.append((st, _Staged(weight)))
                        continue
                    buf = self.ctx.alloc(st.n * st.in_np.itemsize)
                    tx.bufs.append(buf)
                    self._side_bufs.append(buf)
                    keep, ptr, nbytes, on_dev = self._source(v)
                    if on_dev:
                        self.ctx.d2d(buf.ptr, ptr, nbytes)
                        self.ctx.sync()  # as in _stage_arena: the source may be reused once we return
                    else:
                        self.ctx.h2d_ptr(buf.ptr, ptr, nbytes)
                    del keep
                    tx.staged.append((st, _Staged(weight, buf=buf)))
                    tx.moved += nbytes
                tx.counts = [(st, st.count, weight if st.count is None else st.count + weight) for st, _ in states]
            except BaseException:
                self._give_back(tx)
                raise
            # commit (nothing below raises)
            for st, p in tx.staged:
                st.pending.append(p)
            for st, _, new in tx.counts:
                st.count = new
            self._round_clients += 1
            self.stats["h2d_bytes"] += tx.moved
            tx.committed = True
            self._last_add = tx
            return tx

    def _give_back(self, tx: "_AddTx") -> None:
        """Return what an uncommitted (or undone) contribution took: slots, side buffers, the keys it
        introduced and their place in the arenas' flat layouts."""
        try:
            self.ctx.sync()  # copies into the slots / buffers may still be in flight
        except Exception:  # pragma: no cover - the device error is the one being raised
            pass
        for slot in tx.slots:
            slot.refs = 0
            self._release_slot(slot)
        for buf in tx.bufs:
            if buf in self._side_bufs:
                self._side_bufs.remove(buf)
            buf.close()
        for name in list(self.keys)[tx.n_keys:]:  # dicts keep insertion order: the keys this add registered
            del self.keys[name]
        for fmt, a in self.arenas.items():
            a.layout_elems = tx.layout.get(fmt, 0)

    def undo_add(self, tx: "_AddTx") -> None:
        """Take back a committed contribution, which must be this engine's last operation (nothing was added,
        folded, aggregated or reset since): its pending records, its weight in the counts, its slots and side
        buffers and the keys it introduced."""
        with self.lock, self.ctx.lock:
            if tx is None or not tx.committed or tx is not self._last_add:
                raise RuntimeError("nvflare_amd: only the engine's last contribution can be taken back")
            for st, p in reversed(tx.staged):
                if not st.pending or st.pending[-1] is not p:
                    raise RuntimeError("nvflare_amd: contribution already consumed; cannot take it back")
                st.pending.pop()
            for st, old, _ in tx.counts:
                st.count = old
            self._round_clients -= 1
            self.stats["h2d_bytes"] -= tx.moved
            tx.committed = False
            self._last_add = None
            self._give_back(tx)

    # ------------------------------------------------------------------ compute
    def _runs(self, keys: Optional[Dict[str, _KeyState]] = None, arena: Optional[_Arena] = None):
        """One arena's keys (default: fp32) in offset order, grouped into maximal runs with identical launch
        parameters."""
        keys = self.keys if keys is None else keys
        arena = self.f32 if arena is None else arena
        keyed = sorted((st for st in keys.values() if st.arena is arena and st.n > 0 and not st.done),
                       key=lambda s: s.offset)
        runs = []
        for st in keyed:
            sig = (tuple(id(p.slot) for p in st.pending), tuple(p.weight for p in st.pending), st.acc_valid, st.op,
                   st.fin, st.count)
            if runs and runs[-1][0] == sig:
                runs[-1][1].append(st)
            else:
                runs.append((sig, [st]))
        return [g for _, g in runs]

    def _launch_run(self, group: List[_KeyState], final: bool, out: Optional[int] = None,
                    epi: Optional["N.Epilogue"] = None, rng: Optional[Tuple[int, int]] = None) -> None:
        """Launch the kernels for one run of keys into the flat accumulator ``out`` (default: the arena's).
        With ``epi`` (fp32 only) the last launch carries the server-optimizer epilogue (deferred rounds);
        ``rng`` restricts the launches to a sub-range of the run (pipelined egress)."""
        first, last = group[0], group[-1]
        arena = first.arena
        begin, end = rng if rng is not None else (first.offset, arena.launch_end(last))
        pend = first.pending
        if not pend and not (final and first.acc_valid):
            return
        out = arena.acc.ptr if out is None else out
        acc_in = out if first.acc_valid else None
        fin = first.fin if final else N.FEDAVG_FIN_NONE
        scale = _numpy_scale_override(first) if final else None
        if scale is not None:
            if epi is not None:
                raise TypeError("nvflare_amd: a server-optimizer epilogue on a numpy total with narrower numpy-scalar "
                                "weights is unsupported")
            fin = N.FEDAVG_FIN_NONE  # the scaling runs as its own launch below
        # a fold can happen while a contribution is being staged (its second arena needs room), before the
        # contribution's weight is counted: the count only matters to the finalisation
        count = float(first.count) if first.count is not None else 1.0
        if epi is not None and arena.fmt != N.FEDAVG_F32:
            raise TypeError("nvflare_amd: server-optimizer epilogues run on fp32 keys only")
        tails = None
        if first.op == N.FEDAVG_OP_TORCH and arena.fmt in (N.FEDAVG_F16, N.FEDAVG_BF16):
            tails = self._torch16_tails(group)
        elif first.op == N.FEDAVG_OP_TORCH_DEVICE and arena.fmt == N.FEDAVG_F16:
            tails = self._rocm16_tails(group)

        def launch(bases, weights, tile, stride, fin_, last_launch):
            if arena.fmt == N.FEDAVG_F64:
                self.ctx.accumulate_tiled64(bases, weights, tile, stride, begin, end, out, first.op, fin_, count, acc_in)
            elif arena.fmt != N.FEDAVG_F32:
                self.ctx.accumulate_tiled16(arena.fmt, bases, weights, tile, stride, begin, end, out, first.op, fin_,
                                            count, acc_in, tails=tails)
            elif epi is not None and last_launch:
                self.ctx.accumulate_tiled_epi(bases, weights, tile, stride, begin, end, out, first.op, fin_, count,
                                              epi, acc_in)
            else:
                self.ctx.accumulate_tiled(bases, weights, tile, stride, begin, end, out, first.op, fin_, count,
                                          acc_in)
            self.stats["launches"] += 1

        if not pend:  # finalise an already folded sum
            launch([], [], TILE, TILE, fin, True)
            self._scale_range(arena, out, begin, end, scale)
            return
        # consecutive contributions staged in slabs of the same geometry go in one launch; a change of
        # geometry chains the next launch through the accumulator (arrival order is preserved)
        segs: List[List[_Staged]] = []
        for p in pend:
            if segs and segs[-1][-1].slot.slab.layout.tile_stride == p.slot.slab.layout.tile_stride:
                segs[-1].append(p)
            else:
                segs.append([p])
        for i, seg in enumerate(segs):
            lay = seg[0].slot.slab.layout
            last_launch = i == len(segs) - 1
            launch([p.slot.base for p in seg], [p.weight for p in seg], lay.tile, lay.tile_stride,
                   fin if last_launch else N.FEDAVG_FIN_NONE, last_launch)
            acc_in = out
        self._scale_range(arena, out, begin, end, scale)

    def _scale_range(self, arena: _Arena, out: int, begin: int, end: int, scale: Optional[float]) -> None:
        """out[begin:end] *= scale in the total's dtype (the (X, X) rows entry, first step v * w)."""
        if scale is None or end <= begin:
            return
        p = out + begin * arena.esize
        self.ctx.accumulate([p], [scale], end - begin, p, arena.fmt, arena.fmt, N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_NONE, 1.0)
        self.stats["launches"] += 1

    def _torch16_tails(self, group: List[_KeyState]) -> np.ndarray:
        """Flat indices of the group's elements that torch's add_ runs through its scalar loop (torch16.py),
        for the thread count and vector build of this process -- where the reference would run."""
        # host tensors only: the reference adds device-resident tensors with torch's GPU kernel (no CPU loops)
        sig = (tuple((st.offset, st.n) + self.key_spans.get(st.name, (0, st.n)) for st in group
                     if st.torch_device is None), torch16.torch_threads(), torch16.vector_block())
        hit = self._tails_cache.get(sig)
        if hit is None:
            hit = self._tails_cache[sig] = torch16.scalar_tail_indices(sig[0], sig[1], sig[2])
        return hit

    def _rocm16_tails(self, group: List[_KeyState]) -> np.ndarray:
        """Flat indices of the group's float16 device-tensor elements torch-ROCm adds in its unrolled path."""
        sig = ("rocm",) + tuple((st.offset, st.n) + self.key_spans.get(st.name, (0, st.n)) for st in group)
        hit = self._tails_cache.get(sig)
        if hit is None:
            hit = self._tails_cache[sig] = torch16.rocm_f16_unrolled_indices(sig[1:])
        return hit

    def _launch_arena(self, final: bool, keys: Optional[Dict[str, _KeyState]] = None,
                      out: Optional[int] = None, arenas: Optional[List[_Arena]] = None) -> None:
        """Launch every pending run of the given arenas (default: all; with an explicit ``out`` -- a deferred
        round's accumulator -- the fp32 arena)."""
        keys = self.keys if keys is None else keys
        if arenas is None:
            arenas = [self.f32] if out is not None else list(self.arenas.values())
        for arena in arenas:
            if not any(st.arena is arena and st.n > 0 and not st.done for st in keys.values()):
                continue
            if out is None:
                self._ensure_acc(arena)
            for group in self._runs(keys, arena):
                self._launch_run(group, final, out)
                self._consume(group)
                if final:
                    for st in group:
                        st.done = True

    def _consume(self, group: List[_KeyState]) -> None:
        """The group's staged slots are folded into its accumulator: drop them (recycle at refs == 0).

        Only keys that had staged contributions become ``acc_valid``: a fold can run while a contribution is
        being staged, when a key it introduces is registered but not staged yet -- that key has nothing in
        the accumulator, and its first contribution must still take the first-operation path."""
        for st in group:
            if not st.pending:
                continue
            for p in st.pending:
                p.slot.refs -= 1
                if p.slot.refs == 0:
                    self._release_slot(p.slot)
            st.pending = []
            st.acc_valid = True

    def _launch_side(self, final: bool) -> None:
        for st in self.keys.values():
            if st.arena is not None or st.n == 0 or st.doomed or st.done:
                continue
            if not st.pending and not (final and st.acc_valid):
                continue
            if st.int_sum:
                self._launch_int_sum(st, final)
                continue
            if st.acc_buf is None:
                st.acc_buf = self.ctx.alloc(st.n * st.acc_np.itemsize)
            scale = _numpy_scale_override(st) if final else None
            if st.pending or scale is None:
                self.ctx.accumulate(
                    [p.buf.ptr for p in st.pending],
                    [p.weight for p in st.pending],
                    st.n,
                    st.acc_buf.ptr,
                    st.in_dt,
                    st.acc_dt,
                    st.op,
                    st.fin if final and scale is None else N.FEDAVG_FIN_NONE,
                    float(st.count) if st.count is not None else 1.0,
                    acc_in_ptr=st.acc_buf.ptr if st.acc_valid else None,
                )
                self.stats["launches"] += 1
            if scale is not None:
                self.ctx.accumulate([st.acc_buf.ptr], [scale], st.n, st.acc_buf.ptr, st.acc_dt, st.acc_dt,
                                    N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_NONE, 1.0)
                self.stats["launches"] += 1
                st.done = True
            st.pending = []
            st.acc_valid = True

    def _launch_int_sum(self, st: _KeyState, final: bool) -> None:
        """numpy integer / bool arrays with weigh_by_local_iter=False: the running sum stays in the array's
        dtype (wraparound; OR for bool); the final launch turns it into float64(T) * (1.0 / count) (:236)."""
        if st.acc_buf is None:
            st.acc_buf = self.ctx.alloc(st.n * st.in_np.itemsize)
        if st.pending or not st.acc_valid:
            self.ctx.accumulate([p.buf.ptr for p in st.pending], [p.weight for p in st.pending], st.n, st.acc_buf.ptr,
                                st.in_dt, st.in_dt, N.FEDAVG_OP_UNWEIGHTED, N.FEDAVG_FIN_NONE, 1.0,
                                acc_in_ptr=st.acc_buf.ptr if st.acc_valid else None)
            self.stats["launches"] += 1
            st.pending = []
            st.acc_valid = True
        if final:
            ints, st.acc_buf = st.acc_buf, self.ctx.alloc(st.n * 8)
            self.ctx.accumulate([ints.ptr], [1.0 / float(st.count)], st.n, st.acc_buf.ptr, st.in_dt, N.FEDAVG_F64,
                                N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_NONE, 1.0)
            self.ctx.sync()
            ints.close()
            st.done = True
            self.stats["launches"] += 1

    def _fold(self) -> None:
        """Fold pending contributions into the device accumulators (bitwise-neutral) and free slots."""
        self._launch_arena(final=False)
        self._launch_side(final=False)
        self.ctx.sync()
        for b in self._side_bufs:
            b.close()
        self._side_bufs.clear()
        self.stats["folds"] += 1

    def _launch_arena_chunked(self, arena: _Arena) -> None:
        """Final launches of one arena split at every EGRESS_CHUNK bytes of results, with a readiness mark
        (``fedavg_mark``) after each chunk boundary, for ``fedavg_d2h_marked``."""
        self._ensure_acc(arena)
        self.ctx.marks_reset()  # a new marked sequence: nothing stale may vouch for these bytes
        chunk = max(EGRESS_CHUNK // arena.esize // TILE, 1) * TILE
        for group in self._runs(self.keys, arena):
            b, e = group[0].offset, arena.launch_end(group[-1])
            pos = b
            while pos < e:
                hi = min(e, (pos // chunk + 1) * chunk)
                self._launch_run(group, True, rng=(pos, hi))
                if hi % chunk == 0:
                    self.ctx.mark(hi * arena.esize)
                pos = hi
            self._consume(group)
            for st in group:
                st.done = True
        self.ctx.mark(arena.layout_elems * arena.esize)

    def _host_arenas(self, arenas, pipelined: Optional[_Arena] = None, skip=()) -> Dict[int, np.ndarray]:
        """One D2H per arena holding host-container keys (results are views of these arrays); keys in ``skip`` go
        to destinations of their own (``result(host_dest=...)``)."""
        hosts = {}
        for a in sorted(arenas, key=lambda x: x is not pipelined):  # the pipelined D2H first
            if self._has_host_keys(a, skip):
                host = a.host_pool.take(a.layout_elems, a.np_dtype, pin=self.ctx)
                if a is pipelined:
                    self.ctx.d2h_marked(host, a.acc.ptr)
                else:
                    self.ctx.d2h(host, a.acc.ptr)
                hosts[a.fmt] = host
        return hosts

    def _has_host_keys(self, a: _Arena, skip=()) -> bool:
        return bool(a.layout_elems) and any(st.arena is a and st.n > 0 and st.torch_device is None
                                            and st.name not in skip for st in self.keys.values())

    def _check_doomed(self) -> None:
        """Keys the reference's get_result (weighted_aggregation_helper.py:226-240) fails on, in its key order,
        raised before any launch: a torch integer total under weigh_by_local_iter=False (``div_`` refuses it),
        and a numpy key whose python-number weight sum is 0 (``1.0 / count`` -- e.g. every contribution with
        NUM_STEPS_CURRENT_ROUND = 0)."""
        for st in self.keys.values():
            if st.doomed:
                raise RuntimeError(f"result type Float can't be cast to the desired output type {st.doomed}")
            if st.fin == N.FEDAVG_FIN_SCALE and type(st.count) in (int, float, bool) and st.count == 0:  # not numpy scalars
                raise ZeroDivisionError("float division by zero")

    def result(self, host_dest: Optional[Dict[str, Tuple[np.ndarray, int]]] = None) -> Dict[str, Any]:
        """Finalise every key on the device and return host (or device-tensor) results.

        ``host_dest`` ({key: (host array, element offset)}): those of the keys that are host-container arena keys
        are copied straight into the caller's array (one ``fedavg_d2h_multi`` per array and arena, page-locked
        destinations written by the DMA) and come back as None -- sharding.ShardedFedAvg assembles whole keys
        from its buckets this way, without a host-side concatenation."""
        self._check_doomed()
        with self.lock, self.ctx.lock:
            self._last_add = None
            self._settle()
            direct = {}
            for n, d in (host_dest or {}).items():
                st = self.keys.get(n)
                if st is not None and st.arena is not None and st.n > 0 and st.torch_device is None:
                    if np.dtype(d[0].dtype) != st.arena.np_dtype:
                        raise TypeError(f"nvflare_amd: host destination of {n!r} is {d[0].dtype}, not {st.arena.np_dtype}")
                    direct[n] = d
            # the largest host-bound arena leaves in a pipelined D2H that overlaps its own launches
            big = [a for a in self.arenas.values()
                   if a.layout_elems * a.esize >= 2 * EGRESS_CHUNK and self._has_host_keys(a, direct)]
            pipelined = max(big, key=lambda a: a.layout_elems * a.esize) if big else None
            if pipelined is not None:
                self._launch_arena_chunked(pipelined)
            self._launch_arena(final=True, arenas=[a for a in self.arenas.values() if a is not pipelined])
            self._launch_side(final=True)
            hosts = self._host_arenas(self.arenas.values(), pipelined, direct)
            groups: Dict[tuple, tuple] = {}
            for n, (host, off) in direct.items():
                st = self.keys[n]
                es = st.arena.esize
                g = groups.setdefault((id(host), st.arena.fmt), (host, st.arena, []))
                g[2].append((off * es, st.offset * es, st.n * es))
            for host, arena, pieces in groups.values():
                self.ctx.d2h_multi(host, arena.acc.ptr, pieces)
            self.ctx.sync()
            return {name: None if name in direct else self._materialize(st, hosts) for name, st in self.keys.items()}

    def result_deferred(self) -> Dict[str, Any]:
        """``result()`` with the fp32 arena keys left on the device: they come back as ``DeferredAggregate``
        values (nvflare_amd/deferred.py) whose aggregation runs when one is materialised -- or inside a
        server-optimizer launch (``DeferredRound.fused_step``), so the aggregated difference never crosses
        PCIe.  Other keys are finalised now, as in ``result()``.  The round keeps its slots until it is
        settled: by the fused step, by a materialisation, or by the next ``add`` / ``result``."""
        from .deferred import DeferredAggregate, DeferredRound

        self._check_doomed()
        with self.lock, self.ctx.lock:
            self._last_add = None
            self._settle()
            others = [a for a in self.arenas.values() if a.fmt != N.FEDAVG_F32]
            self._launch_arena(final=True, arenas=others)
            self._launch_side(final=True)
            hosts = self._host_arenas(others)
            self.ctx.sync()
            deferred = {n: st for n, st in self.keys.items() if st.arena is not None and st.arena.fmt == N.FEDAVG_F32
                        and st.n > 0}
            eager = {n: self._materialize(st, hosts) for n, st in self.keys.items() if n not in deferred}
            if not deferred:
                return eager
            f32 = self.f32
            self._ensure_acc(f32)
            acc, f32.acc = f32.acc, None  # the round owns this accumulator from now on
            rnd = DeferredRound(self, deferred, acc)
            self._deferred = rnd
            return {n: eager[n] if n in eager else DeferredAggregate(rnd, n) for n in self.keys}

    def _settle(self) -> None:
        """Finish an outstanding deferred round on the device (its values stay readable) and recycle its
        slots.  Called before anything else touches the slabs."""
        rnd, self._deferred = self._deferred, None
        if rnd is not None:
            rnd.settle()
            self._consolidate()

    def _consolidate(self) -> None:
        if self._deferred is not None or self.slab_slots:
            return
        for a in self.arenas.values():
            if not a.live and len(a.slabs) > 1:
                # a round needed several slabs: next round gets one slab of the observed client count
                for s in a.slabs:
                    s.buf.close()
                a.slabs.clear()

    def _materialize(self, st: _KeyState, hosts: Dict[int, np.ndarray]):
        if st.n == 0:
            if st.container == "torch":
                return torch.empty(st.shape, dtype=_NP_TO_TORCH[st.acc_np],
                                   device=st.torch_device if st.torch_device is not None else "cpu")
            arr = np.empty(st.shape, dtype=st.acc_np)
        elif st.torch_device is not None:
            t = torch.empty(st.shape, dtype=_NP_TO_TORCH[st.acc_np], device=st.torch_device)
            src = st.arena.acc.ptr + st.offset * st.arena.esize if st.arena is not None else st.acc_buf.ptr
            self.ctx.d2d(t.data_ptr(), src, st.n * st.acc_np.itemsize)
            self.ctx.sync()
            return t
        elif st.arena is not None:
            arr = hosts[st.arena.fmt][st.offset: st.offset + st.n].reshape(st.shape)
        else:
            arr = np.empty(st.shape, dtype=st.acc_np)
            self.ctx.d2h(arr.reshape(-1) if arr.ndim else arr.reshape(1), st.acc_buf.ptr)
        if st.container == "torch":
            if st.acc_np == BF16_NP:
                return torch.from_numpy(arr.view(np.uint16)).view(torch.bfloat16)
            return torch.from_numpy(arr)
        if arr.ndim == 0:
            return arr[()]  # numpy arithmetic on 0-d arrays returns a numpy scalar
        return arr

    # ------------------------------------------------------------------ lifetime
    def reset(self) -> None:
        """Drop the round's state; slabs are kept (and consolidated) for the next round."""
        self.peak_clients = max(self.peak_clients, self._round_clients)
        self._round_clients = 0
        self._last_add = None
        if self._ctx is None:
            self.keys.clear()
            for a in self.arenas.values():
                a.layout_elems = 0
            return
        with self.lock, self.ctx.lock:
            for a in self.arenas.values():
                if self._deferred is not None and a.fmt == N.FEDAVG_F32:
                    continue  # a deferred round keeps its fp32 slots until it is settled
                for slot in list(a.live):
                    self._release_slot(slot)
            for b in self._side_bufs:
                b.close()
            self._side_bufs.clear()
            for st in self.keys.values():
                if st.acc_buf is not None:
                    st.acc_buf.close()
            self._consolidate()
            self.keys.clear()
            self._tails_cache.clear()
            self.key_spans.clear()
            for a in self.arenas.values():
                a.layout_elems = 0

    def release(self) -> None:
        """Free every device buffer held by this engine."""
        with self.lock:
            if self._ctx is not None:
                with self.ctx.lock:
                    self._settle()
            self.reset()
            for a in self.arenas.values():
                for s in a.slabs:
                    s.buf.close()
                a.slabs.clear()
                if a.acc is not None:
                    a.acc.close()
                    a.acc = None
