"""Aggregation results that stay in HBM until they are read (SAG-level fusion of aggregation and server step).

In a scatter-and-gather FedOpt job the aggregated difference makes a round trip the reference pays on
the host: ``DXOAggregator.aggregate`` -> ``get_result`` returns host arrays (weighted_aggregation_helper.py:
226-240), ``ScatterAndGather`` hands them to ``shareable_gen.shareable_to_learnable``
(scatter_and_gather.py:298-318) and ``PTFedOptModelShareableGenerator.server_update`` copies them back to
the model's device as ``param.grad`` (app_opt/pt/fedopt.py:157-182).  On the MI355X that is a 4·P-byte
D2H, a 4·P-byte H2D and a separate optimizer pass over p, m, v.

With ``defer_result=True`` on the aggregator, ``get_result`` returns a ``DeferredAggregate`` for every fp32
key instead: nothing is launched yet.  The device FedOpt generator recognises them and runs the K-client
aggregation and the optimizer step in ONE launch per run of parameters (``fedavg_accumulate_tiled_epi``
over the client slots, the parameter / state pointers offset so the optimizer's flat layout lines up with
the aggregation layout); the aggregated difference is still written to the round's accumulator, so a
later ``materialize()`` returns exactly what the eager path would have returned.  Any other consumer
reads a value through ``materialize()`` (NVFlare's own lazy-ref protocol, weighted_aggregation_helper.py:
170-175) or ``np.asarray`` (``__array__``); either one settles the round first.
"""

from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _native as N

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


class FusedEntry:
    """One parameter of a fused server step: where it lives in the optimizer's flat buffers and the
    epilogue (pointers to the flat buffers' element 0) that steps it.  ``sig`` groups parameters that
    may share a launch (same param group, step count and state presence)."""

    __slots__ = ("offset", "epi", "sig")

    def __init__(self, offset: int, epi: "N.Epilogue", sig):
        self.offset = int(offset)
        self.epi = epi
        self.sig = sig


def _shifted(epi: "N.Epilogue", delta_elems: int) -> "N.Epilogue":
    """A copy of ``epi`` whose flat operand pointers are moved by ``delta_elems`` fp32 elements, so that
    element i of the aggregation layout addresses element i + delta of the optimizer's buffers."""
    e = N.Epilogue.from_buffer_copy(epi)
    for f in ("param", "state1", "state2", "state3", "base"):
        p = getattr(e, f)
        if p:
            setattr(e, f, ctypes.c_void_p(p + 4 * delta_elems).value)
    return e


class DeferredRound:
    """The fp32 keys of one finished round, their staged client slots and the accumulator they finalise into."""

    def __init__(self, engine, keys: Dict[str, object], acc):
        self.engine = engine
        self.keys = keys
        self.acc = acc  # DeviceBuffer over the round's flat layout
        self.settled = False
        self._values: Dict[str, object] = {}

    @property
    def device(self) -> int:
        return self.engine.device

    def _locked(self):
        return _Locks(self.engine)

    def settle(self) -> None:
        """Finalise every key not yet consumed by a fused step into the accumulator and free the slots."""
        with self._locked():
            if self.settled:
                return
            self.engine._launch_arena(final=True, keys=self.keys, out=self.acc.ptr)
            self.settled = True
            if self.engine._deferred is self:
                self.engine._deferred = None
                self.engine._consolidate()

    def fusable(self, name: str) -> bool:
        st = self.keys.get(name)
        return not self.settled and st is not None and not st.done

    def fused_step(self, entries: Dict[str, FusedEntry], egress_marks: bool = False) -> List[str]:
        """Aggregate-and-step every key in ``entries`` that is still pending, one launch per run of keys
        that share the aggregation signature, the entry signature and the layout offset; returns the names
        stepped.  d = fin(acc) is also stored to the round's accumulator (a later materialize() reads it).

        ``egress_marks``: the caller guarantees the entries' optimizer offsets increase with the aggregation
        offsets and cover the optimizer's whole parameter buffer; launches are then split at every
        EGRESS_CHUNK bytes and each piece records a readiness mark (``fedavg_mark``) on the parameter
        bytes it finalised, so the D2H of the new weights (``fedavg_d2h_marked``) overlaps the rest."""
        from .engine import EGRESS_CHUNK, TILE

        eng = self.engine
        chunk = max(EGRESS_CHUNK // 4 // TILE, 1) * TILE
        stepped: List[str] = []
        with self._locked():
            if egress_marks:
                eng.ctx.marks_reset()
            if self.settled:
                return stepped
            for group in eng._runs(self.keys):
                sub: List[object] = []
                sub_key: Optional[Tuple] = None

                def flush():
                    if sub:
                        ent = entries[sub[0].name]
                        delta = ent.offset - sub[0].offset
                        epi = _shifted(ent.epi, delta)
                        if egress_marks:
                            b, e = sub[0].offset, sub[0].arena.launch_end(sub[-1])
                            while b < e:
                                hi = min(e, (b // chunk + 1) * chunk)
                                eng._launch_run(sub, True, self.acc.ptr, epi, rng=(b, hi))
                                eng.ctx.mark((hi + delta) * 4)
                                b = hi
                        else:
                            eng._launch_run(sub, True, self.acc.ptr, epi)
                        eng._consume(sub)
                        for st in sub:
                            st.done = True
                            stepped.append(st.name)

                for st in group:
                    ent = entries.get(st.name)
                    if ent is None:
                        flush()
                        sub, sub_key = [], None
                        continue
                    key = (ent.sig, ent.offset - st.offset)
                    if sub and key == sub_key:
                        sub.append(st)
                    else:
                        flush()
                        sub, sub_key = [st], key
                flush()
            if all(st.done for st in self.keys.values()):
                self.settle()  # nothing left to launch: recycle the slots now
        return stepped

    def fused_apply(self, bases: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        """WEIGHT_DIFF apply ``base + d`` (full_model_shareable_generator.py:58-67) fused with the aggregation:
        the fp32 host bases are staged at the keys' aggregation offsets, and the aggregation launch carries
        an SGD(lr = 1) epilogue -- ``fma(-d, -1, base)`` is the correctly rounded ``base + d``, the
        reference's single fp32 add -- so d never leaves HBM.  Returns new host arrays for the keys applied
        (the ones still pending with a matching shape); d is stored to the accumulator as well."""
        eng = self.engine
        with self._locked():
            todo = {n: np.ascontiguousarray(b) for n, b in bases.items()
                    if self.fusable(n) and b.dtype == np.float32 and tuple(b.shape) == tuple(self.keys[n].shape)}
            if not todo:
                return {}
            ctx = eng.ctx
            span = max(self.keys[n].offset + self.keys[n].n for n in todo)
            span = (span + 63) // 64 * 64
            buf = ctx.alloc(span * 4)
            pieces = sorted((self.keys[n].offset * 4, b.ctypes.data, b.nbytes) for n, b in todo.items())
            ctx.h2d_tiled_multi(buf.ptr, 4096 * 4, 4096 * 4, pieces)  # tile == stride: contiguous
            e = N.Epilogue()
            e.kind = N.FEDAVG_EPI_SGD
            e.lr = 1.0
            e.first_step = 1
            e.param = buf.ptr  # momentum 0: no momentum buffer
            entries = {n: FusedEntry(self.keys[n].offset, e, 0) for n in todo}
            done = self.fused_step(entries)
            host = np.empty(span, dtype=np.float32)
            ctx.d2h(host, buf.ptr)
            buf.close()
            out = {}
            for n in done:
                st = self.keys[n]
                out[n] = host[st.offset:st.offset + st.n].reshape(st.shape)
            return out

    def value(self, name: str):
        """The aggregated value of one key, as the eager ``DeviceFedAvg.result()`` returns it."""
        with self._locked():
            if name in self._values:
                return self._values[name]
            self.settle()
            st = self.keys[name]
            ctx = self.engine.ctx
            src = self.acc.ptr + st.offset * 4
            if st.torch_device is not None:
                t = torch.empty(st.shape, dtype=torch.float32, device=st.torch_device)
                ctx.d2d(t.data_ptr(), src, st.n * 4)
                ctx.sync()
                v = t
            else:
                arr = np.empty(st.n, dtype=np.float32)
                ctx.d2h(arr, src)
                arr = arr.reshape(st.shape)
                if st.container == "torch":
                    v = torch.from_numpy(arr)
                else:
                    v = arr[()] if arr.ndim == 0 else arr
            self._values[name] = v
            return v


class _Locks:
    """engine.lock then ctx.lock, the order every engine entry point takes them in."""

    def __init__(self, engine):
        self.engine = engine

    def __enter__(self):
        self.engine.lock.acquire()
        try:
            self.engine.ctx.lock.acquire()
        except BaseException:
            self.engine.lock.release()
            raise
        return self

    def __exit__(self, *exc):
        self.engine.ctx.lock.release()
        self.engine.lock.release()
        return False


class DeferredValue:
    """An aggregated value still in HBM (one key of a deferred round).  ``materialize()`` returns what the
    eager path returns (numpy array / torch tensor of the key's container and shape); reading it any other
    way (``np.asarray``, arithmetic) materialises it first."""

    __slots__ = ()

    shape: tuple
    container: str

    def materialize(self):  # pragma: no cover - abstract
        raise NotImplementedError

    @property
    def dtype(self):
        return torch.float32 if self.container == "torch" else np.dtype(np.float32)

    @property
    def ndim(self) -> int:
        return len(self.shape)

    def __array__(self, dtype=None, copy=None):
        v = self.materialize()
        a = v.numpy() if (torch is not None and isinstance(v, torch.Tensor) and v.device.type == "cpu") else v
        if torch is not None and isinstance(a, torch.Tensor):
            a = a.cpu().numpy()
        return np.asarray(a, dtype=dtype)

    # arithmetic on the materialised value (the reference's consumers do ``base + diff``)
    def __add__(self, o):
        return self.materialize() + o

    def __radd__(self, o):
        return o + self.materialize()

    def __sub__(self, o):
        return self.materialize() - o

    def __rsub__(self, o):
        return o - self.materialize()

    def __mul__(self, o):
        return self.materialize() * o

    def __rmul__(self, o):
        return o * self.materialize()

    def __truediv__(self, o):
        return self.materialize() / o

    def __neg__(self):
        return -self.materialize()


class DeferredAggregate(DeferredValue):
    """The aggregated value of one key of a ``DeferredRound`` on one device."""

    __slots__ = ("round", "name", "__weakref__")

    def __init__(self, rnd: DeferredRound, name: str):
        self.round = rnd
        self.name = name

    @property
    def _state(self):
        return self.round.keys[self.name]

    @property
    def shape(self):
        return self._state.shape

    @property
    def container(self) -> str:
        return self._state.container

    @property
    def size(self) -> int:
        return self._state.n

    def fusable(self, device: int) -> bool:
        return self.round.device == device and self.round.fusable(self.name)

    def materialize(self):
        return self.round.value(self.name)

    def __repr__(self) -> str:
        return f"DeferredAggregate({self.name!r}, shape={self.shape}, {self.container}, device={self.round.device})"


class ShardedDeferredAggregate(DeferredValue):
    """One key aggregated in parameter buckets over several devices (``sharding.ShardedFedAvg``), still in
    HBM: ``pieces`` = [(lo, hi, DeferredAggregate)] over the flattened key, in bucket order.  A sharded
    device optimizer steps each piece on its own device (``fusable``); ``materialize()`` assembles the
    pieces as the eager sharded result does."""

    __slots__ = ("name", "shape", "container", "pieces", "_value", "__weakref__")

    def __init__(self, name: str, shape: tuple, container: str, pieces: List[Tuple[int, int, DeferredAggregate]]):
        self.name = name
        self.shape = tuple(shape)
        self.container = container
        self.pieces = list(pieces)
        self._value = None

    @property
    def size(self) -> int:
        return int(np.prod(self.shape, dtype=np.int64)) if self.shape else 1

    def materialize(self):
        if self._value is None:
            vals = [d.materialize() for _, _, d in self.pieces]
            if torch is not None and isinstance(vals[0], torch.Tensor):
                flat = torch.cat([v.reshape(-1) for v in vals]) if len(vals) > 1 else vals[0].reshape(-1)
                self._value = flat.reshape(self.shape)
            else:
                flat = np.concatenate([np.asarray(v).reshape(-1) for v in vals]) if len(vals) > 1 \
                    else np.asarray(vals[0]).reshape(-1)
                res = flat.reshape(self.shape)
                self._value = res[()] if res.ndim == 0 else res
        return self._value

    def __repr__(self) -> str:
        devs = [d.round.device for _, _, d in self.pieces]
        return f"ShardedDeferredAggregate({self.name!r}, shape={self.shape}, {self.container}, devices={devs})"


def materialize_deferred(v):
    """``v.materialize()`` for a deferred value (one device or sharded), ``v`` otherwise."""
    return v.materialize() if isinstance(v, DeferredValue) else v
