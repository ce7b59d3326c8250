"""Parameter-bucket sharding of the FedAvg aggregation across GPUs.

Every parameter is an independent unit of the hot path, so the flattened model splits into contiguous
buckets, one per GPU; each GPU aggregates its bucket of every client with the same arrival order and
weights.  No collective touches the data, and the result is bit-identical to one GPU -- which a
client-sharded RCCL reduce would not be (it re-associates the sums).

* ``bucket_ranges``   -- the partition (aligned so every bucket boundary is a whole tile).
* ``ShardedFedAvg``   -- one process, N devices: each contribution's arrays are sliced (views, no copy)
                         and staged to every device's engine from a thread per device, so the N PCIe
                         links run in parallel; results are reassembled per key.
* ``bench.py`` under torchrun uses the same partition with one process per GPU.
"""

from __future__ import annotations

import logging
import threading
import weakref
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .device import BF16_NP, HostArenaPool
from .engine import DeviceFedAvg, is_torch_tensor

BUCKET_ALIGN = 4096  # elements: a bucket boundary never splits a kernel tile


def bucket_ranges(total: int, parts: int, align: int = BUCKET_ALIGN) -> List[Tuple[int, int]]:
    """Split [0, total) into `parts` contiguous ranges whose inner boundaries are multiples of `align`
    and whose sizes differ by at most one `align` unit."""
    if parts < 1:
        raise ValueError("parts must be >= 1")
    units = (total + align - 1) // align
    base, extra = divmod(units, parts)
    out, start = [], 0
    for r in range(parts):
        # the extra units go to the LAST buckets, so the partial last unit evens out instead of adding up
        n_units = base + (1 if r >= parts - extra else 0)
        end = min(total, start + n_units * align)
        out.append((start, end))
        start = end
    return out


def _flat_view(v):
    if is_torch_tensor(v):
        t = v.detach()
        return t.contiguous().reshape(-1)
    return np.ascontiguousarray(v).reshape(-1)


class ShardedFedAvg:
    """DeviceFedAvg over several devices, by parameter bucket: every key of n elements is split into
    `len(devices)` contiguous, tile-aligned pieces (keys shorter than one tile stay whole on one
    device).  Partial keys and keys first seen late work exactly as on one device, bucket by bucket."""

    direct_egress = True  # False: round 2's per-key concatenation of the bucket results (A/B tools only)

    def __init__(self, devices: Sequence[int], max_resident_bytes: Optional[int] = None):
        self.devices = list(devices)
        if not self.devices:
            raise ValueError("at least one device")
        self.engines = [DeviceFedAvg(device=d, max_resident_bytes=max_resident_bytes) for d in self.devices]
        self.lock = threading.RLock()
        self._pool = ThreadPoolExecutor(max_workers=len(self.devices), thread_name_prefix="nvflare-amd-shard")
        self._pool_fin = weakref.finalize(self, self._pool.shutdown, wait=False)  # threads end with the engine
        self._shapes: Dict[str, tuple] = {}

    def _pieces(self, bucket: int, items):
        """(subkey, 1-D slice view) of every key overlapping `bucket`; each subkey's place in its whole key goes
        to the bucket's engine (``key_spans``: torch's 16-bit scalar-loop elements are those of the whole
        tensor, engine.py ``_torch16_tails``)."""
        out = []
        spans = self.engines[bucket].key_spans
        for k, v in items:
            n = int(np.prod(v.shape, dtype=np.int64)) if v.shape else 1
            lo, hi = bucket_ranges(n, len(self.engines))[bucket]
            if lo < hi or (n == 0 and bucket == 0):
                sub = f"{k}\x00{lo}"
                spans[sub] = (lo, n)
                out.append((sub, _flat_view(v)[lo:hi]))
        return out

    def add(self, items: List[Tuple[str, Any]], weight, weighted: bool) -> None:
        """Stage one contribution's pieces on every device in parallel; all or nothing (engine.DeviceFedAvg.add)."""
        with self.lock:
            # Each engine sees only flat slices, so a reshaped contribution with the same element count
            # would pass every shard: check the shape here, for every item before any shard is staged,
            # with the single-device engine's message (engine.py DeviceFedAvg._register_key).
            new = {}
            for k, v in items:
                shape = tuple(v.shape)
                first = self._shapes.get(k, new.get(k))
                if first is not None and first != shape:
                    raise ValueError(f"nvflare_amd: key {k!r} shape {shape} != first contribution's {first}")
                new.setdefault(k, shape)
            introduced = [k for k in new if k not in self._shapes]
            for k, shape in new.items():
                self._shapes.setdefault(k, shape)
            futs = [self._pool.submit(eng.add, self._pieces(b, items), weight, weighted)
                    for b, eng in enumerate(self.engines)]
            txs, err = [], None
            for f in futs:
                try:
                    txs.append(f.result())
                except BaseException as e:  # noqa: B036 - re-raised below, after the other buckets are undone
                    txs.append(None)
                    err = err or e
            if err is not None:
                # all or nothing across buckets too: the buckets that staged give their piece back (each engine's
                # add is already atomic), so no bucket counts a weight the others do not.  Every bucket is undone
                # even when one undo fails; the staging error is the one raised, the undo failures chained to it.
                undo_errs = []
                for b, (eng, tx) in enumerate(zip(self.engines, txs)):
                    if tx is not None:
                        try:
                            eng.undo_add(tx)
                        except BaseException as e:  # noqa: B036 - reported with the staging error below
                            undo_errs.append((b, e))
                for k in introduced:
                    self._shapes.pop(k, None)
                if undo_errs:
                    # the undo failures came after the staging error: reported beside it (a note on 3.11+, and the
                    # log), never as its cause -- err is re-raised with its own __cause__ unchanged
                    msg = "; ".join(f"bucket {b}: {type(e).__name__}: {e}" for b, e in undo_errs)
                    note = f"nvflare_amd: undoing the other buckets also failed ({msg})"
                    logging.getLogger(__name__).error(note)
                    if hasattr(err, "add_note"):
                        err.add_note(note)
                    else:
                        err.undo_failures = undo_errs
                raise err

    def _assemble(self, k: str, plist: List[Tuple[int, Any]]):
        """The whole key from its bucket results (plist sorted by offset)."""
        shape = self._shapes[k]
        arrs = [a for _, a in plist]
        if is_torch_tensor(arrs[0]):
            import torch

            flat = torch.cat([a.reshape(-1) for a in arrs]) if len(arrs) > 1 else arrs[0].reshape(-1)
            return flat.reshape(shape)
        flat = np.concatenate([np.asarray(a).reshape(-1) for a in arrs]) if len(arrs) > 1 else np.asarray(arrs[0]).reshape(-1)
        res = flat.reshape(shape)
        return res[()] if res.ndim == 0 else res

    def _bucket_results(self, deferred: bool, dests=None) -> Dict[str, List[Tuple[int, Any]]]:
        if deferred:
            def fn(b):
                return self.engines[b].result_deferred() if self.engines[b].keys else {}
        else:
            def fn(b):
                return self.engines[b].result(host_dest=dests[b] if dests else None) if self.engines[b].keys else {}
        pieces: Dict[str, List[Tuple[int, Any]]] = {}
        for res in self._pool.map(fn, range(len(self.engines))):
            for sub, arr in res.items():
                k, off = sub.rsplit("\x00", 1)  # a key may itself hold NULs (SCAFFOLD control prefix)
                pieces.setdefault(k, []).append((int(off), arr))
        for plist in pieces.values():
            plist.sort(key=lambda x: x[0])
        return pieces

    def _direct_plan(self):
        """Whole-key host destinations for the keys whose every bucket is a host-container arena key: one host
        array per element format (page-locked once, reused across rounds by a HostArenaPool), each such key at its
        own offset.  Returns ({key: (array, element offset, container)}, per-engine {subkey: (array, offset)})."""
        fmt: Dict[str, Any] = {}
        for e in self.engines:
            for sub, st in e.keys.items():
                k = sub.rsplit("\x00", 1)[0]
                ok = st.arena is not None and st.n > 0 and st.torch_device is None
                tag = (st.arena.np_dtype, st.container) if ok else None
                fmt[k] = tag if fmt.get(k, tag) == tag and tag is not None else False
        sizes: Dict[Any, int] = {}
        offsets: Dict[str, Tuple[Any, int]] = {}
        for k, tag in fmt.items():
            if not tag:
                continue
            n = int(np.prod(self._shapes[k], dtype=np.int64)) if self._shapes[k] else 1
            offsets[k] = (tag[0], sizes.get(tag[0], 0))
            sizes[tag[0]] = sizes.get(tag[0], 0) + n
        hosts = {dt: self._host_pool(dt).take(n, dt, pin=self.engines[0].ctx) for dt, n in sizes.items()}
        plan = {k: (hosts[dt], off, fmt[k][1]) for k, (dt, off) in offsets.items()}
        dests = []
        for e in self.engines:
            d = {}
            for sub in e.keys:
                k, lo = sub.rsplit("\x00", 1)
                if k in plan:
                    d[sub] = (plan[k][0], plan[k][1] + int(lo))
            dests.append(d)
        return plan, dests

    def _host_pool(self, dt):
        pools = self.__dict__.setdefault("_host_pools", {})
        if dt not in pools:
            pools[dt] = HostArenaPool()
        return pools[dt]

    def _view(self, k: str, host: np.ndarray, off: int, container: str):
        """Key k as a view of the host array its buckets were copied into (the engine's _materialize rules)."""
        shape = self._shapes[k]
        n = int(np.prod(shape, dtype=np.int64)) if shape else 1
        arr = host[off: off + n].reshape(shape)
        if container == "torch":
            import torch

            if arr.dtype == BF16_NP:
                return torch.from_numpy(arr.view(np.uint16)).view(torch.bfloat16)
            return torch.from_numpy(arr)
        return arr[()] if arr.ndim == 0 else arr

    def result(self) -> Dict[str, Any]:
        """Every bucket finalised on its device; keys whose buckets are all host-container arena keys are copied by
        each device straight to their place in one page-locked host array (each GPU over its own PCIe link, no
        host-side concatenation); others (device tensors, side-buffer keys) are reassembled per key."""
        with self.lock:
            plan, dests = self._direct_plan() if self.direct_egress else ({}, None)
            pieces = self._bucket_results(False, dests)
            return {k: self._view(k, *plan[k]) if k in plan else self._assemble(k, plist) for k, plist in pieces.items()}

    def result_deferred(self) -> Dict[str, Any]:
        """``result()`` with every fp32 key left on the devices, one ``ShardedDeferredAggregate`` per key whose
        bucket pieces are ``DeferredAggregate`` values of each device's round (engine.result_deferred); other
        keys come back eagerly, assembled."""
        from .deferred import DeferredAggregate, ShardedDeferredAggregate

        with self.lock:
            out = {}
            for k, plist in self._bucket_results(True).items():
                if all(isinstance(v, DeferredAggregate) for _, v in plist):
                    spans = [(lo, lo + v.size, v) for lo, v in plist]
                    out[k] = ShardedDeferredAggregate(k, self._shapes[k], plist[0][1].container, spans)
                else:
                    out[k] = self._assemble(k, [(lo, getattr(v, "materialize", lambda v=v: v)()) for lo, v in plist])
            return out

    @property
    def keys(self):
        return {s.rsplit("\x00", 1)[0] for e in self.engines for s in e.keys}

    @property
    def stats(self):
        agg = {}
        for e in self.engines:
            for k, v in e.stats.items():
                agg[k] = agg.get(k, 0) + v
        return agg

    def reset(self) -> None:
        with self.lock:
            for e in self.engines:
                e.reset()
            self._shapes.clear()

    def release(self) -> None:
        for e in self.engines:
            e.release()
        self._pool_fin.detach()
        self._pool.shutdown(wait=True)
