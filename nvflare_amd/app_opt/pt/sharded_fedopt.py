"""The FedOpt server step on several GPUs of one server process, by parameter bucket (rows a10 / e).

SURVEY.md section 8(e): every parameter is an independent unit, so the server optimizer's state shards
like the aggregation does -- "FedOpt state (p, m, v) shards identically, with no collective".  With
``devices=[d0, d1, ...]`` on both the aggregator (``sharding.ShardedFedAvg``, ``defer_result=True``) and
``PTFedOptModelShareableGenerator``, device ``d_b`` holds bucket ``b`` of every parameter
(``sharding.bucket_ranges``, the aggregation's own split) together with its optimizer state, and steps it
in the same launch that aggregates that bucket of every client (the ``ShardedDeferredAggregate``'s piece
on that device).  The new weights leave every GPU over its own PCIe link (``fedavg_d2h_multi``, one call
per device, page-locked destination) straight into one host array; the model's parameters become views of
it.  Arithmetic per element is the single-device path's, so results are bit-identical to it.

Layout:

* one ``DeviceServerOptimizer`` per device over a *shard module*: a module tree with the original
  parameter names whose parameters are the flat bucket slices, and a *shard optimizer* of the original's
  type with the same param groups (hyperparameters copied from the original before every step, so lr
  schedulers on the original optimizer keep working);
* the original model lives on the host: its parameters are views of the latest host weights.  A parameter
  the caller modifies in place (``load_state_dict``, ``param.copy_``: its ``_version`` moves) is uploaded to
  its shards before the next step.  Per-parameter optimizer state lives in the shard optimizers
  (``shards[b].optimizer.state``, views of each device's buffers); ``export_state`` assembles it into the
  original optimizer's ``state`` (host tensors of the parameters' shapes) whenever the original is asked for
  its ``state_dict()`` (a pre-hook) and before the generator re-binds a new sharded image of the same
  optimizer, so neither sees stale or empty moments.
"""

from __future__ import annotations

import threading
import weakref
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...deferred import ShardedDeferredAggregate, materialize_deferred
from ...device import HostArenaPool
from ...sharding import bucket_ranges
from .fedopt import DeviceServerOptimizer

_HOST_ALIGN = 16  # elements: every parameter of the host weights starts 64-byte aligned


def shard_spans(named: Sequence[Tuple[str, torch.nn.Parameter]], n_shards: int) -> List[Dict[str, Tuple[int, int]]]:
    """Per shard, {parameter name: (lo, hi)} of its flattened bucket -- ``ShardedFedAvg``'s split of the
    same key (``bucket_ranges``); empty buckets and empty parameters are left out."""
    spans: List[Dict[str, Tuple[int, int]]] = [dict() for _ in range(n_shards)]
    for name, p in named:
        n = p.numel()
        if n == 0:
            continue
        for b, (lo, hi) in enumerate(bucket_ranges(n, n_shards)):
            if hi > lo:
                spans[b][name] = (lo, hi)
    return spans


def shard_module(named: Sequence[Tuple[str, torch.nn.Parameter]], span: Dict[str, Tuple[int, int]]) -> torch.nn.Module:
    """A module tree whose ``named_parameters()`` are the original names, each parameter the flat slice
    ``[lo, hi)`` of the original (copied)."""
    root = torch.nn.Module()
    for name, p in named:
        if name not in span:
            continue
        lo, hi = span[name]
        *path, leaf = name.split(".")
        mod = root
        for part in path:
            child = mod._modules.get(part)
            if child is None:
                child = torch.nn.Module()
                mod.add_module(part, child)
            mod = child
        mod.register_parameter(leaf, torch.nn.Parameter(p.detach().reshape(-1)[lo:hi].clone()))
    return root


def shard_optimizer(optimizer: torch.optim.Optimizer, named: Sequence[Tuple[str, torch.nn.Parameter]],
                    module: torch.nn.Module, span: Dict[str, Tuple[int, int]]) -> torch.optim.Optimizer:
    """An optimizer of ``optimizer``'s type over ``module``'s parameters with the same param groups (in the
    same order, hyperparameters copied; a group may be empty) and the original's per-parameter state sliced
    to the bucket (tensors shaped like the parameter) or copied (scalar state such as ``step``)."""
    by_id = {id(p): n for n, p in named}
    mine = dict(module.named_parameters())
    groups = []
    for g in optimizer.param_groups:
        params = [mine[by_id[id(p)]] for p in g["params"] if by_id.get(id(p)) in mine]
        groups.append({**{k: v for k, v in g.items() if k != "params"}, "params": params})
    opt = type(optimizer)(groups)
    originals = dict(named)
    for name, sp in mine.items():
        st = optimizer.state.get(originals[name])
        if not st:
            continue
        lo, hi = span[name]
        n = originals[name].numel()
        opt.state[sp] = {k: (v.detach().reshape(-1)[lo:hi].clone() if isinstance(v, torch.Tensor) and v.numel() == n
                             else (v.clone() if isinstance(v, torch.Tensor) else v))
                         for k, v in st.items()}
    return opt


class ShardedServerOptimizer:
    """The device server optimizer of ``fedopt.DeviceServerOptimizer`` split by parameter bucket over
    ``devices`` (module docstring)."""

    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, devices: Sequence[int]):
        self.model = model
        self.optimizer = optimizer
        self.devices = [int(d) for d in devices]
        if len(self.devices) < 2:
            raise ValueError("ShardedServerOptimizer needs at least two devices")
        DeviceServerOptimizer._kind(optimizer)  # supported optimizer type, or NotImplementedError
        named = list(model.named_parameters())
        grouped = {id(p) for g in optimizer.param_groups for p in g["params"]}
        for name, p in named:
            if p.dtype != torch.float32:
                raise TypeError(f"nvflare_amd: parameter {name!r} is {p.dtype}; the device optimizer runs float32")
            if id(p) not in grouped:
                raise ValueError(f"nvflare_amd: parameter {name!r} is not managed by the optimizer")
        self.params: Dict[str, torch.nn.Parameter] = dict(named)
        self.spans = shard_spans(named, len(self.devices))
        self.shards: List[DeviceServerOptimizer] = []
        for b, dev in enumerate(self.devices):
            mod = shard_module(named, self.spans[b])
            shard = DeviceServerOptimizer(mod, shard_optimizer(optimizer, named, mod, self.spans[b]), dev)
            shard.pipelined_egress = False  # every device's weights leave in _egress; shards may share a context
            self.shards.append(shard)
        # host weights: every parameter contiguous at a 64-byte aligned offset of one flat fp32 array
        self.layout: Dict[str, Tuple[int, int]] = {}
        off = 0
        for name, p in named:
            self.layout[name] = (off, p.numel())
            off += (p.numel() + _HOST_ALIGN - 1) // _HOST_ALIGN * _HOST_ALIGN
        self.total = max(off, _HOST_ALIGN)
        self.host_pool = HostArenaPool()
        # the weights handed out by to_host (independent of the live parameters); depth 2: the caller holds last
        # round's hand-out while this round's is pulled, so two page-locked arrays suffice (depth 3 here
        # beside host_pool's 3 page-locked five full-model arrays)
        self.out_pool = HostArenaPool(depth=2)
        self._pool = ThreadPoolExecutor(max_workers=len(self.devices), thread_name_prefix="nvflare-amd-fedopt-shard")
        self._pool_fin = weakref.finalize(self, self._pool.shutdown, wait=False)  # a re-bound generator drops us
        me = weakref.ref(self)

        def _export(opt, _me=me):  # optimizer.state_dict() sees the shards' current state
            obj = _me()
            if obj is not None and obj.optimizer is opt:
                obj.export_state()

        self._hook = optimizer.register_state_dict_pre_hook(_export) \
            if hasattr(optimizer, "register_state_dict_pre_hook") else None
        self._lock = threading.Lock()
        model.to("cpu")  # buffers (batch-norm statistics) stay with the model; parameters are re-pointed below
        host = self.host_pool.take(self.total, pin=self.shards[0].ctx)
        with torch.no_grad():
            for name, p in named:
                o, n = self.layout[name]
                host[o:o + n] = p.detach().reshape(-1).numpy()
        self._point_params(host)

    # -- host weights ------------------------------------------------------------------------------
    def _point_params(self, host: np.ndarray) -> None:
        """Re-point every model parameter at its slice of ``host`` and remember the version counters."""
        self.host = host
        for name, p in self.params.items():
            o, n = self.layout[name]
            p.data = torch.from_numpy(host[o:o + n]).view(p.shape)
        self._versions = {name: p._version for name, p in self.params.items()}

    def is_bound(self) -> bool:
        named = dict(self.model.named_parameters())
        if set(named) != set(self.params):
            return False
        base = self.host.ctypes.data
        return all(named[n] is p and p.data_ptr() == base + 4 * self.layout[n][0] for n, p in self.params.items())

    def _upload_modified(self) -> None:
        """Parameters written in place since the last step (``_version`` moved) go to their shards."""
        changed = [n for n, p in self.params.items() if p._version != self._versions.get(n)]
        if not changed:
            return
        with torch.no_grad():
            for b, shard in enumerate(self.shards):
                for n in changed:
                    if n in self.spans[b]:
                        lo, hi = self.spans[b][n]
                        s = shard.by_name[n]
                        s.param.data.copy_(self.params[n].detach().reshape(-1)[lo:hi])
            for shard in self.shards:
                torch.cuda.synchronize(shard.torch_device)
        for n in changed:
            self._versions[n] = self.params[n]._version

    def _sync_groups(self) -> None:
        """The original optimizer's hyperparameters (lr schedulers write them) into every shard optimizer."""
        for shard in self.shards:
            for g, sg in zip(self.optimizer.param_groups, shard.optimizer.param_groups):
                for k, v in g.items():
                    if k != "params":
                        sg[k] = v

    # -- the step ----------------------------------------------------------------------------------
    def _split(self, model_diff: Dict) -> List[Dict]:
        """Per shard, {name: this bucket's difference}: the ShardedDeferredAggregate's own piece when it lies on
        the shard's device with the shard's span (aggregated and stepped in one launch there), else a slice of
        the materialised difference."""
        per: List[Dict] = [dict() for _ in self.shards]
        for name, d in model_diff.items():
            if name not in self.params:
                continue
            holders = [b for b in range(len(self.shards)) if name in self.spans[b]]
            if isinstance(d, ShardedDeferredAggregate) and len(d.pieces) == len(holders) and all(
                    (lo, hi) == self.spans[b][name] and piece.round.device == self.shards[b].hip_device
                    for b, (lo, hi, piece) in zip(holders, d.pieces)):
                for b, (_, _, piece) in zip(holders, d.pieces):
                    per[b][name] = piece
                continue
            v = materialize_deferred(d)
            flat = v.detach().reshape(-1) if isinstance(v, torch.Tensor) else np.ascontiguousarray(np.asarray(v)).reshape(-1)
            for b in holders:
                lo, hi = self.spans[b][name]
                per[b][name] = flat[lo:hi]
        return per

    def _check(self, model_diff: Dict) -> None:
        """fedopt.DeviceServerOptimizer._check_diffs on the whole parameters (before any shard is touched)."""
        for name, p in self.params.items():
            if name not in model_diff:
                continue
            d = model_diff[name]
            if not hasattr(d, "shape") or not hasattr(d, "dtype"):
                d = np.asarray(d)
            if d.dtype not in (torch.float32, np.dtype(np.float32)):
                raise RuntimeError(f"assigned grad has data of a different type ({d.dtype}) for {name!r}")
            if tuple(d.shape) != tuple(p.shape):
                raise RuntimeError(f"assigned grad has data of a different size for {name!r}")

    def step(self, model_diff: Dict) -> List[str]:
        """One server step on g = -diff for every parameter named in ``model_diff`` (all shards in parallel,
        one thread per device); the new weights are in the model's parameters (host views) on return."""
        with self._lock:
            self._check(model_diff)
            self._upload_modified()
            self._sync_groups()
            per = self._split(model_diff)
            stepped = set()
            for names in self._pool.map(lambda sp: sp[0].step(sp[1]), zip(self.shards, per)):
                stepped.update(names)
            self._egress()
            return [n for n in self.params if n in stepped]

    def _pull(self, pool: HostArenaPool) -> np.ndarray:
        """Every device's buckets into one fresh host array from ``pool`` (each device over its own PCIe link, one
        fedavg_d2h_multi each, in parallel)."""
        host = pool.take(self.total, pin=self.shards[0].ctx)

        def pull(b: int) -> None:
            shard = self.shards[b]
            torch.cuda.synchronize(shard.torch_device)
            pieces = []
            for name, (lo, hi) in self.spans[b].items():
                s = shard.by_name[name]
                pieces.append((4 * (self.layout[name][0] + lo), 4 * s.offset, 4 * (hi - lo)))
            with shard.ctx.lock:
                shard.ctx.d2h_multi(host, shard.p.data_ptr(), pieces)

        list(self._pool.map(pull, range(len(self.shards))))
        return host

    def _egress(self) -> None:
        """The new weights into a fresh host array that the model's parameters are re-pointed at."""
        self._point_params(self._pull(self.host_pool))

    def to_host(self, state: Dict, preserve_torch: bool) -> Dict:
        """state_dict -> host values as the reference hands them out (fedopt.py:232-236: ``detach().cpu().clone()``
        for torch, ``detach().cpu().numpy()`` of its GPU model for numpy): independent, writable copies.  The
        parameters' values are pulled from the devices a second time into an array of their own (``out_pool``;
        every device over its own link, in parallel -- cheaper than a host copy of the weights), so nothing the
        caller does to the returned weights reaches the live parameters or the shards' next step; other entries
        are copied as the single-device path copies them."""
        out = {}
        base = self.host.ctypes.data
        handout = None
        for k, v in state.items():
            lay = self.layout.get(k)
            if lay is not None and v.dtype == torch.float32 and v.data_ptr() == base + 4 * lay[0]:
                if handout is None:
                    with self._lock:
                        # a parameter written in place on the host since the last step (load_state_dict, copy_) is
                        # on the host only: upload it first, or the pull below would hand out the stale shard value
                        self._upload_modified()
                        handout = self._pull(self.out_pool)
                h = handout[lay[0]:lay[0] + lay[1]].reshape(tuple(v.shape))
                out[k] = torch.from_numpy(h) if preserve_torch else h
                continue
            h = v.detach().cpu()
            out[k] = h.clone() if preserve_torch else h.numpy()
        return out

    def export_state(self) -> None:
        """Every parameter's optimizer state, assembled from its shards into the original optimizer's ``state``:
        per-element tensors (exp_avg, momentum_buffer, ...) as host tensors of the parameter's shape, the shard
        slices in bucket order; scalar entries (step, mu_product, eta, ...) from the first shard holding the
        parameter (every shard of a parameter steps it together).  A parameter no shard has stepped keeps its
        original state."""
        with self._lock:
            for shard in self.shards:
                torch.cuda.synchronize(shard.torch_device)
            for name, p in self.params.items():
                holders = [b for b in range(len(self.shards)) if name in self.spans[b]]
                sts = [self.shards[b].optimizer.state.get(self.shards[b].by_name[name].param) for b in holders]
                if not holders or not all(sts):
                    continue
                out = {}
                for key, v0 in sts[0].items():
                    if isinstance(v0, torch.Tensor) and v0.dim() >= 1:
                        parts = [st[key].detach().reshape(-1).cpu() for st in sts]
                        out[key] = torch.cat(parts).reshape(p.shape) if len(parts) > 1 else parts[0].clone().reshape(p.shape)
                    else:
                        out[key] = v0.clone() if isinstance(v0, torch.Tensor) else v0
                self.optimizer.state[p] = out

    def release(self) -> None:
        if self._hook is not None:
            self._hook.remove()
            self._hook = None
        self._pool_fin.detach()
        self._pool.shutdown(wait=True)
