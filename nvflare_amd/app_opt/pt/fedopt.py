"""Drop-in ``PTFedOptModelShareableGenerator`` with the server optimizer step on the MI355X (row a10 / f1).

Reference: ``nvflare/app_opt/pt/fedopt.py:29-270``.  Same constructor, START_RUN set-up (model from the
engine or a module, optimizer / lr scheduler built from ``{'path'|'class_path', 'args'}``), the same
``system_panic`` conditions, WEIGHT_DIFF-only input, ``-1.0 * diff`` as the gradient of every named
parameter present in the diff, FedAvg (``base + diff``) for the other keys, and the same output
representation (torch tensors if the global model holds tensors, numpy otherwise).

What differs is where the step runs.  The reference sets ``param.grad`` and calls
``optimizer.step()``; here the model's parameters are re-pointed into ONE flat fp32 buffer in HBM and
``torch.optim.SGD`` / ``Adam`` / ``AdamW`` / ``Adagrad`` / ``RMSprop`` / ``Adamax`` / ``NAdam`` / ``RAdam`` / ``Rprop`` / ``ASGD`` steps are executed by the HIP fused-epilogue kernel
(``fedavg_accumulate_tiled_epi`` with the aggregated difference as ``acc_in``), with torch's
single-tensor rounding sequence (``tests/test_fedopt_oracle.py``).  The torch optimizer object is kept
for its ``param_groups`` (read every step, so lr schedulers work unchanged) and its ``state`` is filled
with views of the device buffers (``momentum_buffer`` / ``exp_avg`` / ``exp_avg_sq`` / ``max_exp_avg_sq``
with amsgrad / Adagrad's ``sum`` / Adamax's ``exp_inf`` / ``step``), so ``optimizer.state_dict()`` checkpoints as before.  Other optimizers raise:
there is no CPU fallback.

``device`` names the HIP device ("cuda:N" or N); "cpu" (and None) select $NVFLARE_AMD_DEVICE / 0 --
the product has no CPU path.
"""

from __future__ import annotations

import importlib
import os
import time
import warnings
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ... import _native as N
from ...app_common.shareablegenerators.full_model_shareable_generator import (
    FullModelShareableGenerator,
    apply_weight_diff,
)
from ...compat import (
    AppConstants,
    DataKind,
    EventType,
    FLContext,
    Learnable,
    MetaKey,
    ModelLearnableKey,
    Shareable,
    from_shareable,
    make_model_learnable,
)
from ...deferred import DeferredAggregate, DeferredValue, FusedEntry, materialize_deferred
from ... import torch_sqrt
from ...device import DeviceContext, HostArenaPool

_ALIGN = 64  # elements per parameter slot boundary (256 B), as in the aggregation engine


def hip_device_index(device) -> int:
    """HIP device index for a reference-style ``device`` argument."""
    if isinstance(device, int):
        return device
    if device is not None:
        d = torch.device(device)
        if d.type == "cuda":
            return 0 if d.index is None else d.index
    return int(os.environ.get("NVFLARE_AMD_DEVICE", "0"))


def build_component_from_args(args: dict):
    """``{'path'|'class_path', 'args'}`` -> instance (what ``engine.build_component`` does for these)."""
    path = args.get("path") or args.get("class_path") or args.get("name")
    if not path:
        raise ValueError(f"component args need 'path' or 'class_path': {args}")
    mod, _, cls = path.rpartition(".")
    return getattr(importlib.import_module(mod), cls)(**args.get("args", {}))


# server optimizers whose torch step takes a sqrt (exp_avg_sq.sqrt(), state_sum.sqrt(), square_avg.sqrt())
_SQRT_KINDS = (N.FEDAVG_EPI_ADAM, N.FEDAVG_EPI_ADAGRAD, N.FEDAVG_EPI_RMSPROP, N.FEDAVG_EPI_NADAM, N.FEDAVG_EPI_RADAM)

class _Slot:
    __slots__ = ("name", "param", "offset", "n", "step", "has_momentum_buffer", "state_initialised", "mu_product",
                 "eta", "mu")

    def __init__(self, name, param, offset, n):
        self.name, self.param, self.offset, self.n = name, param, offset, n
        self.step = 0.0
        self.has_momentum_buffer = False  # SGD: torch holds a momentum_buffer for this parameter
        self.state_initialised = False  # Rprop / ASGD: the state _init_group makes at the first step exists
        self.mu_product = np.float32(1.0)  # NAdam's fp32 state tensor, kept on the host
        self.eta = np.float32(0.0)  # ASGD's fp32 eta / mu state tensors, kept on the host
        self.mu = np.float32(1.0)

    def host_key(self) -> tuple:
        """Per-parameter host state a launch shares (runs group parameters whose keys are equal)."""
        return (self.step, self.has_momentum_buffer, self.state_initialised, float(self.mu_product), float(self.eta),
                float(self.mu))


class DeviceServerOptimizer:
    """Flat HBM image of a model's parameters plus optimizer state, stepped by the HIP epilogue kernel.

    Layout: parameter ``j`` occupies ``[offset_j, offset_j + n_j)`` of the flat buffers ``p`` (the live
    parameter storage: ``param.data`` is a view of it), ``m`` (momentum buffer / exp_avg / Adagrad sum), ``v``
    (exp_avg_sq) and ``g`` (staged aggregated difference, allocated on first use: a round whose
    differences are deferred aggregates never needs it), offsets 256-byte aligned."""

    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, device: int):
        self.hip_device = device
        self.torch_device = torch.device("cuda", device)
        self.ctx = DeviceContext.get(device)
        self.model = model
        self.optimizer = optimizer
        self.kind = self._kind(optimizer)
        self.sqrt_mode = torch_sqrt.mode()  # torch_sqrt.MODES: the sqrt of the reference's step on this host
        self._bind()

    @staticmethod
    def _kind(optimizer) -> int:
        if isinstance(optimizer, torch.optim.SGD):
            return N.FEDAVG_EPI_SGD
        if isinstance(optimizer, torch.optim.Adam):  # AdamW subclasses Adam (decoupled_weight_decay=True)
            return N.FEDAVG_EPI_ADAM
        if isinstance(optimizer, torch.optim.Adagrad):
            return N.FEDAVG_EPI_ADAGRAD
        if isinstance(optimizer, torch.optim.RMSprop):
            return N.FEDAVG_EPI_RMSPROP
        if isinstance(optimizer, torch.optim.Adamax):
            return N.FEDAVG_EPI_ADAMAX
        if isinstance(optimizer, torch.optim.NAdam):
            return N.FEDAVG_EPI_NADAM
        if isinstance(optimizer, torch.optim.RAdam):
            return N.FEDAVG_EPI_RADAM
        if isinstance(optimizer, torch.optim.Rprop):
            return N.FEDAVG_EPI_RPROP
        if isinstance(optimizer, torch.optim.ASGD):
            return N.FEDAVG_EPI_ASGD
        raise NotImplementedError(
            f"nvflare_amd: server optimizer {type(optimizer).__module__}.{type(optimizer).__name__} has no device "
            "kernel (supported: torch.optim.SGD, Adam, AdamW, Adagrad, RMSprop, Adamax, NAdam, RAdam, Rprop, ASGD)")

    def _group_of(self) -> Dict[int, dict]:
        return {id(p): g for g in self.optimizer.param_groups for p in g["params"]}

    def _bind(self) -> None:
        named = list(self.model.named_parameters())
        groups = self._group_of()
        slots, off = [], 0
        for name, p in named:
            if p.dtype != torch.float32:
                raise TypeError(f"nvflare_amd: parameter {name!r} is {p.dtype}; the device optimizer runs float32")
            slots.append(_Slot(name, p, off, p.numel()))
            off += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        total = max(off, _ALIGN)
        dev = self.torch_device
        self.p = torch.zeros(total, dtype=torch.float32, device=dev)
        self.m = torch.zeros(total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(total, dtype=torch.float32, device=dev)
        self.vmax = None  # Adam(amsgrad=True): max_exp_avg_sq, allocated with the first amsgrad group
        if any(g.get("amsgrad") or g.get("centered") for g in self.optimizer.param_groups):  # Adam / RMSprop
            self.vmax = torch.zeros(total, dtype=torch.float32, device=dev)
        self.g = None
        self.host_pool = HostArenaPool()  # host copies of p returned by the generator, reused when released
        self.egress_pending = False  # the last fused step left readiness marks for a pipelined D2H of p
        self.pipelined_egress = True  # fused steps may leave such marks (off for the shards of a sharded step)
        with torch.no_grad():
            for s in slots:
                view = self.p[s.offset:s.offset + s.n].view(s.param.shape)
                view.copy_(s.param.detach().to(dev))
                s.param.data = view
                st = self.optimizer.state.get(s.param) or {}
                # resume from optimizer state present before binding (e.g. a loaded state_dict)
                if self.kind == N.FEDAVG_EPI_RMSPROP:
                    self._resume_rmsprop(s, st, dev)
                elif "momentum_buffer" in st and st["momentum_buffer"] is not None:
                    self.m[s.offset:s.offset + s.n].copy_(st["momentum_buffer"].reshape(-1).to(dev))
                    s.has_momentum_buffer = True
                if "exp_avg" in st:  # Adam: exp_avg_sq, Adamax: exp_inf -> v
                    self.m[s.offset:s.offset + s.n].copy_(st["exp_avg"].reshape(-1).to(dev))
                    second = st["exp_inf"] if self.kind == N.FEDAVG_EPI_ADAMAX else st["exp_avg_sq"]
                    self.v[s.offset:s.offset + s.n].copy_(second.reshape(-1).to(dev))
                    s.step = float(st["step"])
                if "step_size" in st:  # Rprop: prev -> m, step_size -> v
                    self.m[s.offset:s.offset + s.n].copy_(st["prev"].reshape(-1).to(dev))
                    self.v[s.offset:s.offset + s.n].copy_(st["step_size"].reshape(-1).to(dev))
                    s.step = float(st["step"])
                    s.state_initialised = True
                if "ax" in st:  # ASGD: ax -> m, eta / mu host scalars
                    self.m[s.offset:s.offset + s.n].copy_(st["ax"].reshape(-1).to(dev))
                    s.eta, s.mu = np.float32(float(st["eta"])), np.float32(float(st["mu"]))
                    s.step = float(st["step"])
                    s.state_initialised = True
                if "mu_product" in st:  # NAdam
                    s.mu_product = np.float32(float(st["mu_product"]))
                if "sum" in st:  # Adagrad: state made at construction (initial_accumulator_value)
                    self.m[s.offset:s.offset + s.n].copy_(st["sum"].reshape(-1).to(dev))
                    s.step = float(st["step"])
                if st.get("max_exp_avg_sq") is not None and self.vmax is not None:
                    self.vmax[s.offset:s.offset + s.n].copy_(st["max_exp_avg_sq"].reshape(-1).to(dev))
                if id(s.param) not in groups:
                    raise ValueError(f"nvflare_amd: parameter {s.name!r} is not managed by the optimizer")
        self.model.to(dev)  # buffers follow; parameters already live in self.p
        self.slots = slots
        self.by_name = {s.name: s for s in slots}
        torch.cuda.synchronize(dev)

    def _resume_rmsprop(self, s: "_Slot", st: dict, dev) -> None:
        """RMSprop state: square_avg -> m, momentum_buffer -> v, grad_avg -> vmax."""
        for key, buf in (("square_avg", self.m), ("momentum_buffer", self.v), ("grad_avg", self.vmax)):
            if st.get(key) is not None and buf is not None:
                buf[s.offset:s.offset + s.n].copy_(st[key].reshape(-1).to(dev))
        if "step" in st:
            s.step = float(st["step"])

    def is_bound(self) -> bool:
        named = dict(self.model.named_parameters())
        if set(named) != set(self.by_name):
            return False
        base = self.p.data_ptr()
        return all(named[s.name] is s.param and s.param.data_ptr() == base + 4 * s.offset for s in self.slots)

    def _expose_state(self, s: _Slot, group: dict) -> None:
        st = self.optimizer.state[s.param]
        if self.kind == N.FEDAVG_EPI_SGD:
            if s.has_momentum_buffer:  # torch stores the buffer only when momentum != 0
                st["momentum_buffer"] = self.m[s.offset:s.offset + s.n].view(s.param.shape)
        elif self.kind == N.FEDAVG_EPI_ADAGRAD:
            st["step"] = torch.tensor(s.step, dtype=torch.float32)
            st["sum"] = self.m[s.offset:s.offset + s.n].view(s.param.shape)
        elif self.kind == N.FEDAVG_EPI_RMSPROP:
            g = group
            st["step"] = torch.tensor(s.step, dtype=torch.float32)
            st["square_avg"] = self.m[s.offset:s.offset + s.n].view(s.param.shape)
            if g.get("momentum", 0.0) > 0:
                st["momentum_buffer"] = self.v[s.offset:s.offset + s.n].view(s.param.shape)
            if g.get("centered"):
                st["grad_avg"] = self._max_exp_avg_sq()[s.offset:s.offset + s.n].view(s.param.shape)
        elif self.kind == N.FEDAVG_EPI_ASGD:
            st["step"] = torch.tensor(s.step, dtype=torch.float32)
            st["eta"] = torch.tensor(s.eta, dtype=torch.float32)
            st["mu"] = torch.tensor(s.mu, dtype=torch.float32)
            st["ax"] = self.m[s.offset:s.offset + s.n].view(s.param.shape)
        elif self.kind == N.FEDAVG_EPI_RPROP:
            st["step"] = torch.tensor(s.step, dtype=torch.float32)
            st["prev"] = self.m[s.offset:s.offset + s.n].view(s.param.shape)
            st["step_size"] = self.v[s.offset:s.offset + s.n].view(s.param.shape)
        elif self.kind == N.FEDAVG_EPI_ADAMAX:
            st["step"] = torch.tensor(s.step, dtype=torch.float32)
            st["exp_avg"] = self.m[s.offset:s.offset + s.n].view(s.param.shape)
            st["exp_inf"] = self.v[s.offset:s.offset + s.n].view(s.param.shape)
        else:
            st["step"] = torch.tensor(s.step, dtype=torch.float32)
            st["exp_avg"] = self.m[s.offset:s.offset + s.n].view(s.param.shape)
            st["exp_avg_sq"] = self.v[s.offset:s.offset + s.n].view(s.param.shape)
            if self.kind == N.FEDAVG_EPI_NADAM:
                st["mu_product"] = torch.tensor(s.mu_product, dtype=torch.float32)
            if group.get("amsgrad"):
                st["max_exp_avg_sq"] = self._max_exp_avg_sq()[s.offset:s.offset + s.n].view(s.param.shape)

    def _max_exp_avg_sq(self) -> torch.Tensor:
        if self.vmax is None:  # a group switched amsgrad on after binding: torch starts the max at zeros
            self.vmax = torch.zeros_like(self.v)
        return self.vmax

    def _epilogue(self, group: dict, s: _Slot) -> "N.Epilogue":
        e = N.Epilogue()
        e.kind = self.kind
        e.maximize = int(bool(group.get("maximize", False)))
        e.lr = float(group["lr"])
        e.weight_decay = float(group.get("weight_decay", 0.0))
        e.param = self.p.data_ptr()
        e.state1 = self.m.data_ptr()
        if self.kind == N.FEDAVG_EPI_SGD:
            e.momentum = float(group.get("momentum", 0.0))
            e.dampening = float(group.get("dampening", 0.0))
            e.nesterov = int(bool(group.get("nesterov", False)))
            e.first_step = int(not s.has_momentum_buffer)
        elif self.kind == N.FEDAVG_EPI_ADAGRAD:
            e.lr_decay = float(group.get("lr_decay", 0.0))
            e.eps = float(group["eps"])
            e.step = s.step + 1.0
        elif self.kind == N.FEDAVG_EPI_RMSPROP:
            e.alpha = float(group["alpha"])
            e.eps = float(group["eps"])
            e.momentum = float(group.get("momentum", 0.0))
            e.state2 = self.v.data_ptr()
            e.step = s.step + 1.0
            if group.get("centered"):
                e.centered = 1
                e.state3 = self._max_exp_avg_sq().data_ptr()
        elif self.kind == N.FEDAVG_EPI_ASGD:
            e.eta, e.mu, e.lambd = float(s.eta), float(s.mu), float(group["lambd"])
            e.step = s.step + 1.0
        elif self.kind == N.FEDAVG_EPI_RPROP:
            e.etaminus, e.etaplus = (float(x) for x in group["etas"])
            e.step_size_min, e.step_size_max = (float(x) for x in group["step_sizes"])
            e.state2 = self.v.data_ptr()
            e.step = s.step + 1.0
        elif self.kind == N.FEDAVG_EPI_ADAMAX:
            b1, b2 = group["betas"]
            e.beta1, e.beta2, e.eps = float(b1), float(b2), float(group["eps"])
            e.state2 = self.v.data_ptr()
            e.step = s.step + 1.0
        else:
            b1, b2 = group["betas"]
            e.beta1, e.beta2, e.eps = float(b1), float(b2), float(group["eps"])
            e.decoupled_weight_decay = int(bool(group.get("decoupled_weight_decay", False)))
            e.state2 = self.v.data_ptr()
            e.step = s.step + 1.0
            if self.kind == N.FEDAVG_EPI_NADAM:
                e.momentum_decay = float(group["momentum_decay"])
                e.mu_product = float(s.mu_product)
            if group.get("amsgrad"):
                e.amsgrad = 1
                e.state3 = self._max_exp_avg_sq().data_ptr()
        if self.kind in _SQRT_KINDS:
            # the reference's sqrt is torch CPU's on the server (vsSqrt, not correctly rounded; torch_sqrt.py)
            e.torch_sqrt = torch_sqrt.epilogue_flag(self.sqrt_mode)
        return e

    def step(self, model_diff: Dict) -> List[str]:
        """One server step on g = -diff for every parameter named in ``model_diff``; returns their names.

        Differences that are ``DeferredAggregate`` values of a round still staged on this device are
        aggregated and stepped in the same launch (``_fused_step``); the others are copied in and stepped
        with ``K = 0`` (the aggregated difference as ``acc_in``)."""
        groups = self._group_of()
        present = []
        self._check_diffs(model_diff)  # before any state is made or any launch, as torch fails at param.grad = ...
        self._init_lazy_state(model_diff, groups)
        fused = self._fused_step(model_diff, groups)
        host_pieces, keep = [], []  # host differences: one pass through the pinned ring, not a copy per tensor
        with torch.no_grad():
            for s in self.slots:
                if s.name not in model_diff or s.name in fused:
                    continue
                d = materialize_deferred(model_diff[s.name])
                t = d.detach() if isinstance(d, torch.Tensor) else torch.as_tensor(np.asarray(d))
                if t.dtype != torch.float32:  # param.grad = ... would refuse a different dtype
                    raise RuntimeError(f"assigned grad has data of a different type ({t.dtype}) for {s.name!r}")
                if tuple(t.shape) != tuple(s.param.shape):
                    raise RuntimeError(f"assigned grad has data of a different size for {s.name!r}")
                if self.g is None:
                    self.g = torch.zeros_like(self.p)
                if t.device.type == "cpu":
                    t = t.contiguous()
                    keep.append(t)
                    host_pieces.append((s.offset * 4, t.data_ptr(), s.n * 4))
                else:
                    self.g[s.offset:s.offset + s.n].copy_(t.reshape(-1), non_blocking=False)
                present.append(s)
        if not present:
            return [s.name for s in self.slots if s.name in fused]
        torch.cuda.synchronize(self.torch_device)
        if host_pieces:  # the compute stream waits for these copies (fedavg_h2d_tiled_multi)
            with self.ctx.lock:
                self.ctx.h2d_tiled_multi(self.g.data_ptr(), 4096 * 4, 4096 * 4, sorted(host_pieces))
        del keep
        # one launch per run of consecutive stepped parameters sharing group and per-parameter state
        runs: List[Tuple[tuple, List[_Slot]]] = []
        pos = {id(s): i for i, s in enumerate(self.slots)}
        for s in present:
            g = groups[id(s.param)]
            key = (id(g),) + s.host_key()
            prev = runs[-1][1][-1] if runs else None
            contiguous = prev is not None and pos[id(s)] == pos[id(prev)] + 1
            if runs and runs[-1][0] == key and contiguous:
                runs[-1][1].append(s)
            else:
                runs.append((key, [s]))
        # torch's copies above are complete (synchronised); the kernels run on the context's own stream
        with self.ctx.lock:
            for key, run in runs:
                e = self._epilogue(groups[id(run[0].param)], run[0])
                begin = run[0].offset
                end = (run[-1].offset + run[-1].n + 3) // 4 * 4
                self.ctx.accumulate_tiled_epi([], [], 4096, 4096, begin, end, None, N.FEDAVG_OP_TORCH,
                                              N.FEDAVG_FIN_NONE, 1.0, e, acc_in_ptr=self.g.data_ptr())
            self.ctx.sync()
        self._advance(present, groups)
        return [s.name for s in self.slots if s.name in fused or s in present]

    def _check_diffs(self, model_diff: Dict) -> None:
        """The reference assigns every difference to ``param.grad`` before ``optimizer.step()``
        (fedopt.py:157-182); torch refuses a grad of another dtype or size there, so a bad difference fails
        the round before any optimizer state is made.  Checked on shape / dtype attributes (a deferred
        aggregate is not materialised for it)."""
        for s in self.slots:
            if s.name not in model_diff:
                continue
            d = model_diff[s.name]
            if not hasattr(d, "shape") or not hasattr(d, "dtype"):
                d = np.asarray(d)
            dt = d.dtype
            if dt not in (torch.float32, np.dtype(np.float32)):
                raise RuntimeError(f"assigned grad has data of a different type ({dt}) for {s.name!r}")
            if tuple(d.shape) != tuple(s.param.shape):
                raise RuntimeError(f"assigned grad has data of a different size for {s.name!r}")

    def _init_lazy_state(self, model_diff: Dict, groups: Dict[int, dict]) -> None:
        """Rprop and ASGD make their state at the first step (rprop.py / asgd.py ``_init_group``): Rprop prev = 0,
        step_size = full_like(grad, lr); ASGD ax = 0, eta = lr (fp32), mu = 1.  Runs after ``_check_diffs``."""
        if self.kind not in (N.FEDAVG_EPI_RPROP, N.FEDAVG_EPI_ASGD):
            return
        with torch.no_grad():
            for s in self.slots:
                if s.name in model_diff and not s.state_initialised:
                    lr = float(groups[id(s.param)]["lr"])
                    self.m[s.offset:s.offset + s.n].zero_()
                    if self.kind == N.FEDAVG_EPI_RPROP:
                        self.v[s.offset:s.offset + s.n].fill_(lr)
                    else:
                        s.eta, s.mu = np.float32(lr), np.float32(1.0)
                    s.state_initialised = True

    def _advance(self, stepped: List[_Slot], groups: Dict[int, dict]) -> None:
        for s in stepped:
            s.step += 1.0
            if self.kind == N.FEDAVG_EPI_ASGD:  # asgd.py: new eta / mu from the python-float formulas
                g = groups[id(s.param)]
                s.eta = np.float32(g["lr"] / ((1 + g["lambd"] * g["lr"] * s.step) ** g["alpha"]))
                s.mu = np.float32(1 / max(1, s.step - g["t0"]))
            if self.kind == N.FEDAVG_EPI_NADAM:  # nadam.py: mu_product *= mu on an fp32 tensor
                g = groups[id(s.param)]
                mu = g["betas"][0] * (1.0 - 0.5 * (0.96 ** (s.step * g["momentum_decay"])))
                s.mu_product = np.float32(np.float32(s.mu_product) * np.float32(mu))
            if self.kind == N.FEDAVG_EPI_SGD and groups[id(s.param)].get("momentum", 0.0) != 0.0:
                s.has_momentum_buffer = True
            self._expose_state(s, groups[id(s.param)])

    def _fused_step(self, model_diff: Dict, groups: Dict[int, dict]) -> set:
        """Aggregation + optimizer step in one launch for the parameters whose difference is a deferred
        aggregate on this device (same shape; fp32 by construction).  Returns the names stepped."""
        cand = {}
        for s in self.slots:
            d = model_diff.get(s.name)
            if isinstance(d, DeferredAggregate) and d.fusable(self.hip_device) and tuple(d.shape) == tuple(s.param.shape):
                cand.setdefault(id(d.round), (d.round, {}))[1][d.name] = s
        done = set()
        if not cand:
            return done
        torch.cuda.synchronize(self.torch_device)  # p, m, v written by torch (binding, checkpoint loads)
        # pipelined egress of the new weights: only when this one round steps every parameter, in a launch order
        # whose parameter offsets increase (then "bytes [0, X) of p are final" is a true statement per mark)
        egress = False
        if len(cand) == 1 and self.pipelined_egress:
            rnd, by_key = next(iter(cand.values()))
            if len(by_key) == len(self.slots):
                order = sorted(by_key.items(), key=lambda kv: rnd.keys[kv[0]].offset)
                offs = [s.offset for _, s in order]
                egress = all(a < b for a, b in zip(offs, offs[1:]))
        for rnd, by_key in cand.values():
            entries = {}
            for key, s in by_key.items():
                g = groups[id(s.param)]
                entries[key] = FusedEntry(s.offset, self._epilogue(g, s), (id(g),) + s.host_key())
            names = set(rnd.fused_step(entries, egress_marks=egress))
            stepped = [s for key, s in by_key.items() if key in names]
            with self.ctx.lock:
                if egress and len(stepped) == len(self.slots):
                    self.ctx.mark(self.p.numel() * 4)
                    self.egress_pending = True  # _to_host reads p with fedavg_d2h_marked
                else:
                    if egress:
                        self.ctx.marks_reset()
                    self.ctx.sync()
            self._advance(stepped, groups)
            done.update(s.name for s in stepped)
        return done


class PTFedOptModelShareableGenerator(FullModelShareableGenerator):
    def __init__(self, optimizer_args: dict = None, lr_scheduler_args: dict = None, source_model="model", device=None,
                 devices: Optional[list] = None):
        """Same arguments as the reference (fedopt.py:30-81); ``device`` picks the HIP device.  ``devices``
        (two or more HIP devices, the aggregator's ``devices`` in the same order): the optimizer state is
        split by parameter bucket over them and each bucket is stepped on its device, in the launch that
        aggregates it when the aggregator defers its result (``sharded_fedopt.ShardedServerOptimizer``)."""
        super().__init__(device=hip_device_index(device) if device not in (None, "cpu") else None)
        self.devices = [int(d) for d in devices] if devices and len(devices) > 1 else None
        if not optimizer_args:
            self.logger.warning("No optimizer_args provided. Using FedOpt with SGD and lr 1.0")
            optimizer_args = {"path": "torch.optim.SGD", "args": {"lr": 1.0}}
        if not isinstance(optimizer_args, dict):
            raise TypeError(
                "optimizer_args must be a dict of format, e.g. {'path': 'torch.optim.SGD', 'args': {'lr': 1.0}}."
            )
        if lr_scheduler_args is not None and not isinstance(lr_scheduler_args, dict):
            raise TypeError(
                "lr_scheduler_args must be a dict of format, e.g. "
                "{'path': 'torch.optim.lr_scheduler.CosineAnnealingLR', 'args': {'T_max': 100}}."
            )
        self.source_model = source_model
        self.optimizer_args = optimizer_args
        self.lr_scheduler_args = lr_scheduler_args
        self.model = None
        self.optimizer = None
        self.lr_scheduler = None
        self.device = device
        self.optimizer_name = None
        self.lr_scheduler_name = None
        self._dev_opt: Optional[DeviceServerOptimizer] = None

    @staticmethod
    def _get_component_name(component_args):
        if component_args is None:
            return None
        return component_args.get("path") or component_args.get("class_path") or component_args.get("name", None)

    def handle_event(self, event_type: str, fl_ctx: FLContext):
        if event_type != EventType.START_RUN:
            return
        engine = fl_ctx.get_engine()
        self.device = torch.device("cuda", hip_device_index(self.device))
        if isinstance(self.source_model, str):
            self.model = engine.get_component(self.source_model) if engine is not None else None
        else:
            self.model = self.source_model
        if self.model is None:
            self.system_panic("Model is not available", fl_ctx)
            return
        if not isinstance(self.model, torch.nn.Module):
            self.system_panic(f"Expected model to be a torch.nn.Module but got {type(self.model)}", fl_ctx)
            return
        if self.devices is None:  # sharded: the model stays on the host (its parameters view the host weights)
            self.model.to(self.device)
        build = getattr(engine, "build_component", None) or build_component_from_args
        try:
            self.optimizer_args.setdefault("args", {})
            self.optimizer_args["args"]["params"] = self.model.parameters()
            self.optimizer = build(self.optimizer_args)
            self.optimizer_name = self._get_component_name(self.optimizer_args)
        except Exception as e:
            self.system_panic(f"Exception while parsing `optimizer_args`({self.optimizer_args}): {e}", fl_ctx)
            return
        if self.lr_scheduler_args is not None:
            try:
                self.lr_scheduler_name = self._get_component_name(self.lr_scheduler_args)
                self.lr_scheduler_args.setdefault("args", {})
                self.lr_scheduler_args["args"]["optimizer"] = self.optimizer
                self.lr_scheduler = build(self.lr_scheduler_args)
            except Exception as e:
                self.system_panic(f"Exception while parsing `lr_scheduler_args`({self.lr_scheduler_args}): {e}", fl_ctx)
                return

    def device_optimizer(self):
        """The HBM image of (model, optimizer) -- one device, or sharded over ``devices``; (re)bound when
        either changed since the last step."""
        d = self._dev_opt
        if d is None or d.model is not self.model or d.optimizer is not self.optimizer or not d.is_bound():
            if self.devices is not None:
                from .sharded_fedopt import ShardedServerOptimizer

                if isinstance(d, ShardedServerOptimizer):
                    if d.optimizer is self.optimizer:
                        d.export_state()  # the new image starts from the shards' moments, not stale state
                    d.release()
                self._dev_opt = ShardedServerOptimizer(self.model, self.optimizer, self.devices)
            else:
                self._dev_opt = DeviceServerOptimizer(self.model, self.optimizer, hip_device_index(self.device))
        return self._dev_opt

    def server_update(self, model_diff):
        """fedopt.py:157-182: the optimizer step on g = -diff, then the lr scheduler; returns
        (state_dict, names of the stepped parameters)."""
        self.model.train()
        dev = self.device_optimizer()
        updated_params = dev.step(model_diff)
        if self.lr_scheduler is not None:
            with warnings.catch_warnings():  # the step ran on the device, not through optimizer.step()
                warnings.simplefilter("ignore", UserWarning)
                self.lr_scheduler.step()
        return self.model.state_dict(), updated_params

    def shareable_to_learnable(self, shareable: Shareable, fl_ctx: FLContext) -> Learnable:
        dxo = from_shareable(shareable)
        if dxo.data_kind != DataKind.WEIGHT_DIFF:
            self.system_panic("FedOpt is only implemented for data_kind == DataKind.WEIGHT_DIFF", fl_ctx)
            return Learnable()
        processed_algorithm = dxo.get_meta_prop(MetaKey.PROCESSED_ALGORITHM)
        if processed_algorithm is not None:
            self.system_panic(f"FedOpt is not implemented for shareable processed by {processed_algorithm}", fl_ctx)
            return Learnable()
        model_diff = dxo.data
        base_model = fl_ctx.get_prop(AppConstants.GLOBAL_MODEL)
        if not base_model:
            self.system_panic(reason="No global base model!", fl_ctx=fl_ctx)
            return base_model
        base_model_weights = base_model[ModelLearnableKey.WEIGHTS]
        if base_model_weights:
            preserve_torch = any(isinstance(v, torch.Tensor) for v in base_model_weights.values())
        else:
            preserve_torch = any(isinstance(v, torch.Tensor) or (isinstance(v, DeferredValue) and v.container == "torch")
                                 for v in model_diff.values())

        start = time.time()
        weights, updated_params = self.server_update(model_diff)
        secs = time.time() - start

        start = time.time()
        if isinstance(self._dev_opt, DeviceServerOptimizer):
            weights = self._to_host(weights, preserve_torch, self._dev_opt)
        else:  # sharded: the parameters already are host views of the new weights
            weights = self._dev_opt.to_host(weights, preserve_torch)
        secs_detach = time.time() - start

        # FedAvg for the keys the optimizer does not own (e.g. batch-norm statistics), fedopt.py:247-263
        rest = [k for k in model_diff if k not in updated_params]
        base = {}
        for key in rest:
            base_value = base_model_weights[key] if key in base_model_weights else weights[key]
            value = model_diff[key]
            if isinstance(value, DeferredAggregate) and (value.container == "torch") == preserve_torch \
                    and isinstance(base_value, torch.Tensor) == preserve_torch \
                    and not (isinstance(base_value, torch.Tensor) and base_value.device.type != "cpu"):
                base[key] = (base_value, value)  # aggregated and added in one launch (apply_weight_diff)
                continue
            value = materialize_deferred(value)
            if preserve_torch:
                base_value = base_value.detach().cpu() if isinstance(base_value, torch.Tensor) else torch.as_tensor(base_value)
                value = value.detach().cpu() if isinstance(value, torch.Tensor) else torch.as_tensor(value)
            base[key] = (base_value, value)
        merged = apply_weight_diff(self._adder, {k: b for k, (b, _) in base.items()}, {k: d for k, (_, d) in base.items()})
        weights.update(merged)

        self.log_info(
            fl_ctx,
            f"FedOpt ({self.optimizer_name}, {self.devices or self.device}) server model update "
            f"round {fl_ctx.get_prop(AppConstants.CURRENT_ROUND)}, "
            f"{self.lr_scheduler_name if self.lr_scheduler_name else ''} "
            f"lr: {self.optimizer.param_groups[-1]['lr']}, "
            f"fedopt layers: {len(updated_params)}, fedavg layers: {len(rest)}, "
            f"update: {secs} secs., detach: {secs_detach} secs.",
        )
        return make_model_learnable(weights, dxo.get_meta_props())

    @staticmethod
    def _to_host(state: Dict, preserve_torch: bool, dev: Optional[DeviceServerOptimizer] = None) -> Dict:
        """state_dict -> host copies (``.detach().cpu().clone()`` / ``.numpy()``, fedopt.py:238-244).

        The parameters live in one flat HBM buffer: it comes back in ONE D2H through the handle's pinned
        ring (a pageable ``.cpu()`` per tensor is several times slower); each parameter is a view of that
        fresh host copy, as the aggregation engine's numpy results are views of its host arena."""
        out = {}
        host_p = None
        if dev is not None and dev.slots:
            torch.cuda.synchronize(dev.torch_device)
            host_p = dev.host_pool.take(dev.p.numel(), pin=dev.ctx)
            with dev.ctx.lock:  # the handle is shared with the aggregation engine (accepts on other threads)
                if dev.egress_pending:  # chunks of p leave while the fused launches still run
                    dev.egress_pending = False
                    dev.ctx.d2h_marked(host_p, dev.p.data_ptr())
                    dev.ctx.sync()
                else:
                    dev.ctx.d2h(host_p, dev.p.data_ptr())
        base = dev.p.data_ptr() if host_p is not None else 0
        for k, v in state.items():
            s = dev.by_name.get(k) if host_p is not None else None
            if s is not None and v.dtype == torch.float32 and v.is_contiguous() and v.data_ptr() == base + 4 * s.offset:
                h = host_p[s.offset:s.offset + s.n].reshape(tuple(v.shape))
                out[k] = torch.from_numpy(h) if preserve_torch else h
                continue
            h = v.detach().cpu()
            out[k] = h.clone() if preserve_torch else h.numpy()
        return out
