"""Generate the golden vectors in tests/golden/ by running the NVFlare reference itself.

Runs ONLY in the build container, where the reference tree is mounted read-only at /root/reference.
Nothing here runs on the GPU box; the outputs (``helper_cases.npz`` + ``helper_cases.json``) are plain
data: inputs, weights and the reference's outputs.

``import nvflare`` fails in the container with an ordinary ModuleNotFoundError (``cryptography``,
pulled in by ``nvflare/__init__.py:21-23``); this is not a permission denial.  The script registers
``nvflare``, ``nvflare.app_opt`` and ``nvflare.app_opt.pt`` as bare namespace packages whose
``__path__`` points into the reference tree, then imports the aggregation modules normally
(SURVEY.md section 8c).  No reference source is copied.

Reference code exercised:
  nvflare/app_common/aggregators/weighted_aggregation_helper.py:153-240  (helper cases)
  nvflare/app_common/workflows/base_fedavg.py:93-230  (``--set fedavg``: aggregate_fn cases)
  nvflare/app_common/workflows/fedavg.py:268-366      (``--set fedavg``: built-in in-time FedAvg cases)
  nvflare/app_common/workflows/scaffold.py:149-189    (``--set scaffold``: scaffold_aggregate_fn cases)
  nvflare/app_opt/pt/fedopt.py:157-270                 (``--set fedopt``: PTFedOptModelShareableGenerator, CPU)
  nvflare/app_common/shareablegenerators/full_model_shareable_generator.py:37-83  (``--set fedopt``)
  nvflare/app_opt/pt/quantization/ada_quant.py:39-87  (``--set quant``: AdaQuantizer quantize / dequantized)
  nvflare/app_common/aggregators/intime_accumulate_model_aggregator.py   (intime cases)
  nvflare/app_common/aggregators/dxo_aggregator.py:71-191

Usage:  python tests/golden/make_golden.py [--ref /root/reference] [--set helper|fedavg|scaffold|fedopt|quant|dtypes]
        (helper -> helper_cases.{npz,json}; fedavg -> fedavg_cases.{npz,json}; scaffold -> scaffold_cases.{npz,json};
         fedopt -> fedopt_cases.{npz,json}; quant -> quant_cases.{npz,json};
         dtypes -> dtype_cases.{npz,json}: float16 / bfloat16 / integer / bool client arrays)
"""

from __future__ import annotations

import argparse
import json
import os
import random
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True  # the reference tree is read-only input: never leave __pycache__ in it

HERE = os.path.dirname(os.path.abspath(__file__))


def install_shim(ref_root: str) -> None:
    for name, sub in (("nvflare", "nvflare"), ("nvflare.app_opt", "nvflare/app_opt"), ("nvflare.app_opt.pt", "nvflare/app_opt/pt")):
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.__path__ = [os.path.join(ref_root, sub)]
            sys.modules[name] = m
    if ref_root not in sys.path:
        sys.path.insert(0, ref_root)


class Store:
    def __init__(self):
        self.arrays = {}
        self.n = 0

    def put(self, arr, tag="a") -> str:
        if isinstance(arr, torch.Tensor):
            arr = arr.detach().cpu().numpy()
        arr = np.array(arr, copy=True)  # snapshot: a reference result may alias live state (fedopt on CPU)
        name = f"{tag}{self.n:05d}"
        self.n += 1
        self.arrays[name] = arr
        return name


def to_container(arr: np.ndarray, container: str):
    if container == "torch":
        return torch.from_numpy(np.array(arr, copy=True))
    return np.array(arr, copy=True)


def special_values(rng, n, dtype=np.float32):
    base = rng.standard_normal(n).astype(dtype)
    specials = np.array(
        [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -3e-42, 1.4e-45, 3.0e38, -3.0e38, 1e-38, 65504.0, 1.0, -1.0],
        dtype=dtype,
    )
    idx = rng.choice(n, size=min(n, 3 * specials.size), replace=False)
    base[idx] = np.resize(specials, idx.size)
    return base


def run_helper_case(store, cases, name, container, contributions, exclude_vars=None, weigh_by_local_iter=True):
    """contributions: list of (contributor_name, weight, {key: np.ndarray})"""
    from nvflare.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    helper = WeightedAggregationHelper(exclude_vars=exclude_vars, weigh_by_local_iter=weigh_by_local_iter)
    rec = []
    for cname, w, data in contributions:
        dmap = {k: store.put(v, "in") for k, v in data.items()}
        rec.append({"name": cname, "weight": w, "data": dmap})
        helper.add({k: to_container(v, container) for k, v in data.items()}, w, cname, 0)
    result = helper.get_result()
    stats = helper.last_aggregation_stats
    exp = {}
    exp_dtype = {}
    for k, v in result.items():
        if isinstance(v, torch.Tensor):
            exp_dtype[k] = str(v.dtype).replace("torch.", "")
        else:
            exp_dtype[k] = str(np.asarray(v).dtype)
        exp[k] = store.put(v, "out")
    cases.append(
        {
            "kind": "helper",
            "name": name,
            "container": container,
            "exclude_vars": exclude_vars,
            "weigh_by_local_iter": weigh_by_local_iter,
            "contributions": rec,
            "expected": exp,
            "expected_dtype": exp_dtype,
            "stats": stats,
        }
    )


def run_intime_case(store, cases, name, container, clients, expected_data_kind, aggregation_weights=None, exclude_vars=None):
    """clients: list of (contributor_name, {dxo_key or '': (n_iter, {key: array})})"""
    from nvflare.apis.dxo import DXO, DataKind, MetaKey, from_shareable
    from nvflare.apis.fl_constant import ReservedKey
    from nvflare.apis.fl_context import FLContext
    from nvflare.apis.shareable import Shareable
    from nvflare.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator
    from nvflare.app_common.app_constant import AppConstants

    agg = InTimeAccumulateWeightedAggregator(
        exclude_vars=exclude_vars, aggregation_weights=aggregation_weights, expected_data_kind=expected_data_kind
    )
    agg._initialize(agg.aggregation_weights, agg.exclude_vars, agg.expected_data_kind)
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0)
    rec = []
    for cname, dxos in clients:
        entry = {"name": cname, "dxos": {}}
        if "" in dxos:
            n_iter, data = dxos[""]
            kind = expected_data_kind
            dxo = DXO(kind, data={k: to_container(v, container) for k, v in data.items()}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: n_iter})
            entry["dxos"][""] = {"n_iter": n_iter, "kind": kind, "data": {k: store.put(v, "in") for k, v in data.items()}}
        else:
            sub = {}
            for dk, (n_iter, data) in dxos.items():
                kind = expected_data_kind[dk]
                sub[dk] = DXO(kind, data={k: to_container(v, container) for k, v in data.items()}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: n_iter})
                entry["dxos"][dk] = {"n_iter": n_iter, "kind": kind, "data": {k: store.put(v, "in") for k, v in data.items()}}
            dxo = DXO(DataKind.COLLECTION, data=sub)
        s = Shareable()
        s.set_peer_props({ReservedKey.IDENTITY_NAME: cname})
        s.add_cookie(AppConstants.CONTRIBUTION_ROUND, 0)
        entry["accepted"] = bool(agg.accept(dxo.update_shareable(s), fl_ctx))
        rec.append(entry)
    result = from_shareable(agg.aggregate(fl_ctx))
    stats = fl_ctx.get_prop(AppConstants.AGGREGATION_STATS)
    expected = {}
    if result.data_kind == DataKind.COLLECTION:
        for dk, sub in result.data.items():
            expected[dk] = {"kind": sub.data_kind, "data": {k: store.put(v, "out") for k, v in sub.data.items()}}
    else:
        expected[""] = {"kind": result.data_kind, "data": {k: store.put(v, "out") for k, v in result.data.items()}}
    cases.append(
        {
            "kind": "intime",
            "name": name,
            "container": container,
            "expected_data_kind": expected_data_kind,
            "aggregation_weights": aggregation_weights,
            "exclude_vars": exclude_vars,
            "clients": rec,
            "expected": expected,
            "stats": stats,
        }
    )


def _jsonable_steps(v):
    """NUM_STEPS values are recorded with a type tag so the JSON round trip keeps them exact."""
    if v is None:
        return {"t": "none"}
    if isinstance(v, bool):
        return {"t": "bool", "v": v}
    if isinstance(v, int):
        return {"t": "int", "v": v}
    if isinstance(v, float):
        return {"t": "float", "v": repr(v)}
    return {"t": "str", "v": str(v)}


def _fl_models(store, container, clients):
    """clients: [(name, num_steps, {key: arr}, metrics)] -> (FLModels, json record)"""
    from nvflare.apis.fl_constant import FLMetaKey
    from nvflare.app_common.abstract.fl_model import FLModel

    models, rec = [], []
    for name, steps, data, metrics in clients:
        meta = {"client_name": name}
        if steps is not None:
            meta[FLMetaKey.NUM_STEPS_CURRENT_ROUND] = steps
        models.append(FLModel(params={k: to_container(v, container) for k, v in data.items()}, metrics=metrics,
                              current_round=3, meta=meta))
        rec.append({"name": name, "num_steps": _jsonable_steps(steps), "data": {k: store.put(v, "in") for k, v in data.items()},
                    "metrics": metrics})
    return models, rec


def _result_record(store, model):
    return {
        "params": {k: store.put(v, "out") for k, v in model.params.items()},
        "params_dtype": {k: (str(v.dtype).replace("torch.", "") if isinstance(v, torch.Tensor) else str(np.asarray(v).dtype))
                         for k, v in model.params.items()},
        "params_type": str(model.params_type.value if model.params_type is not None else None),
        "metrics": model.metrics,
        "meta": {k: v for k, v in model.meta.items()},
        "current_round": model.current_round,
    }


def run_fedavg_fn_case(store, cases, name, container, clients):
    from nvflare.app_common.workflows.base_fedavg import BaseFedAvg

    models, rec = _fl_models(store, container, clients)
    out = BaseFedAvg.aggregate_fn(models)
    cases.append({"kind": "aggregate_fn", "name": name, "container": container, "clients": rec, "expected": _result_record(store, out)})


def run_fedavg_intime_case(store, cases, name, container, clients, aggregation_weights):
    """FedAvg's built-in in-time path: _aggregate_one_result per client, then _get_aggregated_result."""
    from nvflare.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper
    from nvflare.app_common.workflows.fedavg import FedAvg

    wf = FedAvg(num_clients=len(clients), num_rounds=1, aggregation_weights=aggregation_weights)
    wf.info = wf.warning = lambda *a, **k: None
    wf.fl_ctx = None
    wf.current_round = 3
    wf._aggr_helper = WeightedAggregationHelper()
    wf._aggr_metrics_helper = WeightedAggregationHelper()
    wf._expected_count = len(clients)
    models, rec = _fl_models(store, container, clients)
    accepted = [bool(wf._aggregate_one_result(m)) for m in models]
    out = wf._get_aggregated_result()
    cases.append({"kind": "fedavg_intime", "name": name, "container": container, "aggregation_weights": aggregation_weights,
                  "clients": rec, "accepted": accepted, "expected": _result_record(store, out)})


def main_fedavg():
    rng = np.random.default_rng(20261016)
    store = Store()
    cases = []
    odd_steps = [3, None, True, -2, float("nan"), "7", 2.5, "abc", 0, float("inf"), 1e300, False]
    for container in ("numpy", "torch"):
        # torch's add_(alpha=1e300) raises for an fp32 total (tests/test_gpu_fedavg_path.py checks that we
        # raise too); the torch cases use the largest finite-in-fp32 weight instead
        steps = odd_steps if container == "numpy" else [3e38 if s == 1e300 else s for s in odd_steps]
        K = len(steps)
        clients = [(f"site-{i+1}", steps[i], {"w": rng.standard_normal(1031).astype(np.float32),
                                                  "b": rng.standard_normal(7).astype(np.float32)},
                    {"acc": float(rng.random()), "flag": bool(i % 2), "info": {"x": 1}, "tag": "s"}) for i in range(K)]
        run_fedavg_fn_case(store, cases, f"{container}_fn_weight_rule", container, clients)
        # a client without metrics disables metric aggregation; one unnamed client
        clients2 = [(f"site-{i+1}" if i else "", int(rng.integers(1, 60)), {"layer.weight": rng.standard_normal((17, 5)).astype(np.float32)},
                     None if i == 2 else {"loss": float(rng.random())}) for i in range(5)]
        run_fedavg_fn_case(store, cases, f"{container}_fn_no_metrics", container, clients2)
        aw = {f"site-{i+1}": float(rng.random()) * 3 for i in range(0, K, 2)}
        run_fedavg_intime_case(store, cases, f"{container}_intime_weights", container, clients, aw)
        run_fedavg_intime_case(store, cases, f"{container}_intime_plain", container, clients2, None)
    np.savez_compressed(os.path.join(HERE, "fedavg_cases.npz"), **store.arrays)
    with open(os.path.join(HERE, "fedavg_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --set fedavg", "reference": "NVFlare (/root/reference, ~2.9.0-dev)",
                   "numpy": np.__version__, "torch": torch.__version__, "cases": cases}, f, indent=1, default=str)
    print(f"wrote {len(cases)} fedavg cases, {len(store.arrays)} arrays")


def run_scaffold_case(store, cases, name, clients):
    """clients: [(name, num_steps, params, ctrl_diff, metrics, params_container, ctrl_container)]; ctrl None:
    the client omits SCAFFOLD_CTRL_DIFF (the reference raises)."""
    from nvflare.apis.fl_constant import FLMetaKey
    from nvflare.app_common.abstract.fl_model import FLModel
    from nvflare.app_common.app_constant import AlgorithmConstants
    from nvflare.app_common.workflows.scaffold import scaffold_aggregate_fn

    models, rec = [], []
    for cname, steps, params, ctrl, metrics, pc, cc in clients:
        meta = {"client_name": cname}
        if steps is not None:
            meta[FLMetaKey.NUM_STEPS_CURRENT_ROUND] = steps
        if ctrl is not None:
            meta[AlgorithmConstants.SCAFFOLD_CTRL_DIFF] = {k: to_container(v, cc) for k, v in ctrl.items()}
        models.append(FLModel(params={k: to_container(v, pc) for k, v in params.items()}, metrics=metrics,
                              current_round=3, meta=meta))
        rec.append({"name": cname, "num_steps": _jsonable_steps(steps), "metrics": metrics,
                    "params_container": pc, "ctrl_container": cc,
                    "params": {k: store.put(v, "in") for k, v in params.items()},
                    "ctrl": None if ctrl is None else {k: store.put(v, "in") for k, v in ctrl.items()}})
    try:
        out = scaffold_aggregate_fn(models)
    except ValueError as e:
        cases.append({"kind": "scaffold", "name": name, "clients": rec, "error": str(e)})
        return
    ctrl_out = out.meta[AlgorithmConstants.SCAFFOLD_CTRL_DIFF]

    def dt(v):
        return str(v.dtype).replace("torch.", "") if isinstance(v, torch.Tensor) else str(np.asarray(v).dtype)

    expected = _result_record(store, out)
    expected["meta"] = {k: v for k, v in out.meta.items() if k != AlgorithmConstants.SCAFFOLD_CTRL_DIFF}
    expected["params_order"] = list(out.params)
    expected["params_kind"] = {k: "torch" if isinstance(v, torch.Tensor) else "numpy" for k, v in out.params.items()}
    expected["ctrl"] = {k: store.put(v, "out") for k, v in ctrl_out.items()}
    expected["ctrl_order"] = list(ctrl_out)
    expected["ctrl_dtype"] = {k: dt(v) for k, v in ctrl_out.items()}
    expected["ctrl_kind"] = {k: "torch" if isinstance(v, torch.Tensor) else "numpy" for k, v in ctrl_out.items()}
    cases.append({"kind": "scaffold", "name": name, "clients": rec, "expected": expected})


def main_scaffold():
    rng = np.random.default_rng(20261017)
    store = Store()
    cases = []
    shapes = {"conv.weight": (8, 3, 3, 3), "conv.bias": (8,), "fc.weight": (10, 72), "fc.bias": (10,)}

    def arr(shape, dtype=np.float32):
        return rng.standard_normal(shape).astype(dtype)

    def metrics(i):
        return {"loss": float(rng.random()), "acc": float(rng.random()), "tag": "s", "flag": bool(i % 2)}

    steps = [12, None, 3.5, "9", -1, True, 40]
    for pc, cc in (("numpy", "numpy"), ("torch", "torch"), ("torch", "numpy")):
        tag = pc if pc == cc else f"{pc}_{cc}"
        # every client sends every key; the FedAvg weight rule on odd NUM_STEPS values
        clients = [(f"site-{i+1}", steps[i], {k: arr(v) for k, v in shapes.items()},
                    {k: arr(v) * 1e-2 for k, v in shapes.items()}, metrics(i), pc, cc) for i in range(len(steps))]
        run_scaffold_case(store, cases, f"{tag}_full", clients)
        # ragged keys: params and controls each miss keys on some clients; a control for a key no client
        # sends as a param (a buffer); arrival order of new keys differs between params and controls
        ragged = []
        for i in range(5):
            pk = [k for j, k in enumerate(shapes) if (i + j) % 4 != 3]
            ck = [k for j, k in enumerate(reversed(list(shapes))) if (i * 3 + j) % 5 != 1]
            ctrl = {k: arr(shapes[k]) for k in ck}
            if i >= 2:
                ctrl["bn.running_mean"] = arr(8)
            ragged.append((f"site-{i+1}" if i != 3 else "", int(rng.integers(1, 50)), {k: arr(shapes[k]) for k in pk},
                           ctrl, None if i == 4 else metrics(i), pc, cc))
        run_scaffold_case(store, cases, f"{tag}_ragged", ragged)
    # more clients, larger ragged tiles, special values in the controls, an fp64 control key
    K, P = 20, 4099
    clients = [(f"site-{i+1}", float(rng.integers(1, 100)), {"w": arr(P), "b": arr(33)},
                {"w": special_values(rng, P) * np.float32(1e-3), "b": arr(33), "scale": rng.random(5)},
                metrics(i), "numpy", "numpy") for i in range(K)]
    run_scaffold_case(store, cases, "numpy_k20_special", clients)
    # a client without SCAFFOLD_CTRL_DIFF: the reference's ValueError
    bad = [(f"site-{i+1}", 2, {"w": arr(5)}, None if i == 1 else {"w": arr(5)}, None, "numpy", "numpy") for i in range(3)]
    run_scaffold_case(store, cases, "missing_ctrl", bad)
    np.savez_compressed(os.path.join(HERE, "scaffold_cases.npz"), **store.arrays)
    with open(os.path.join(HERE, "scaffold_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --set scaffold", "reference": "NVFlare (/root/reference, ~2.9.0-dev)",
                   "numpy": np.__version__, "torch": torch.__version__, "cases": cases}, f, indent=1, default=str)
    print(f"wrote {len(cases)} scaffold cases, {len(store.arrays)} arrays")


FEDOPT_CONFIGS = [
    # (name, optimizer_args, lr_scheduler_args)
    ("sgd_default", {"path": "torch.optim.SGD", "args": {"lr": 1.0}}, None),
    ("sgd_momentum_wd", {"path": "torch.optim.SGD", "args": {"lr": 0.5, "momentum": 0.9, "dampening": 0.1, "weight_decay": 1e-3}}, None),
    ("sgd_nesterov", {"path": "torch.optim.SGD", "args": {"lr": 0.3, "momentum": 0.9, "nesterov": True}}, None),
    ("sgd_steplr", {"path": "torch.optim.SGD", "args": {"lr": 1.0, "momentum": 0.6}},
     {"path": "torch.optim.lr_scheduler.StepLR", "args": {"step_size": 1, "gamma": 0.5}}),
    ("adam_default", {"path": "torch.optim.Adam", "args": {"lr": 1e-3}}, None),
    ("adam_wd", {"path": "torch.optim.Adam", "args": {"lr": 1e-2, "betas": [0.8, 0.99], "eps": 1e-6, "weight_decay": 1e-2}}, None),
    ("adamw", {"path": "torch.optim.AdamW", "args": {"lr": 1e-2, "weight_decay": 0.1}}, None),
    ("adam_cosine", {"path": "torch.optim.Adam", "args": {"lr": 1e-2, "maximize": False}},
     {"path": "torch.optim.lr_scheduler.CosineAnnealingLR", "args": {"T_max": 5}}),
]


def fedopt_model():
    """Small model with fp32 params, BatchNorm buffers (incl. int64 num_batches_tracked) and a plain
    buffer; the test side rebuilds the same architecture (tests/test_gpu_fedopt_generator.py)."""
    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin1 = torch.nn.Linear(7, 64)
            self.bn = torch.nn.BatchNorm1d(64)
            self.lin2 = torch.nn.Linear(64, 90, bias=False)
            self.register_buffer("offset", torch.zeros(5))

    return Net()


def _import_path(path):
    import importlib

    mod, _, cls = path.rpartition(".")
    return getattr(importlib.import_module(mod), cls)


def main_fedopt():
    from nvflare.apis.dxo import DXO, DataKind
    from nvflare.apis.fl_context import FLContext
    from nvflare.app_common.abstract.model import ModelLearnableKey, make_model_learnable
    from nvflare.app_common.app_constant import AppConstants
    from nvflare.app_opt.pt.fedopt import PTFedOptModelShareableGenerator

    rng = np.random.default_rng(20261017)
    torch.manual_seed(0)
    store = Store()
    cases = []
    init_model = fedopt_model()
    init_state = {k: v.detach().clone() for k, v in init_model.state_dict().items()}
    init_names = {k: store.put(v, "init") for k, v in init_state.items()}
    n_rounds = 3
    for container in ("numpy", "torch"):
        configs = FEDOPT_CONFIGS if container == "numpy" else [FEDOPT_CONFIGS[1], FEDOPT_CONFIGS[4]]
        for name, opt_args, sched_args in configs:
            model = fedopt_model()
            model.load_state_dict(init_state)
            gen = PTFedOptModelShareableGenerator(optimizer_args=json.loads(json.dumps(opt_args)), device="cpu")
            gen.model = model
            gen.device = torch.device("cpu")
            args = dict(opt_args["args"])
            if "betas" in args:
                args["betas"] = tuple(args["betas"])
            gen.optimizer = _import_path(opt_args["path"])(model.parameters(), **args)
            gen.optimizer_name = opt_args["path"]
            if sched_args:
                gen.lr_scheduler = _import_path(sched_args["path"])(gen.optimizer, **sched_args["args"])
                gen.lr_scheduler_name = sched_args["path"]
            weights = {k: (v.numpy().copy() if container == "numpy" else v.clone()) for k, v in init_state.items()}
            rounds = []
            for rnd in range(n_rounds):
                diff = {}
                for k, v in init_state.items():
                    if rnd == 1 and k == "lin2.weight":
                        continue  # a parameter missing from one round's aggregate: not stepped that round
                    if v.dtype == torch.int64:
                        a = np.array(rnd + 1, dtype=np.int64).reshape(v.shape)
                    else:
                        a = (rng.standard_normal(tuple(v.shape)) * 0.05).astype(np.float32)
                    diff[k] = a
                fl_ctx = FLContext()
                fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(weights, {}), private=True, sticky=True)
                fl_ctx.set_prop(AppConstants.CURRENT_ROUND, rnd, private=True, sticky=False)
                cdiff = {k: to_container(v, container) for k, v in diff.items()}
                learnable = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=cdiff, meta={"m": rnd}).to_shareable(), fl_ctx)
                weights = learnable[ModelLearnableKey.WEIGHTS]
                rounds.append({
                    "diff": {k: store.put(v, "diff") for k, v in diff.items()},
                    "weights": {k: store.put(v, "w") for k, v in weights.items()},
                    "weights_type": {k: type(v).__name__ for k, v in weights.items()},
                    "lr_after": gen.optimizer.param_groups[-1]["lr"],
                    "meta": learnable[ModelLearnableKey.META],
                })
            cases.append({"kind": "fedopt", "name": f"{container}_{name}", "container": container, "optimizer_args": opt_args,
                          "lr_scheduler_args": sched_args, "init": init_names, "rounds": rounds})
    np.savez_compressed(os.path.join(HERE, "fedopt_cases.npz"), **store.arrays)
    with open(os.path.join(HERE, "fedopt_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --set fedopt", "reference": "NVFlare (/root/reference, ~2.9.0-dev)",
                   "numpy": np.__version__, "torch": torch.__version__, "torch_threads": torch.get_num_threads(),
                   "cases": cases}, f, indent=1, default=str)
    print(f"wrote {len(cases)} fedopt cases, {len(store.arrays)} arrays")


def main_quant():
    """AdaQuantizer round trips from the reference (ada_quant.py imports only bz2 / numpy / torch; the
    bitsandbytes formats cannot be produced here -- bitsandbytes is not installed)."""
    from nvflare.app_opt.pt.quantization.ada_quant import AdaQuantizer

    rng = np.random.default_rng(20261018)
    store = Store()
    cases = []
    inputs = {
        "normal_4099": rng.standard_normal(4099).astype(np.float32),
        "normal_2d": rng.standard_normal((33, 130)).astype(np.float32),
        "wide_range_u16": (rng.standard_normal(5000) * 300.0).astype(np.float32),
        "constant": np.full((7, 3), 0.625, np.float32),
        "compressible": np.repeat(rng.standard_normal(16).astype(np.float32), 512),
        "tiny": rng.standard_normal(5).astype(np.float32),
    }
    for name, arr in inputs.items():
        for compression in (True, False):
            q, st = AdaQuantizer(compression=compression).quantize(torch.from_numpy(arr.copy()))
            qt = q if isinstance(q, torch.Tensor) else torch.as_tensor(q)  # dequantizer.py:150-153
            deq = AdaQuantizer().dequantized(qt, st) if st else qt
            out = deq.float().numpy() if isinstance(deq, torch.Tensor) else np.asarray(deq, np.float32)
            rec_state = {}
            for k, v in st.items():
                if isinstance(v, np.ndarray):
                    rec_state[k] = {"array": store.put(v, "qs")}
                else:
                    rec_state[k] = v
            qv = q.numpy() if isinstance(q, torch.Tensor) else np.asarray(q)
            cases.append({"kind": "adaquant", "name": f"{name}_{'bz2' if compression else 'raw'}",
                          "input": store.put(arr, "in"), "quantized": store.put(qv, "q"),
                          "quantized_dtype": str(qv.dtype), "quant_state": rec_state,
                          "expected": store.put(out, "out")})
    np.savez_compressed(os.path.join(HERE, "quant_cases.npz"), **store.arrays)
    with open(os.path.join(HERE, "quant_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --set quant", "reference": "NVFlare (/root/reference, ~2.9.0-dev)",
                   "numpy": np.__version__, "torch": torch.__version__, "cases": cases}, f, indent=1, default=str)
    print(f"wrote {len(cases)} quant cases, {len(store.arrays)} arrays")


def _put_any(arrays, tag, v):
    """Store one array of any dtype: (name, dtype string).  bfloat16 is kept as its uint16 bit pattern."""
    name = f"{tag}{len(arrays):05d}"
    if isinstance(v, torch.Tensor):
        dt = str(v.dtype).replace("torch.", "")
        a = v.detach().cpu()
        a = a.view(torch.int16).numpy().view(np.uint16) if v.dtype == torch.bfloat16 else a.numpy()
    else:
        a = np.asarray(v)
        dt = str(a.dtype)
    arrays[name] = np.array(a, copy=True)
    return name, dt


def _as_container(a: np.ndarray, dt: str, container: str):
    if container == "numpy":
        return np.array(a, copy=True)
    if dt == "bfloat16":
        return torch.from_numpy(np.array(a, copy=True)).to(torch.float32).to(torch.bfloat16)
    return torch.from_numpy(np.array(a, copy=True))


def main_dtypes():
    """Reduced-precision and integer client arrays through the reference helper (weighted_aggregation_helper.py:
    153-240): numpy float16 / uint8 / int8 / int16 / bool / uint16 / uint32 / uint64, torch float16 / bfloat16 /
    uint8 / int8 / int16 / bool.  torch runs single-threaded: its 16-bit add_ computes the vectorised path
    (one fp32 fma, one rounding) except on the last n % 32 elements of each thread's chunk, which take the
    scalar path -- recorded as ``vector_end`` so the tests know which elements the vector semantics cover."""
    from nvflare.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    torch.set_num_threads(1)
    rng = np.random.default_rng(20261016)
    arrays, cases = {}, {}

    def values(n, dt, special=False):
        if dt in ("float16", "bfloat16"):
            a = (rng.standard_normal(n) * 3).astype(np.float32)
            if special:
                sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 6e-8, -3e-5, 65504.0, -65504.0, 1e-40, 3e38, 1.0],
                              np.float32)
                idx = rng.choice(n, size=min(n, 2 * sp.size), replace=False)
                a[idx] = np.resize(sp, idx.size)
            if dt == "float16":
                with np.errstate(over="ignore"):
                    return a.astype(np.float16)
            return torch.from_numpy(a).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
        if dt == "bool":
            return rng.integers(0, 2, n).astype(np.bool_)
        info = np.iinfo(np.dtype(dt))
        return rng.integers(max(info.min, -10 ** 6), min(info.max, 10 ** 6), n, endpoint=True).astype(dt)

    def case(name, container, dt, n, K, weights, weighted=True, special=False):
        rows = [values(n, dt, special) for _ in range(K)]
        h = WeightedAggregationHelper(weigh_by_local_iter=weighted)
        for k, r in enumerate(rows):
            src = r if dt != "bfloat16" else r  # bit patterns; converted below
            if dt == "bfloat16":
                v = torch.from_numpy(src.view(np.int16).copy()).view(torch.bfloat16)
            else:
                v = torch.from_numpy(src.copy()) if container == "torch" else src.copy()
            h.add({"w": v}, weights[k], f"site-{k}", 0)
        out = h.get_result()["w"]
        rec = {"container": container, "dtype": dt, "n": n, "weighted": weighted,
               "weights": [repr(w) if isinstance(w, np.generic) else w for w in weights],
               "weight_types": [type(w).__name__ for w in weights],
               "rows": [_put_any(arrays, "in", r)[0] for r in rows]}
        rec["expected"], rec["expected_dtype"] = _put_any(arrays, "out", out)
        rec["vector_end"] = n - n % 32 if container == "torch" and dt in ("float16", "bfloat16") else n
        cases[name] = rec

    def rw(K):
        return [random.random() * float(random.randint(1, 50)) for _ in range(K)]

    random.seed(20261016)
    for n in (64 * 40, 1003):
        for K in (1, 5, 9):
            case(f"numpy_float16_k{K}_n{n}", "numpy", "float16", n, K, rw(K))
            for dt in ("float16", "bfloat16"):
                case(f"torch_{dt}_k{K}_n{n}", "torch", dt, n, K, rw(K))
    for dt in ("float16", "bfloat16"):
        case(f"torch_{dt}_special", "torch", dt, 64 * 8, 6, [1e-3, 3.5, 1e3, 0.1, 7.0, 2.0 ** -20], special=True)
        case(f"torch_{dt}_unweighted", "torch", dt, 64 * 9 + 5, 5, rw(5), weighted=False)
        case(f"torch_{dt}_intweights", "torch", dt, 64 * 16, 16, [1.0 * float(1 + (37 * k) % 100) for k in range(16)])
    case("numpy_float16_special", "numpy", "float16", 509, 6, [1e-3, 3.5, 1e3, 0.1, 7.0, 2.0 ** -20], special=True)
    case("numpy_float16_unweighted", "numpy", "float16", 300, 5, rw(5), weighted=False)
    case("numpy_float16_intweights", "numpy", "float16", 777, 16, [1.0 * float(1 + (37 * k) % 100) for k in range(16)])
    case("numpy_float16_f32weights", "numpy", "float16", 333, 4, [np.float32(x) for x in rw(4)])
    case("numpy_float16_f64weights", "numpy", "float16", 333, 4, [np.float64(x) for x in rw(4)])
    for dt in ("uint8", "int8", "int16", "bool", "uint16", "uint32", "uint64"):
        case(f"numpy_{dt}", "numpy", dt, 257, 5, rw(5))
    for dt in ("uint8", "int8", "int16", "bool"):
        case(f"torch_{dt}", "torch", dt, 257, 5, rw(5))
    np.savez_compressed(os.path.join(HERE, "dtype_cases.npz"), **arrays)
    with open(os.path.join(HERE, "dtype_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --set dtypes", "reference": "NVFlare (/root/reference, ~2.9.0-dev)",
                   "numpy": np.__version__, "torch": torch.__version__, "torch_threads": 1, "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} dtype cases, {len(arrays)} arrays")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--set", choices=["helper", "fedavg", "scaffold", "fedopt", "quant", "dtypes"], default="helper")
    args = ap.parse_args()
    install_shim(args.ref)
    torch.set_num_threads(8)
    if args.set == "fedavg":
        return main_fedavg()
    if args.set == "scaffold":
        return main_scaffold()
    if args.set == "fedopt":
        return main_fedopt()
    if args.set == "quant":
        return main_quant()
    if args.set == "dtypes":
        return main_dtypes()

    rng = np.random.default_rng(20261015)
    random.seed(20261015)
    store = Store()
    cases = []

    def rweights(K):
        # the reference tests' style: random.random() aggregation weight x integer NUM_STEPS
        return [random.random() * float(random.randint(1, 50)) for _ in range(K)]

    for container in ("numpy", "torch"):
        # 1. plain fp32, ragged sizes, random weights
        for K, P in ((1, 1003), (2, 1003), (8, 4099), (64, 2053)):
            rows = [rng.standard_normal(P).astype(np.float32) for _ in range(K)]
            ws = rweights(K)
            run_helper_case(store, cases, f"{container}_f32_k{K}_p{P}", container,
                            [(f"site-{i+1}", ws[i], {"w": rows[i]}) for i in range(K)])
        # 2. synthetic weights of the bench (integers)
        K, P = 16, 777
        rows = [rng.standard_normal(P).astype(np.float32) for _ in range(K)]
        ws = [1.0 * float(1 + (37 * k) % 100) for k in range(K)]
        run_helper_case(store, cases, f"{container}_f32_intweights_k{K}", container,
                        [(f"site-{i+1}", ws[i], {"w": rows[i]}) for i in range(K)])
        # 3. special values: denormals, signed zeros, inf, nan, overflow; tiny and huge weights
        K, P = 6, 509
        rows = [special_values(rng, P) for _ in range(K)]
        ws = [1e-30, 3.5, 1e30, 0.1, 7.0, 2.0 ** -126]
        run_helper_case(store, cases, f"{container}_f32_special", container,
                        [(f"site-{i+1}", ws[i], {"w": rows[i]}) for i in range(K)])
        # 4. denormal-only path (results stay subnormal)
        K, P = 4, 256
        rows = [(rng.standard_normal(P) * 1e-39).astype(np.float32) for _ in range(K)]
        ws = [0.75, 1.25, 3.0, 0.5]
        run_helper_case(store, cases, f"{container}_f32_denormal", container,
                        [(f"site-{i+1}", ws[i], {"w": rows[i]}) for i in range(K)])
        # 5. unweighted (weigh_by_local_iter=False)
        K, P = 5, 300
        rows = [rng.standard_normal(P).astype(np.float32) for _ in range(K)]
        ws = rweights(K)
        run_helper_case(store, cases, f"{container}_f32_unweighted", container,
                        [(f"site-{i+1}", ws[i], {"w": rows[i]}) for i in range(K)], weigh_by_local_iter=False)
        # 6. fp64 inputs
        K, P = 5, 37
        rows = [rng.random(P) for _ in range(K)]
        ws = rweights(K)
        run_helper_case(store, cases, f"{container}_f64_k{K}", container,
                        [(f"site-{i+1}", ws[i], {"w": rows[i]}) for i in range(K)])
        # 7. int64 inputs (torch: promoted to fp32; numpy: promoted to fp64)
        K, P = 3, 7
        rows = [rng.integers(-1000, 1000, P).astype(np.int64) for _ in range(K)]
        ws = [2.0, 3.0, 0.5]
        run_helper_case(store, cases, f"{container}_i64_k{K}", container,
                        [(f"site-{i+1}", ws[i], {"count": rows[i]}) for i in range(K)])
        # 8. partial keys, shapes, 0-d and empty arrays
        shapes = {"conv.weight": (4, 3, 3, 3), "conv.bias": (4,), "fc.weight": (10, 33), "scalar": (), "empty": (0,), "fc.bias": (10,)}
        def mk(keys):
            return {k: rng.standard_normal(shapes[k]).astype(np.float32) for k in keys}
        contribs = [
            ("site-1", 1.5, mk(["conv.weight", "conv.bias", "fc.weight", "scalar", "empty"])),
            ("site-2", 2.0, mk(["conv.weight", "fc.weight", "fc.bias", "scalar"])),
            ("site-3", 0.25, mk(["conv.bias", "fc.weight", "fc.bias", "empty"])),
            ("site-4", 4.0, mk(["conv.weight", "conv.bias", "fc.weight", "fc.bias", "scalar", "empty"])),
        ]
        run_helper_case(store, cases, f"{container}_partial_keys", container, contribs)
        # 9. exclude_vars
        run_helper_case(store, cases, f"{container}_exclude_vars", container, contribs, exclude_vars="bias|scalar")
        # 10. permuted arrival order of the same contributions (different bits)
        K, P = 8, 1021
        rows = [rng.standard_normal(P).astype(np.float32) for _ in range(K)]
        ws = rweights(K)
        base = [(f"site-{i+1}", ws[i], {"w": rows[i]}) for i in range(K)]
        perm = list(rng.permutation(K))
        run_helper_case(store, cases, f"{container}_order_a", container, base)
        run_helper_case(store, cases, f"{container}_order_b", container, [base[i] for i in perm])
        # 11. many keys with ragged sizes (flattened-arena packing)
        sizes = [1, 3, 63, 64, 65, 127, 1000, 4097, 5]
        K = 7
        ws = rweights(K)
        contribs = [(f"site-{i+1}", ws[i], {f"k{j}": rng.standard_normal(s).astype(np.float32) for j, s in enumerate(sizes)}) for i in range(K)]
        run_helper_case(store, cases, f"{container}_many_keys", container, contribs)

    # InTime-level flows (numpy containers, as the SAG numpy jobs deliver them)
    for container in ("numpy", "torch"):
        K = 6
        names = [f"client_{i}" for i in range(K)]
        aw = {n: random.random() for n in names}
        clients = [(n, {"": (random.randint(1, 50), {"var1": rng.standard_normal((6, 6)).astype(np.float32)})}) for n in names]
        run_intime_case(store, cases, f"{container}_intime_single", container, clients, "WEIGHT_DIFF", aggregation_weights=aw)
        dk = {"dxo_0": "WEIGHT_DIFF", "dxo_1": "WEIGHTS"}
        aw2 = {d: {n: random.random() for n in names} for d in dk}
        clients = [(n, {d: (random.randint(1, 50), {"var1": rng.standard_normal(4).astype(np.float32), "bias": rng.standard_normal(3).astype(np.float32)}) for d in dk}) for n in names]
        run_intime_case(store, cases, f"{container}_intime_collection", container, clients, dk, aggregation_weights=aw2, exclude_vars={"dxo_0": "bias", "dxo_1": ""})

    np.savez_compressed(os.path.join(HERE, "helper_cases.npz"), **store.arrays)
    with open(os.path.join(HERE, "helper_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "reference": "NVFlare (/root/reference, ~2.9.0-dev)",
                   "numpy": np.__version__, "torch": torch.__version__, "cases": cases}, f, indent=1, default=str)
    print(f"wrote {len(cases)} cases, {len(store.arrays)} arrays")


if __name__ == "__main__":
    main()
