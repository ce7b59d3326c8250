"""Random FedOpt server steps: the REFERENCE PTFedOptModelShareableGenerator recorded, for replay on the GPU --
TEST INFRASTRUCTURE.

``--record`` (build container, reference tree mounted, namespace shim of tests/ref_suite_plugin.py) runs
nvflare/app_opt/pt/fedopt.py:184-270 on CPU over random cases and writes, per round, the SHA-256 of every
returned weight's bits (NaNs canonicalised), its container type, dtype and shape, and the lr after the step.
Nothing else is stored: tests/test_gpu_fuzz_fedopt.py regenerates every input from the seed (the model
architecture, its initial weights, the optimizer and scheduler settings, the per-round
differences and the keys each round leaves out) and replays them through the drop-in generator on the GPU.

Two families of cases: ``plain`` (SGD with momentum / dampening / nesterov / weight decay / maximize, Adamax,
Rprop, ASGD: no sqrt on the path) and ``sqrt`` (round 3: Adam, AdamW, amsgrad, NAdam, RAdam, RMSprop, Adagrad,
whose steps take torch CPU's sqrt -- MKL vsSqrt, not correctly rounded -- which the drop-in restates,
DESIGN.md section 5.1; replayed with NVFLARE_AMD_TORCH_SQRT=torch_cpu, the sqrt this container's torch computes).

  python tests/fuzz_reference_fedopt.py --record tests/golden/fuzz_fedopt_s31.json --cases 60 --seed 31
  python tests/fuzz_reference_fedopt.py --record tests/golden/fuzz_fedopt_sqrt_s41.json --cases 60 --seed 41 --family sqrt
"""

import argparse
import hashlib
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROUNDS = 3


def build_model(spec):
    """The case's architecture holding its numpy-drawn initial weights (spec["init"])."""
    layers = []
    dims = spec["dims"]
    for i in range(len(dims) - 1):
        layers.append(torch.nn.Linear(dims[i], dims[i + 1], bias=spec["bias"][i]))
        if spec["bn"][i]:
            layers.append(torch.nn.BatchNorm1d(dims[i + 1]))
    model = torch.nn.Sequential(*layers)
    if "init" in spec:
        model.load_state_dict({k: torch.from_numpy(np.array(v, copy=True)) for k, v in spec["init"].items()})
    return model


def sqrt_optimizer(rng) -> dict:
    """A torch optimizer whose step takes a sqrt, with random hyperparameters (family "sqrt")."""
    kind = int(rng.integers(0, 6))
    lr = float(rng.choice([1e-3, 2e-3, 1e-2]))
    if kind in (0, 1):  # Adam / AdamW
        args = {"lr": lr, "betas": [float(rng.choice([0.9, 0.8, 0.3])), float(rng.choice([0.999, 0.99, 0.9]))],
                "eps": float(rng.choice([1e-8, 1e-6]))}
        if rng.random() < 0.4:
            args["weight_decay"] = float(rng.choice([1e-3, 1e-2]))
        if rng.random() < 0.3:
            args["amsgrad"] = True
        if rng.random() < 0.15:
            args["maximize"] = True
        return {"path": "torch.optim.AdamW" if kind == 1 else "torch.optim.Adam", "args": args}
    if kind == 2:
        args = {"lr": lr, "momentum_decay": float(rng.choice([4e-3, 5e-3]))}
        if rng.random() < 0.4:
            args["weight_decay"] = float(rng.choice([1e-3, 1e-2]))
            args["decoupled_weight_decay"] = bool(rng.random() < 0.5)
        return {"path": "torch.optim.NAdam", "args": args}
    if kind == 3:
        args = {"lr": lr}
        if rng.random() < 0.4:
            args["weight_decay"] = float(rng.choice([1e-3, 1e-2]))
        return {"path": "torch.optim.RAdam", "args": args}
    if kind == 4:
        args = {"lr": lr, "alpha": float(rng.choice([0.99, 0.9]))}
        if rng.random() < 0.5:
            args["centered"] = True
        if rng.random() < 0.5:
            args["momentum"] = float(rng.choice([0.5, 0.9]))
        return {"path": "torch.optim.RMSprop", "args": args}
    args = {"lr": float(rng.choice([1e-2, 0.1])), "lr_decay": float(rng.choice([0.0, 0.05]))}
    if rng.random() < 0.4:
        args["weight_decay"] = 1e-3
    return {"path": "torch.optim.Adagrad", "args": args}


def gen_case(rng, family: str = "plain") -> dict:
    container = "torch" if rng.random() < 0.5 else "numpy"
    depth = int(rng.integers(1, 4))
    dims = [int(rng.integers(1, 200)) for _ in range(depth + 1)]
    spec = {"container": container, "dims": dims, "bias": [bool(rng.random() < 0.7) for _ in range(depth)],
            "bn": [bool(rng.random() < 0.4) for _ in range(depth)]}
    kind = int(rng.integers(0, 4)) if family == "plain" else -1
    if family == "sqrt":
        opt = sqrt_optimizer(rng)
    elif kind == 0:
        args = {"lr": float(rng.choice([1.0, 0.5, 0.05]))}
        if rng.random() < 0.7:
            args["momentum"] = float(rng.choice([0.5, 0.9]))
            if rng.random() < 0.4:
                args["nesterov"] = True
            elif rng.random() < 0.5:
                args["dampening"] = float(rng.choice([0.1, 0.5]))
        if rng.random() < 0.4:
            args["weight_decay"] = float(rng.choice([1e-3, 1e-2]))
        if rng.random() < 0.2:
            args["maximize"] = True
        opt = {"path": "torch.optim.SGD", "args": args}
    elif kind == 1:
        opt = {"path": "torch.optim.Adamax", "args": {"lr": float(rng.choice([2e-3, 1e-2])),
                                                      "weight_decay": float(rng.choice([0.0, 1e-2]))}}
    elif kind == 2:
        opt = {"path": "torch.optim.Rprop", "args": {"lr": float(rng.choice([1e-3, 1e-2]))}}
    else:
        opt = {"path": "torch.optim.ASGD", "args": {"lr": float(rng.choice([1e-2, 0.1])),
                                                    "t0": float(rng.choice([1.0, 1e6]))}}
    spec["optimizer_args"] = opt
    spec["lr_scheduler_args"] = ({"path": "torch.optim.lr_scheduler.StepLR", "args": {"step_size": 1, "gamma": 0.5}}
                                 if rng.random() < 0.3 else None)
    state = build_model(spec).state_dict()
    spec["init"] = {k: (np.zeros(tuple(v.shape), np.int64) if v.dtype == torch.int64
                        else (rng.standard_normal(tuple(v.shape)) * 0.1).astype(np.float32)) for k, v in state.items()}
    rounds = []
    for rnd in range(ROUNDS):
        diff = {}
        for k, v in state.items():
            if rnd > 0 and rng.random() < 0.15:
                continue  # a key missing from this round's aggregate
            if v.dtype == torch.int64:
                diff[k] = np.array(int(rng.integers(1, 4)), dtype=np.int64).reshape(tuple(v.shape))
            else:
                diff[k] = (rng.standard_normal(tuple(v.shape)) * float(rng.choice([0.05, 1.0]))).astype(np.float32)
        rounds.append(diff)
    spec["rounds"] = rounds
    return spec


def box(a, container):
    a = np.array(a, copy=True)
    return torch.from_numpy(a) if container == "torch" else a


def digest(v) -> list:
    if isinstance(v, torch.Tensor):
        t = v.detach().cpu()
        kind, dtype, shape = "Tensor", str(t.dtype).replace("torch.", ""), list(t.shape)
        a = t.numpy().copy()
    else:
        a = np.array(np.asarray(v), copy=True)
        kind, dtype, shape = type(v).__name__, str(a.dtype), list(a.shape)
    if a.dtype.kind == "f":
        a[np.isnan(a)] = np.nan
    return [kind, dtype, shape, hashlib.sha256(a.tobytes()).hexdigest()]


def play(gen, spec, FLContext, AppConstants, make_model_learnable, DXO, DataKind, ModelLearnableKey):
    """Run the case's rounds through a generator (the reference's or the drop-in; the API classes are passed in
    so that each side uses its own); per round {key: digest} in output order, the lr after the step, the meta."""
    weights = {k: box(v, spec["container"]) for k, v in spec["init"].items()}
    out = []
    for rnd, diff in enumerate(spec["rounds"]):
        fl_ctx = FLContext()
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(weights, {}), private=True, sticky=True)
        fl_ctx.set_prop(AppConstants.CURRENT_ROUND, rnd, private=True, sticky=False)
        d = {k: box(v, spec["container"]) for k, v in diff.items()}
        learnable = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=d, meta={"r": rnd}).to_shareable(), fl_ctx)
        weights = learnable[ModelLearnableKey.WEIGHTS]
        out.append({"weights": {k: digest(v) for k, v in weights.items()}, "lr": gen.optimizer.param_groups[-1]["lr"],
                    "meta": learnable[ModelLearnableKey.META]})
    return out


def record(path: str, cases: int, seed: int, family: str = "plain") -> None:
    from ref_suite_plugin import _install_shim

    _install_shim(os.environ.get("NVFLARE_REF_ROOT", "/root/reference"))
    from nvflare.apis.dxo import DXO, DataKind
    from nvflare.apis.fl_context import FLContext
    from nvflare.app_common.abstract.model import ModelLearnableKey, make_model_learnable
    from nvflare.app_common.app_constant import AppConstants
    from nvflare.app_opt.pt.fedopt import PTFedOptModelShareableGenerator

    import importlib

    def imp(path):
        mod, _, cls = path.rpartition(".")
        return getattr(importlib.import_module(mod), cls)

    rng = np.random.default_rng(seed)
    recs = []
    for case in range(cases):
        spec = gen_case(rng, family)
        model = build_model(spec)
        opt_args = json.loads(json.dumps(spec["optimizer_args"]))
        gen = PTFedOptModelShareableGenerator(optimizer_args=opt_args, device="cpu")
        gen.model = model
        gen.device = torch.device("cpu")
        gen.optimizer = imp(opt_args["path"])(model.parameters(), **opt_args["args"])
        gen.optimizer_name = opt_args["path"]
        if spec["lr_scheduler_args"]:
            s = spec["lr_scheduler_args"]
            gen.lr_scheduler = imp(s["path"])(gen.optimizer, **s["args"])
            gen.lr_scheduler_name = s["path"]
        rounds = play(gen, spec, FLContext, AppConstants, make_model_learnable, DXO, DataKind, ModelLearnableKey)
        recs.append({"case": case, "optimizer": opt_args["path"], "container": spec["container"], "rounds": rounds})
    with open(path, "w") as f:
        json.dump({"generator": "tests/fuzz_reference_fedopt.py --record", "seed": seed, "cases": cases,
                   "family": family,
                   "reference": "NVFlare app_opt/pt/fedopt.py (/root/reference), torch CPU",
                   "numpy": np.__version__, "torch": torch.__version__, "torch_threads": torch.get_num_threads(),
                   "records": recs}, f, indent=0)
    print(json.dumps({"cases": cases, "rounds": sum(len(r["rounds"]) for r in recs)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--record", required=True)
    ap.add_argument("--cases", type=int, default=40)
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("--family", choices=["plain", "sqrt"], default="plain")
    a = ap.parse_args()
    record(a.record, a.cases, a.seed, a.family)


if __name__ == "__main__":
    main()
