"""Drop-in FedOpt shareable generator on the GPU vs the reference generator's own outputs.

tests/golden/fedopt_cases.* hold three rounds of ``PTFedOptModelShareableGenerator.shareable_to_learnable``
(nvflare/app_opt/pt/fedopt.py:184-270, run on CPU by make_golden.py --set fedopt) for SGD (plain,
momentum + dampening + weight decay, nesterov, StepLR), Adam (default, betas/eps/weight decay,
CosineAnnealingLR) and AdamW, numpy and torch containers, a BatchNorm model (fp32 running stats and an
int64 ``num_batches_tracked`` go through the FedAvg ``base + diff`` branch) and a parameter missing from
round 2 (not stepped that round).

Bar: every output bit-exact -- Adam / AdamW parameters too, with the device epilogue running torch CPU's sqrt
(MKL vsSqrt, not correctly rounded; restated, nvflare_amd/torch_sqrt.py and tests/test_torch_sqrt.py); with the
correctly rounded sqrt (NVFLARE_AMD_TORCH_SQRT=ieee) Adam parameters are within
``2 * steps * spacing(max(|p0|, |p_torch|, lr))``; lr schedule and meta identical.  Tests against torch running
on this host use the sqrt torch_sqrt.detect() finds here (exact when it is one of the two)."""

import numpy as np
import pytest
import torch

from golden_util import assert_fedopt_param, fedopt_model, load_fedopt_golden, same_bits
from nvflare_amd.app_opt.pt import PTFedOptModelShareableGenerator
from nvflare_amd.compat import DXO, AppConstants, DataKind, EventType, FLContext, ModelLearnableKey, make_model_learnable

pytestmark = pytest.mark.gpu

META, ARRAYS = load_fedopt_golden()
CASES = META["cases"]


def _container(a, container):
    a = np.array(a, copy=True)
    return torch.from_numpy(a) if container == "torch" else a


def _np(v):
    return v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


@pytest.mark.parametrize("sqrt_mode", ["torch_cpu", "ieee"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_fedopt_generator_matches_reference(case, sqrt_mode, monkeypatch):
    monkeypatch.setenv("NVFLARE_AMD_TORCH_SQRT", sqrt_mode)
    container = case["container"]
    model = fedopt_model()
    model.load_state_dict({k: torch.from_numpy(np.array(ARRAYS[v], copy=True)) for k, v in case["init"].items()})
    import copy

    gen = PTFedOptModelShareableGenerator(optimizer_args=copy.deepcopy(case["optimizer_args"]),
                                          lr_scheduler_args=copy.deepcopy(case["lr_scheduler_args"]),
                                          source_model=model, device="cuda:0")
    gen.handle_event(EventType.START_RUN, FLContext())
    assert gen.optimizer is not None
    is_adam = "Adam" in case["optimizer_args"]["path"]
    lr = case["optimizer_args"]["args"]["lr"]
    param_names = {n for n, _ in model.named_parameters()}
    weights = {k: _container(ARRAYS[v], container) for k, v in case["init"].items()}
    steps = {n: 0 for n in param_names}
    for rnd, exp in enumerate(case["rounds"]):
        fl_ctx = FLContext()
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(weights, {}), private=True, sticky=True)
        fl_ctx.set_prop(AppConstants.CURRENT_ROUND, rnd, private=True, sticky=False)
        diff = {k: _container(ARRAYS[v], container) for k, v in exp["diff"].items()}
        learnable = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff, meta={"m": rnd}).to_shareable(), fl_ctx)
        out = learnable[ModelLearnableKey.WEIGHTS]
        assert learnable[ModelLearnableKey.META] == exp["meta"]
        assert set(out) == set(exp["weights"])
        for n in param_names:
            if n in diff:
                steps[n] += 1
        for k, name in exp["weights"].items():
            assert type(out[k]).__name__ == exp["weights_type"][k], k
            got, ref = _np(out[k]), ARRAYS[name]
            assert got.dtype == ref.dtype and got.shape == ref.shape, k
            if is_adam and k in param_names:
                assert_fedopt_param(got, ref, ARRAYS[case["init"][k]], lr, steps[k], "torch_cpu", (case["name"], rnd, k))
            else:
                assert same_bits(got, ref), (case["name"], rnd, k)
        assert gen.optimizer.param_groups[-1]["lr"] == exp["lr_after"]
        weights = out


def test_fedopt_generator_optimizer_state_views():
    """optimizer.state holds views of the device buffers after a step (checkpointable as with torch)."""
    model = fedopt_model()
    gen = PTFedOptModelShareableGenerator(optimizer_args={"path": "torch.optim.Adam", "args": {"lr": 1e-3}},
                                          source_model=model, device=0)
    gen.handle_event(EventType.START_RUN, FLContext())
    w = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(w, {}))
    diff = {k: np.full(v.shape, 0.01, np.float32) for k, v in w.items() if v.dtype == np.float32}
    gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff).to_shareable(), fl_ctx)
    sd = gen.optimizer.state_dict()
    p = model.lin1.weight
    st = gen.optimizer.state[p]
    assert float(st["step"]) == 1.0
    assert st["exp_avg"].device.type == "cuda" and st["exp_avg"].shape == p.shape
    # exp_avg after one step = (1 - beta1) * g with g = -0.01
    assert torch.allclose(st["exp_avg"].cpu(), torch.full(p.shape, -0.001))
    assert len(sd["state"]) == len(list(model.parameters()))


def test_fedopt_generator_rprop_matches_torch():
    """Rprop through the drop-in generator for four rounds, one parameter skipped in round 1 (its state is
    made at its own first step, as torch's is): params, prev and step_size bit-exact against torch CPU."""
    import copy

    model = fedopt_model()
    ref_model = copy.deepcopy(model)
    ref_opt = torch.optim.Rprop(ref_model.parameters(), lr=1e-2, foreach=False)
    gen = PTFedOptModelShareableGenerator(optimizer_args={"path": "torch.optim.Rprop", "args": {"lr": 1e-2}},
                                          source_model=model, device=0)
    gen.handle_event(EventType.START_RUN, FLContext())
    w = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    rng = np.random.default_rng(14)
    for rnd in range(4):
        fl_ctx = FLContext()
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(w, {}))
        diff = {k: (rng.standard_normal(v.shape) * 0.05).astype(np.float32) for k, v in w.items()
                if v.dtype == np.float32 and not (rnd == 0 and k == "lin2.weight")}
        w = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff).to_shareable(), fl_ctx)[
            ModelLearnableKey.WEIGHTS]
        ref_opt.zero_grad()
        for n, p in ref_model.named_parameters():
            p.grad = torch.tensor(-1.0 * diff[n]) if n in diff else None
        ref_opt.step()
    for (n, p), (_, rp) in zip(model.named_parameters(), ref_model.named_parameters()):
        st, rst = gen.optimizer.state[p], ref_opt.state[rp]
        assert float(st["step"]) == float(rst["step"]), n
        assert same_bits(_np(w[n]), rp.detach().numpy()), n
        assert same_bits(st["prev"].cpu().numpy(), rst["prev"].numpy()), n
        assert same_bits(st["step_size"].cpu().numpy(), rst["step_size"].numpy()), n


def test_fedopt_generator_adamax_state_matches_torch():
    """Adamax (no sqrt on its path): params, exp_avg and exp_inf bit-exact against torch CPU stepping the same
    -diff, over two rounds; optimizer.state holds views of the device buffers."""
    import copy

    model = fedopt_model()
    ref_model = copy.deepcopy(model)
    ref_opt = torch.optim.Adamax(ref_model.parameters(), lr=2e-3, weight_decay=1e-3, foreach=False)
    gen = PTFedOptModelShareableGenerator(optimizer_args={"path": "torch.optim.Adamax",
                                                          "args": {"lr": 2e-3, "weight_decay": 1e-3}},
                                          source_model=model, device=0)
    gen.handle_event(EventType.START_RUN, FLContext())
    w = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    rng = np.random.default_rng(12)
    for rnd in range(2):
        fl_ctx = FLContext()
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(w, {}))
        diff = {k: (rng.standard_normal(v.shape) * 0.05).astype(np.float32) for k, v in w.items()
                if v.dtype == np.float32}
        w = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff).to_shareable(), fl_ctx)[
            ModelLearnableKey.WEIGHTS]
        ref_opt.zero_grad()
        for n, p in ref_model.named_parameters():
            p.grad = torch.tensor(-1.0 * diff[n])
        ref_opt.step()
    for (n, p), (_, rp) in zip(model.named_parameters(), ref_model.named_parameters()):
        st, rst = gen.optimizer.state[p], ref_opt.state[rp]
        assert st["exp_inf"].device.type == "cuda" and float(st["step"]) == 2.0
        assert same_bits(_np(w[n]), rp.detach().numpy()), n
        assert same_bits(st["exp_avg"].cpu().numpy(), rst["exp_avg"].numpy()), n
        assert same_bits(st["exp_inf"].cpu().numpy(), rst["exp_inf"].numpy()), n


@pytest.mark.parametrize("opt_name", ["NAdam", "RAdam"])
def test_fedopt_generator_nadam_radam_state(opt_name):
    """NAdam / RAdam through the drop-in generator for three rounds: exp_avg / exp_avg_sq and NAdam's
    mu_product match torch CPU stepping the same -diff (bit-exact), params bit-exact with this host's torch sqrt;
    optimizer.state holds views of the device buffers."""
    import copy

    model = fedopt_model()
    ref_model = copy.deepcopy(model)
    ref_opt = getattr(torch.optim, opt_name)(ref_model.parameters(), lr=2e-3, foreach=False)
    gen = PTFedOptModelShareableGenerator(optimizer_args={"path": f"torch.optim.{opt_name}", "args": {"lr": 2e-3}},
                                          source_model=model, device=0)
    gen.handle_event(EventType.START_RUN, FLContext())
    w = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    p0 = {n: p.detach().cpu().numpy().copy() for n, p in ref_model.named_parameters()}
    rng = np.random.default_rng(13)
    for rnd in range(3):
        fl_ctx = FLContext()
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(w, {}))
        diff = {k: (rng.standard_normal(v.shape) * 0.05).astype(np.float32) for k, v in w.items()
                if v.dtype == np.float32}
        w = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff).to_shareable(), fl_ctx)[
            ModelLearnableKey.WEIGHTS]
        ref_opt.zero_grad()
        for n, p in ref_model.named_parameters():
            p.grad = torch.tensor(-1.0 * diff[n])
        ref_opt.step()
    for (n, p), (_, rp) in zip(model.named_parameters(), ref_model.named_parameters()):
        st, rst = gen.optimizer.state[p], ref_opt.state[rp]
        assert st["exp_avg"].device.type == "cuda" and float(st["step"]) == 3.0
        assert same_bits(st["exp_avg"].cpu().numpy(), rst["exp_avg"].numpy()), n
        assert same_bits(st["exp_avg_sq"].cpu().numpy(), rst["exp_avg_sq"].numpy()), n
        if opt_name == "NAdam":
            assert same_bits(st["mu_product"].numpy(), rst["mu_product"].numpy()), n
        assert_fedopt_param(_np(w[n]), rp.detach().numpy(), p0[n], 2e-3, 3, "live", n)


def test_fedopt_generator_rejects_unsupported_optimizer():
    model = fedopt_model()
    gen = PTFedOptModelShareableGenerator(optimizer_args={"path": "torch.optim.LBFGS", "args": {"lr": 1e-3}},
                                          source_model=model, device=0)
    gen.handle_event(EventType.START_RUN, FLContext())
    w = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(w, {}))
    diff = {"lin1.weight": np.zeros((64, 7), np.float32)}
    with pytest.raises(NotImplementedError, match="LBFGS"):
        gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff).to_shareable(), fl_ctx)


def test_full_model_generator_weight_diff_apply():
    """full_model_shareable_generator.py:58-67 on the device: bit-exact numpy / torch adds, host ints."""
    from nvflare_amd.app_common.shareablegenerators import FullModelShareableGenerator

    rng = np.random.default_rng(3)
    gen = FullModelShareableGenerator(device=0)
    for container in ("numpy", "torch"):
        base = {"a": rng.standard_normal((33, 129)).astype(np.float32), "b": rng.standard_normal(5000).astype(np.float32),
                "n": np.array(7, np.int64), "s": np.array(1.5, np.float32)}
        diff = {"a": rng.standard_normal((33, 129)).astype(np.float32), "b": rng.standard_normal(5000).astype(np.float32),
                "n": np.array(2, np.int64), "s": np.array(0.25, np.float32)}
        expect = {k: base[k] + diff[k] for k in base}
        cb = {k: _container(v, container) for k, v in base.items()}
        cd = {k: _container(v, container) for k, v in diff.items()}
        fl_ctx = FLContext()
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(cb, {}))
        out = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=cd, meta={"x": 1}).to_shareable(), fl_ctx)
        for k in base:
            assert same_bits(_np(out[ModelLearnableKey.WEIGHTS][k]), np.asarray(expect[k])), (container, k)
        assert out[ModelLearnableKey.META] == {"x": 1}


@pytest.mark.parametrize("cls,args", [("torch.optim.Adam", {"lr": 1e-2, "betas": [0.5, 0.9], "amsgrad": True}),
                                      ("torch.optim.AdamW", {"lr": 1e-2, "weight_decay": 0.1, "amsgrad": True})])
def test_fedopt_generator_amsgrad_vs_torch(cls, args):
    """Adam / AdamW(amsgrad=True) on the device against the reference's arithmetic, torch's CPU optimizer
    stepping ``param.grad = -diff`` (fedopt.py:157-182), over four rounds with shrinking differences so
    exp_avg_sq falls below its running max.  m, v, max_exp_avg_sq and the parameters bit-exact (this host's torch
    sqrt, golden_util.assert_fedopt_param); optimizer.state exposes max_exp_avg_sq as a device view."""
    import copy

    rng = np.random.default_rng(11)
    model = fedopt_model()
    ref_model = copy.deepcopy(model)
    kw = dict(args)
    if "betas" in kw:
        kw["betas"] = tuple(kw["betas"])
    ref_opt = {"torch.optim.Adam": torch.optim.Adam, "torch.optim.AdamW": torch.optim.AdamW}[cls](
        ref_model.parameters(), foreach=False, **kw)
    gen = PTFedOptModelShareableGenerator(optimizer_args={"path": cls, "args": copy.deepcopy(args)},
                                          source_model=model, device="cuda:0")
    gen.handle_event(EventType.START_RUN, FLContext())
    w = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    p0 = {n: p.detach().cpu().numpy().copy() for n, p in ref_model.named_parameters()}
    for rnd, scale in enumerate([1.0, 0.02, 1.0, 0.01]):
        diff = {n: (rng.standard_normal(tuple(p.shape)) * 0.05 * scale).astype(np.float32)
                for n, p in ref_model.named_parameters()}
        fl_ctx = FLContext()
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(w, {}))
        out = gen.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data=diff).to_shareable(), fl_ctx)
        w = out[ModelLearnableKey.WEIGHTS]
        for n, p in ref_model.named_parameters():
            p.grad = torch.tensor(-1.0 * diff[n])
        ref_opt.step()
        for n, p in ref_model.named_parameters():
            assert_fedopt_param(_np(w[n]), p.detach().numpy(), p0[n], args["lr"], rnd + 1, "live", (rnd, n))
    gp = dict(model.named_parameters())
    moved = 0
    for n, p in ref_model.named_parameters():
        st, rst = gen.optimizer.state[gp[n]], ref_opt.state[p]
        assert st["max_exp_avg_sq"].device.type == "cuda"
        for key in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
            assert same_bits(st[key].cpu().numpy(), rst[key].numpy()), (n, key)
        moved += int((st["max_exp_avg_sq"] != st["exp_avg_sq"]).sum())
    assert moved > 0
