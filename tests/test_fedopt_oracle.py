"""Pin the server-optimizer epilogue restatement (oracle/fedavg_oracle.c, oracle_epilogue_apply) against
torch's own CPU optimizers, which NVFlare's FedOpt calls (app_opt/pt/fedopt.py:157-182 with
torch/optim/sgd.py and torch/optim/adam.py _single_tensor_*).  No NVFlare test pins these numerics
("parity unpinned" upstream); torch 2.10 CPU is the pin here.

Tolerances:  SGD (all options) and Adam's exp_avg / exp_avg_sq: bit-exact.  Adam params: torch CPU's
sqrt goes through MKL and is not correctly rounded (~0.6 % of results 1 ulp off); the restatement and the
GPU use IEEE sqrt, so a param may differ by one rounding of `p + update` per step:
    |p - p_torch| <= steps * spacing(max(|p_0|, |p_torch|, lr))      (elementwise)
(lr bounds the magnitude of an Adam update; measured: max |diff| = 2^-22 after 5 steps, 0.01-0.1 % of
elements differ at all)."""

import numpy as np
import pytest
import torch

from golden_util import same_bits


def _ulp_diff(a, b):
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


def _torch_steps(opt_cls, kw, p0, deltas):
    p = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    opt = opt_cls([p], foreach=False, **kw)
    for d in deltas:
        opt.zero_grad()
        p.grad = torch.tensor(-1.0 * d)  # fedopt.py:175
        opt.step()
    return p.detach().numpy().copy(), opt.state[p]


@pytest.mark.parametrize("kw", [
    dict(lr=1.0),
    dict(lr=0.7, momentum=0.9),
    dict(lr=0.05, momentum=0.6, dampening=0.1),
    dict(lr=0.05, momentum=0.9, nesterov=True),
    dict(lr=0.1, momentum=0.9, weight_decay=1e-2),
    dict(lr=0.3, maximize=True, momentum=0.5),
])
def test_sgd_bit_exact_vs_torch(oracle, kw):
    rng = np.random.default_rng(0)
    n = 100_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.1).astype(np.float32) for _ in range(4)]
    tp, st = _torch_steps(torch.optim.SGD, kw, p0, deltas)
    p, buf = p0.copy(), np.zeros(n, np.float32)
    for s, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_SGD, p=p, m=buf, first_step=int(s == 0), lr=kw["lr"],
                              momentum=kw.get("momentum", 0.0), dampening=kw.get("dampening", 0.0),
                              weight_decay=kw.get("weight_decay", 0.0), nesterov=int(kw.get("nesterov", False)),
                              maximize=int(kw.get("maximize", False)))
    assert same_bits(p, tp)
    if kw.get("momentum"):
        assert same_bits(buf, st["momentum_buffer"].numpy())


@pytest.mark.parametrize("cls,kw", [
    (torch.optim.Adam, dict(lr=1e-3)),
    (torch.optim.Adam, dict(lr=1e-2, betas=(0.8, 0.99), eps=1e-6)),
    (torch.optim.Adam, dict(lr=1e-3, weight_decay=1e-2)),
    (torch.optim.AdamW, dict(lr=1e-3, weight_decay=1e-2)),
    (torch.optim.Adam, dict(lr=1e-3, betas=(0.3, 0.999))),  # lerp weight >= 0.5 branch
    (torch.optim.Adam, dict(lr=1e-3, amsgrad=True)),
    (torch.optim.AdamW, dict(lr=1e-3, weight_decay=1e-2, amsgrad=True)),
    (torch.optim.Adam, dict(lr=1e-3, betas=(0.5, 0.9), amsgrad=True)),  # v falls below its running max often
])
def test_adam_vs_torch(oracle, cls, kw):
    rng = np.random.default_rng(1)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    # amsgrad: shrinking later updates let exp_avg_sq fall below its running max (both branches of the max)
    scales = [1.0, 1.0, 0.05, 1.0, 0.01] if kw.get("amsgrad") else [1.0] * 5
    deltas = [(rng.standard_normal(n) * 0.01 * sc).astype(np.float32) for sc in scales]
    tp, st = _torch_steps(cls, kw, p0, deltas)
    b1, b2 = kw.get("betas", (0.9, 0.999))
    p, m, v = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    vmax = np.zeros(n, np.float32)
    for s, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p, m=m, v=v, vmax=vmax, lr=kw["lr"], beta1=b1, beta2=b2,
                              eps=kw.get("eps", 1e-8), weight_decay=kw.get("weight_decay", 0.0 if cls is torch.optim.Adam else 1e-2),
                              decoupled_weight_decay=int(cls is torch.optim.AdamW), step=float(s + 1),
                              amsgrad=int(bool(kw.get("amsgrad"))))
    if kw.get("amsgrad"):
        assert same_bits(vmax, st["max_exp_avg_sq"].numpy()), "max_exp_avg_sq"
        assert np.count_nonzero(vmax != v) > n // 100  # the max branch was exercised
    if kw.get("weight_decay") and cls is torch.optim.Adam:
        # coupled weight decay feeds p (a rounding off through torch's sqrt) back into g = -d + wd*p,
        # so m and v inherit it at the scale of wd*|p|: compare within that
        for ours, ref in ((m, st["exp_avg"].numpy()), (v, st["exp_avg_sq"].numpy())):
            scale = np.maximum(np.abs(ref), np.float32(kw["weight_decay"]) * np.abs(p0))
            assert np.all(np.abs(ours.astype(np.float64) - ref) <= len(deltas) * np.spacing(scale))
    else:
        assert same_bits(m, st["exp_avg"].numpy()), "exp_avg"
        assert same_bits(v, st["exp_avg_sq"].numpy()), "exp_avg_sq"
    steps = len(deltas)
    tol = steps * np.spacing(np.maximum(np.maximum(np.abs(p0), np.abs(tp)), np.float32(kw["lr"]))).astype(np.float64)
    diff = np.abs(p.astype(np.float64) - tp.astype(np.float64))
    assert np.all(diff <= tol), float((diff / tol).max())
    assert float((diff > 0).mean()) < 0.01


@pytest.mark.parametrize("kw", [
    dict(lr=1e-2),
    dict(lr=0.1, lr_decay=0.05, weight_decay=1e-3, eps=1e-8),
    dict(lr=1e-2, initial_accumulator_value=0.1, maximize=True),
])
def test_adagrad_vs_torch(oracle, kw):
    """torch/optim/adagrad.py _single_tensor_adagrad (FedAdagrad): state_sum bit-exact; params within the
    sqrt bound (torch CPU's vectorised sqrt), as for Adam."""
    rng = np.random.default_rng(3)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(5)]
    tp, st = _torch_steps(torch.optim.Adagrad, kw, p0, deltas)
    p = p0.copy()
    s = np.full(n, kw.get("initial_accumulator_value", 0.0), np.float32)
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_ADAGRAD, p=p, m=s, lr=kw["lr"], lr_decay=kw.get("lr_decay", 0.0),
                              weight_decay=kw.get("weight_decay", 0.0), eps=kw.get("eps", 1e-10),
                              maximize=int(kw.get("maximize", False)), step=float(k + 1))
    if kw.get("weight_decay"):  # p feeds back into g: sum inherits p's sqrt-rounding differences at wd scale
        scale = np.maximum(np.abs(st["sum"].numpy()), np.float32(kw["weight_decay"]) * np.abs(p0))
        assert np.all(np.abs(s.astype(np.float64) - st["sum"].numpy()) <= len(deltas) * np.spacing(scale))
    else:
        assert same_bits(s, st["sum"].numpy()), "sum"
    tol = len(deltas) * np.spacing(np.maximum(np.maximum(np.abs(p0), np.abs(tp)), np.float32(kw["lr"]))).astype(np.float64)
    diff = np.abs(p.astype(np.float64) - tp.astype(np.float64))
    assert np.all(diff <= tol), float((diff / tol).max())
    assert float((diff > 0).mean()) < 0.01


@pytest.mark.parametrize("kw", [
    dict(lr=1e-2),
    dict(lr=1e-2, alpha=0.9, eps=1e-6, momentum=0.9),
    dict(lr=1e-3, centered=True, weight_decay=1e-3),
    dict(lr=1e-3, centered=True, momentum=0.5, maximize=True),
])
def test_rmsprop_vs_torch(oracle, kw):
    """torch/optim/rmsprop.py _single_tensor_rmsprop: square_avg, momentum_buffer and grad_avg bit-exact
    (without weight decay feeding p back); params within the sqrt bound, as for Adam."""
    rng = np.random.default_rng(4)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(5)]
    tp, st = _torch_steps(torch.optim.RMSprop, kw, p0, deltas)
    p, sq, buf, ga = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_RMSPROP, p=p, m=sq, v=buf, vmax=ga, lr=kw["lr"], alpha=kw.get("alpha", 0.99),
                              eps=kw.get("eps", 1e-8), momentum=kw.get("momentum", 0.0),
                              weight_decay=kw.get("weight_decay", 0.0), centered=int(kw.get("centered", False)),
                              maximize=int(kw.get("maximize", False)), step=float(k + 1))
    steps = len(deltas)
    # every step adds a term g / avg with |g / avg| <= 1 / sqrt(1 - alpha) (square_avg >= (1 - alpha) g^2):
    # torch's sqrt (1 ulp off on ~0.6 % of elements) perturbs such terms, which the momentum buffer sums
    unit = np.float32(1.0 / np.sqrt(1.0 - kw.get("alpha", 0.99)))
    states = [(sq, "square_avg")] + ([(buf, "momentum_buffer")] if kw.get("momentum") else []) + \
             ([(ga, "grad_avg")] if kw.get("centered") else [])
    for ours, key in states:
        ref = st[key].numpy()
        if kw.get("weight_decay") or key == "momentum_buffer":  # inputs carry torch's sqrt roundings
            scale = np.maximum(np.abs(ref), unit if key == "momentum_buffer" else np.float32(0))
            scale = np.maximum(scale, np.float32(kw.get("weight_decay", 0.0)) * np.abs(p0))
            assert np.all(np.abs(ours.astype(np.float64) - ref) <= steps * 2 * np.spacing(scale)), key
            assert float((ours != ref).mean()) < 0.02, key
        else:
            assert same_bits(ours, ref), key
    tol = 2 * steps * np.spacing(np.maximum(np.maximum(np.abs(p0), np.abs(tp)), np.float32(kw["lr"]))).astype(np.float64)
    tol += kw["lr"] * steps * steps * 2 * float(np.spacing(unit))
    diff = np.abs(p.astype(np.float64) - tp.astype(np.float64))
    assert np.all(diff <= tol), float((diff / tol).max())
    assert float((diff > 0).mean()) < 0.02


def test_add_base_matches_numpy_generator(oracle):
    """full_model_shareable_generator.py:58-67: weights[k] = weights[k] + diff[k] (numpy fp32 add)."""
    rng = np.random.default_rng(2)
    base = rng.standard_normal(10_001).astype(np.float32)
    d = rng.standard_normal(10_001).astype(np.float32)
    assert same_bits(oracle.epilogue_apply(d, oracle.EPI_ADD_BASE, base=base), base + d)


@pytest.mark.parametrize("kw", [
    dict(lr=2e-3),
    dict(lr=1e-2, betas=(0.8, 0.95), eps=1e-6, weight_decay=1e-3),
    dict(lr=1e-3, maximize=True),
])
def test_adamax_vs_torch(oracle, kw):
    """torch/optim/adamax.py _single_tensor_adamax (no sqrt on the path): exp_avg, exp_inf and params
    bit-exact against torch CPU."""
    rng = np.random.default_rng(6)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(5)]
    tp, st = _torch_steps(torch.optim.Adamax, kw, p0, deltas)
    p, m, u = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    b1, b2 = kw.get("betas", (0.9, 0.999))
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_ADAMAX, p=p, m=m, v=u, lr=kw["lr"], beta1=b1, beta2=b2,
                              eps=kw.get("eps", 1e-8), weight_decay=kw.get("weight_decay", 0.0),
                              maximize=int(kw.get("maximize", False)), step=float(k + 1))
    assert same_bits(m, st["exp_avg"].numpy()), "exp_avg"
    assert same_bits(u, st["exp_inf"].numpy()), "exp_inf"
    assert same_bits(p, tp), "param"


def nadam_mu_product(mu_product, beta1, momentum_decay, step):
    """torch/optim/nadam.py: ``mu_product *= mu`` on the fp32 state tensor (what DeviceServerOptimizer keeps)."""
    mu = beta1 * (1.0 - 0.5 * (0.96 ** (step * momentum_decay)))
    return np.float32(np.float32(mu_product) * np.float32(mu))


@pytest.mark.parametrize("opt_name,kw", [
    ("NAdam", dict(lr=2e-3)),
    ("NAdam", dict(lr=1e-2, betas=(0.8, 0.95), weight_decay=1e-3, momentum_decay=5e-3)),
    ("NAdam", dict(lr=1e-3, weight_decay=1e-2, decoupled_weight_decay=True, maximize=True)),
    ("RAdam", dict(lr=1e-3)),
    ("RAdam", dict(lr=1e-2, betas=(0.8, 0.9), weight_decay=1e-3)),
    ("RAdam", dict(lr=1e-3, weight_decay=1e-2, decoupled_weight_decay=True, maximize=True)),
])
def test_nadam_radam_vs_torch(oracle, opt_name, kw):
    """torch/optim/nadam.py and radam.py single-tensor steps: exp_avg / exp_avg_sq bit-exact (without weight
    decay feeding p back), NAdam's fp32 mu_product bit-exact, params within the Adam sqrt bound.  Eight steps,
    so RAdam crosses from the unrectified (rho_t <= 5) to the rectified branch with betas (0.9, 0.999)."""
    rng = np.random.default_rng(8)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(8)]
    tp, st = _torch_steps(getattr(torch.optim, opt_name), kw, p0, deltas)
    p, m, v = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    b1, b2 = kw.get("betas", (0.9, 0.999))
    md = kw.get("momentum_decay", 4e-3)
    mp = np.float32(1.0)
    kind = oracle.EPI_NADAM if opt_name == "NAdam" else oracle.EPI_RADAM
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, kind, p=p, m=m, v=v, lr=kw["lr"], beta1=b1, beta2=b2, eps=kw.get("eps", 1e-8),
                              weight_decay=kw.get("weight_decay", 0.0), maximize=int(kw.get("maximize", False)),
                              decoupled_weight_decay=int(kw.get("decoupled_weight_decay", False)),
                              momentum_decay=md, mu_product=float(mp), step=float(k + 1))
        mp = nadam_mu_product(mp, b1, md, k + 1)
    if opt_name == "NAdam":
        assert same_bits(np.array(mp), st["mu_product"].numpy()), "mu_product"
    steps = len(deltas)
    for ours, key in ((m, "exp_avg"), (v, "exp_avg_sq")):
        ref = st[key].numpy()
        if kw.get("weight_decay") and not kw.get("decoupled_weight_decay"):
            scale = np.maximum(np.abs(ref), np.float32(kw["weight_decay"]) * np.abs(p0))
            assert np.all(np.abs(ours.astype(np.float64) - ref) <= steps * np.spacing(scale)), key
        else:
            assert same_bits(ours, ref), key
    tol = 2 * steps * np.spacing(np.maximum(np.maximum(np.abs(p0), np.abs(tp)), np.float32(kw["lr"]))).astype(np.float64)
    diff = np.abs(p.astype(np.float64) - tp.astype(np.float64))
    assert np.all(diff <= tol), float((diff / tol).max())
    assert float((diff > 0).mean()) < 0.02


@pytest.mark.parametrize("kw", [
    dict(lr=1e-2),
    dict(lr=5e-2, etas=(0.3, 1.5), step_sizes=(1e-3, 0.08)),
    dict(lr=1e-3, maximize=True),
])
def test_rprop_vs_torch(oracle, kw):
    """torch/optim/rprop.py _single_tensor_rprop: sign-driven step sizes, no rounding beyond one multiply per
    state, so params, prev and step_size are bit-exact against torch CPU.  Deltas alternate in sign on part
    of the elements so every branch (etaplus, etaminus with the gradient zeroed, 1) is taken."""
    rng = np.random.default_rng(9)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    base = (rng.standard_normal(n) * 0.01).astype(np.float32)
    deltas = [np.where(rng.random(n) < 0.3, -base, base).astype(np.float32) for _ in range(6)]
    deltas[2][::7] = 0.0
    tp, st = _torch_steps(torch.optim.Rprop, kw, p0, deltas)
    p, prev, ss = p0.copy(), np.zeros(n, np.float32), np.full(n, kw["lr"], np.float32)
    em, ep = kw.get("etas", (0.5, 1.2))
    lo, hi = kw.get("step_sizes", (1e-6, 50))
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_RPROP, p=p, m=prev, v=ss, lr=kw["lr"], etaminus=em, etaplus=ep,
                              step_size_min=lo, step_size_max=hi, maximize=int(kw.get("maximize", False)),
                              step=float(k + 1))
    assert same_bits(prev, st["prev"].numpy()), "prev"
    assert same_bits(ss, st["step_size"].numpy()), "step_size"
    assert same_bits(p, tp), "param"


def asgd_host_states(lr, lambd, alpha, t0, step):
    """torch/optim/asgd.py: eta and mu after step ``step`` (fp32 state tensors)."""
    eta = np.float32(lr / ((1 + lambd * lr * step) ** alpha))
    mu = np.float32(1 / max(1, step - t0))
    return eta, mu


@pytest.mark.parametrize("kw", [
    dict(lr=1e-2),
    dict(lr=5e-2, lambd=1e-2, alpha=0.5, t0=2, weight_decay=1e-3),
    dict(lr=1e-2, t0=0, maximize=True),
])
def test_asgd_vs_torch(oracle, kw):
    """torch/optim/asgd.py _single_tensor_asgd (no sqrt): params and ax bit-exact against torch CPU, eta / mu
    host states too; t0 small enough that the averaging branch (mu != 1) is taken."""
    rng = np.random.default_rng(10)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(6)]
    tp, st = _torch_steps(torch.optim.ASGD, kw, p0, deltas)
    p, ax = p0.copy(), np.zeros(n, np.float32)
    lr, lambd, alpha, t0 = kw["lr"], kw.get("lambd", 1e-4), kw.get("alpha", 0.75), kw.get("t0", 1e6)
    eta, mu = np.float32(lr), np.float32(1.0)
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_ASGD, p=p, m=ax, eta=float(eta), mu=float(mu), lambd=lambd,
                              weight_decay=kw.get("weight_decay", 0.0), maximize=int(kw.get("maximize", False)),
                              step=float(k + 1))
        eta, mu = asgd_host_states(lr, lambd, alpha, t0, k + 1)
    assert same_bits(np.array(eta), st["eta"].numpy()) and same_bits(np.array(mu), st["mu"].numpy())
    assert same_bits(ax, st["ax"].numpy()), "ax"
    assert same_bits(p, tp), "param"
