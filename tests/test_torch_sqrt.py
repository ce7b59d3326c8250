"""torch CPU's fp32 sqrt, restated (oracle_sqrt_torch_cpu; the device epilogue's sqrt_torch_cpu) -- CPU tests.

The reference's FedOpt server step runs torch's single-tensor optimizers (nvflare/app_opt/pt/fedopt.py:157-182);
their ``exp_avg_sq.sqrt()`` (torch/optim/adam.py:545) is torch CPU's unary sqrt, which torch 2.10 + MKL computes
with vsSqrt -- one Newton step from the VRSQRT14PS estimate, not the correctly rounded root (tools/sqrt_probe.c).
With the restatement every Adam / AdamW / amsgrad / NAdam / RAdam / Adagrad / RMSprop step is BIT-EXACT against
torch CPU: parameters and every state.  These pins need this host's torch to compute that sqrt (the container the
golden fixtures come from); elsewhere they skip and nvflare_amd.torch_sqrt.detect() says which sqrt it found."""

import numpy as np
import pytest
import torch

from golden_util import same_bits
from nvflare_amd import torch_sqrt

pytestmark = pytest.mark.skipif(torch_sqrt.detect() != "torch_cpu",
                                reason=f"this host's torch sqrt is {torch_sqrt.detect()!r}, not the restated vsSqrt")


def test_table_shape_and_probe_vectors(oracle):
    tab = torch_sqrt.table()
    assert tab.dtype == np.uint16 and tab.size == 65536
    assert same_bits(tab, oracle.sqrt_table())
    v = np.load(torch_sqrt.VECTORS_FILE, allow_pickle=False)
    assert same_bits(oracle.sqrt_torch_cpu(v["x"]), v["torch_cpu"])
    assert same_bits(np.sqrt(v["x"]), v["ieee"])
    assert np.count_nonzero(v["torch_cpu"].view(np.uint32) != v["ieee"].view(np.uint32)) >= 6000


@pytest.mark.parametrize("exp", [-127, -126, -100, -96, -30, 0, 1, 77, 127])
def test_restated_sqrt_every_mantissa(oracle, exp):
    """Every mantissa of one binade (subnormals for -127) -- including the 2^-96 scaling threshold."""
    bits = np.arange(1 << 23, dtype=np.uint32)
    if exp > -127:
        bits = bits | np.uint32((exp + 127) << 23)
    else:
        bits = bits[1:]
    x = bits.view(np.float32)
    got = oracle.sqrt_torch_cpu(x)
    ref = torch.from_numpy(x.copy()).sqrt().numpy()
    assert same_bits(got, ref), int(np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32)))
    if exp in (0, 1):  # the restatement is a different function from the correctly rounded sqrt
        assert np.count_nonzero(ref.view(np.uint32) != np.sqrt(x).view(np.uint32)) > 30_000


def test_restated_sqrt_specials_and_sizes(oracle):
    x = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, -1.0, 1e-45, 3.4028235e38, 1.0, 4.0, 0.25], np.float32)
    got, ref = oracle.sqrt_torch_cpu(x), torch.from_numpy(x.copy()).sqrt().numpy()
    assert same_bits(got, ref)
    rng = np.random.default_rng(5)
    for n in list(range(1, 33)) + [127, 2049, 70_001]:  # vsSqrt's vector tails and torch's 2048-grain chunks
        y = (rng.random(n, dtype=np.float32) * 1e-3).astype(np.float32)
        assert same_bits(oracle.sqrt_torch_cpu(y), torch.from_numpy(y).sqrt().numpy()), n


def _torch_steps(opt_cls, kw, p0, deltas):
    p = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    opt = opt_cls([p], foreach=False, **kw)
    for d in deltas:
        opt.zero_grad()
        p.grad = torch.tensor(-1.0 * d)  # fedopt.py:175
        opt.step()
    return p.detach().numpy().copy(), opt.state[p]


@pytest.mark.parametrize("cls,kw", [
    (torch.optim.Adam, dict(lr=1e-3)),
    (torch.optim.Adam, dict(lr=1e-2, betas=(0.8, 0.99), eps=1e-6)),
    (torch.optim.Adam, dict(lr=1e-3, weight_decay=1e-2)),
    (torch.optim.AdamW, dict(lr=1e-3, weight_decay=1e-2)),
    (torch.optim.Adam, dict(lr=1e-3, betas=(0.3, 0.999))),
    (torch.optim.Adam, dict(lr=1e-3, amsgrad=True)),
    (torch.optim.AdamW, dict(lr=1e-3, weight_decay=1e-2, amsgrad=True)),
    (torch.optim.Adam, dict(lr=1e-3, betas=(0.5, 0.9), amsgrad=True, maximize=True)),
])
def test_adam_bit_exact_vs_torch(oracle, cls, kw):
    rng = np.random.default_rng(11)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    scales = [1.0, 1.0, 0.05, 1.0, 0.01] if kw.get("amsgrad") else [1.0] * 5
    deltas = [(rng.standard_normal(n) * 0.01 * sc).astype(np.float32) for sc in scales]
    tp, st = _torch_steps(cls, kw, p0, deltas)
    b1, b2 = kw.get("betas", (0.9, 0.999))
    p, m, v, vmax = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for s, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p, m=m, v=v, vmax=vmax, lr=kw["lr"], beta1=b1, beta2=b2,
                              eps=kw.get("eps", 1e-8), weight_decay=kw.get("weight_decay", 0.0 if cls is torch.optim.Adam else 1e-2),
                              decoupled_weight_decay=int(cls is torch.optim.AdamW), step=float(s + 1),
                              amsgrad=int(bool(kw.get("amsgrad"))), maximize=int(bool(kw.get("maximize"))),
                              torch_cpu_sqrt=True)
    assert same_bits(p, tp), int(np.count_nonzero(p.view(np.uint32) != tp.view(np.uint32)))
    assert same_bits(m, st["exp_avg"].numpy()) and same_bits(v, st["exp_avg_sq"].numpy())
    if kw.get("amsgrad"):
        assert same_bits(vmax, st["max_exp_avg_sq"].numpy())
    # without the restatement the parameters differ on some elements (torch's sqrt is not the IEEE one)
    p2, m2, v2, vm2 = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for s, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p2, m=m2, v=v2, vmax=vm2, lr=kw["lr"], beta1=b1, beta2=b2,
                              eps=kw.get("eps", 1e-8), weight_decay=kw.get("weight_decay", 0.0 if cls is torch.optim.Adam else 1e-2),
                              decoupled_weight_decay=int(cls is torch.optim.AdamW), step=float(s + 1),
                              amsgrad=int(bool(kw.get("amsgrad"))), maximize=int(bool(kw.get("maximize"))))
    assert not same_bits(p2, tp)


@pytest.mark.parametrize("opt_name,kw", [
    ("NAdam", dict(lr=2e-3)),
    ("NAdam", dict(lr=1e-2, betas=(0.8, 0.95), weight_decay=1e-3, momentum_decay=5e-3)),
    ("NAdam", dict(lr=1e-3, weight_decay=1e-2, decoupled_weight_decay=True, maximize=True)),
    ("RAdam", dict(lr=1e-3)),
    ("RAdam", dict(lr=1e-2, betas=(0.8, 0.9), weight_decay=1e-3)),
    ("RAdam", dict(lr=1e-3, weight_decay=1e-2, decoupled_weight_decay=True, maximize=True)),
])
def test_nadam_radam_bit_exact_vs_torch(oracle, opt_name, kw):
    from test_fedopt_oracle import nadam_mu_product

    rng = np.random.default_rng(12)
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
                              momentum_decay=md, mu_product=float(mp), step=float(k + 1), torch_cpu_sqrt=True)
        mp = nadam_mu_product(mp, b1, md, k + 1)
    assert same_bits(p, tp), int(np.count_nonzero(p.view(np.uint32) != tp.view(np.uint32)))
    assert same_bits(m, st["exp_avg"].numpy()) and same_bits(v, st["exp_avg_sq"].numpy())


@pytest.mark.parametrize("kw", [
    dict(lr=1e-2),
    dict(lr=0.1, lr_decay=0.05, weight_decay=1e-3, eps=1e-8),
    dict(lr=1e-2, initial_accumulator_value=0.1, maximize=True),
])
def test_adagrad_bit_exact_vs_torch(oracle, kw):
    rng = np.random.default_rng(13)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(5)]
    tp, st = _torch_steps(torch.optim.Adagrad, kw, p0, deltas)
    p = p0.copy()
    s = np.full(n, kw.get("initial_accumulator_value", 0.0), np.float32)
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_ADAGRAD, p=p, m=s, lr=kw["lr"], lr_decay=kw.get("lr_decay", 0.0),
                              weight_decay=kw.get("weight_decay", 0.0), eps=kw.get("eps", 1e-10),
                              maximize=int(kw.get("maximize", False)), step=float(k + 1), torch_cpu_sqrt=True)
    assert same_bits(p, tp) and same_bits(s, st["sum"].numpy())


@pytest.mark.parametrize("kw", [
    dict(lr=1e-2),
    dict(lr=1e-2, alpha=0.9, eps=1e-6, momentum=0.9),
    dict(lr=1e-3, centered=True, weight_decay=1e-3),
    dict(lr=1e-3, centered=True, momentum=0.5, maximize=True),
])
def test_rmsprop_bit_exact_vs_torch(oracle, kw):
    rng = np.random.default_rng(14)
    n = 200_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(5)]
    tp, st = _torch_steps(torch.optim.RMSprop, kw, p0, deltas)
    p, sq, buf, ga = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for k, d in enumerate(deltas):
        oracle.epilogue_apply(d, oracle.EPI_RMSPROP, p=p, m=sq, v=buf, vmax=ga, lr=kw["lr"], alpha=kw.get("alpha", 0.99),
                              eps=kw.get("eps", 1e-8), momentum=kw.get("momentum", 0.0),
                              weight_decay=kw.get("weight_decay", 0.0), centered=int(kw.get("centered", False)),
                              maximize=int(kw.get("maximize", False)), step=float(k + 1), torch_cpu_sqrt=True)
    assert same_bits(p, tp)
    assert same_bits(sq, st["square_avg"].numpy())
    if kw.get("momentum"):
        assert same_bits(buf, st["momentum_buffer"].numpy())
    if kw.get("centered"):
        assert same_bits(ga, st["grad_avg"].numpy())
