"""torch CPU's fp32 sqrt on the GPU pool's AMD hosts, restated (oracle_sqrt_mkl_rsqrtps; the device epilogue's
sqrt_mkl_rsqrtps) -- CPU tests.

On AMD EPYC (the GPU box host) MKL runs vsSqrt's SSE4.2 / AVX kernels (mkl_vml_kernel_sSqrt_EXHAynn / _H8HAynn): on
the box torch.sqrt equalled them on all 59.8 M probe inputs (profiles/r03/s12/sqrt_box_kernels.json).  They start a
coupled Newton step in plain fp32 from the RSQRTPS estimate, which differs between CPU vendors.  The pins:

* the kernels ship inside the libtorch_cpu this torch loads, so they run HERE too: the restatement with THIS CPU's
  RSQRTPS (captured by tools/rsqrtps_dump.c at test time) equals MKL's EX kernel on every mantissa of several
  binades and a stride-61 sample of all 2^32 inputs (tools/sqrt_mkl_sse_check.py ran all 2^32: 0 mismatches);
* the SSE2 kernel (E2HA) shares the refinement with an IEEE-only estimate: oracle_sqrt_mkl_sse2 equals it too;
* with the AMD host's table (tests/golden/rsqrtps_amd_epyc9575f.bin, captured on the box) the restatement reproduces the
  box's own torch.sqrt: tests/golden/sqrt_amd_box.npz (100,000 inputs of [1, 4); all 2^24 matched offline);
* whole torch optimizer runs with torch's sqrt swapped for MKL's EX kernel run here equal the oracle's
  "torch_cpu_amd" epilogues given this CPU's table: single-tensor Adam / AdamW / amsgrad / NAdam / RAdam / Adagrad /
  RMSprop, parameters and state bit for bit."""

import ctypes
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest
import torch

from golden_util import same_bits
from nvflare_amd import torch_sqrt


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "sqrt_amd_box.npz")


def _kernel(name):
    try:
        lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_cpu.so"))
        fn = getattr(lib, name)
    except (OSError, AttributeError):
        return None
    fn.restype = None
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return fn


E2, EX = _kernel("mkl_vml_kernel_sSqrt_E2HAynn"), _kernel("mkl_vml_kernel_sSqrt_EXHAynn")
pytestmark = pytest.mark.skipif(E2 is None or EX is None, reason="this torch build has no MKL SSE vsSqrt kernels")


def _run(kernel, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    for i in range(0, x.size, 1 << 30):
        n = min(1 << 30, x.size - i)
        kernel(n, x[i:].ctypes.data, out[i:].ctypes.data)
    return out


def mkl_sse2(x):
    return _run(E2, x)


def mkl_ex(x):
    return _run(EX, x)


@pytest.fixture(scope="module")
def here_rsqrtps(tmp_path_factory):
    """THIS CPU's RSQRTPS table (tools/rsqrtps_dump.c, tools/make_rsqrtps_table.py)."""
    if shutil.which("gcc") is None:
        pytest.skip("gcc is absent")
    d = tmp_path_factory.mktemp("rsqrtps")
    exe = str(d / "rsqrtps_dump")
    subprocess.run(["gcc", "-O2", "-msse2", os.path.join(ROOT, "tools", "rsqrtps_dump.c"), "-o", exe], check=True)
    subprocess.run([exe, str(d / "rsq.bin"), str(d / "rcp.bin")], check=True, capture_output=True)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_rsqrtps_table

    return make_rsqrtps_table.table_from_dump(str(d / "rsq.bin"))


def _same_nan(a, b):
    return np.count_nonzero(~((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))))


@pytest.mark.parametrize("exp", [-127, -126, -100, -96, -30, -20, 0, 1, 77, 126, 127])
def test_every_mantissa_of_a_binade(oracle, here_rsqrtps, exp):
    bits = np.arange(1 << 23, dtype=np.uint32)
    bits = bits | np.uint32((exp + 127) << 23) if exp > -127 else bits
    x = bits.view(np.float32)
    got, ref = oracle.sqrt_torch_cpu_amd(x, here_rsqrtps), mkl_ex(x)
    assert same_bits(got, ref), int(np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32)))
    got2, ref2 = oracle.sqrt_torch_cpu_sse2(x), mkl_sse2(x)
    assert same_bits(got2, ref2), int(np.count_nonzero(got2.view(np.uint32) != ref2.view(np.uint32)))
    if exp in (0, 1):  # a different function from the correctly rounded sqrt and from the AVX-512 path
        amd = oracle.sqrt_torch_cpu_amd(x, oracle.rsqrtps_table_box())
        assert np.count_nonzero(amd.view(np.uint32) != np.sqrt(x).view(np.uint32)) > 500_000
        assert np.count_nonzero(amd.view(np.uint32) != oracle.sqrt_torch_cpu(x).view(np.uint32)) > 500_000


def test_all_bit_patterns_sampled(oracle, here_rsqrtps):
    bits = np.arange(0, 1 << 32, 61, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    with np.errstate(invalid="ignore"):
        assert _same_nan(oracle.sqrt_torch_cpu_amd(x, here_rsqrtps), mkl_ex(x)) == 0
        assert _same_nan(oracle.sqrt_torch_cpu_sse2(x), mkl_sse2(x)) == 0


def test_specials_and_callout_edges(oracle, here_rsqrtps):
    edge = np.array([0, 0x80000000, 1, 0x007FFFFF, 0x00800000, 0x7F7FF000, 0x7F7FF001, 0x7F7FFFFF, 0x7F800000,
                     0xFF800000, 0x7FC00000, 0xBF800000, 0x3F800000, 0x40800000, 0x3E800000], np.uint32)
    x = edge.view(np.float32)
    with np.errstate(invalid="ignore"):
        assert _same_nan(oracle.sqrt_torch_cpu_amd(x, here_rsqrtps), mkl_ex(x)) == 0
        assert _same_nan(oracle.sqrt_torch_cpu_amd(x), mkl_ex(x)) == 0  # the callout does not depend on the table


def test_amd_table_reproduces_the_box_torch(oracle):
    g = np.load(GOLDEN, allow_pickle=False)
    got = oracle.sqrt_torch_cpu_amd(g["x"].view(np.float32), oracle.rsqrtps_table_box()).view(np.uint32)
    assert np.array_equal(got, g["torch_sqrt"]), int(np.count_nonzero(got != g["torch_sqrt"]))
    cr = np.sqrt(g["x"].view(np.float32)).view(np.uint32)
    assert np.count_nonzero(cr != g["torch_sqrt"]) > 10_000  # the box's sqrt is not the correctly rounded one


def test_probe_vectors_and_detection(oracle):
    v = np.load(torch_sqrt.VECTORS_FILE, allow_pickle=False)
    assert same_bits(oracle.sqrt_torch_cpu_amd(v["x"], oracle.rsqrtps_table_box()), v["torch_cpu_amd"])
    for other in ("torch_cpu", "ieee"):  # each mode is told apart from the others by thousands of probe values
        assert np.count_nonzero(v["torch_cpu_amd"].view(np.uint32) != v[other].view(np.uint32)) >= 3000
    assert torch_sqrt.detect() in torch_sqrt.MODES + ("unmatched",)
    assert torch_sqrt.epilogue_flag("torch_cpu_amd") == 2 and torch_sqrt.epilogue_flag("torch_cpu") == 1
    assert torch_sqrt.epilogue_flag("ieee") == 0


def test_detection_selects_the_sse_path_with_this_cpus_table(oracle):
    """MKL's SSE4.2 / AVX kernel run HERE (this CPU's RSQRTPS, not the box's: 4000+ of the 8192
    estimates differ on an Intel host) is identified as "torch_cpu_amd" through the run-time table; with the box's
    fixture table that identification would fail, and the correctly rounded sqrt is still told apart."""
    from nvflare_amd import torch_sqrt as ts

    assert ts.detect(host_sqrt=mkl_ex) == "torch_cpu_amd"
    assert ts.detect(host_sqrt=np.sqrt) == "ieee"
    x = np.load(ts.VECTORS_FILE, allow_pickle=False)["x"]
    here, box = ts.host_rsqrtps_table(), oracle.rsqrtps_table_box()
    if not np.array_equal(here, box):
        assert not np.array_equal(mkl_ex(x).view(np.uint32), ts.sqrt_sse_restated(x, box).view(np.uint32))


@pytest.fixture
def ex_torch(monkeypatch):
    """torch's CPU sqrt replaced by MKL's EX kernel run here (what torch computes on the AMD host, with this CPU's
    RSQRTPS)."""

    def sq(t, *a, **k):
        return torch.from_numpy(mkl_ex(t.detach().contiguous().numpy()).reshape(t.shape))

    def sq_(t):
        t.copy_(sq(t))
        return t

    monkeypatch.setattr(torch.Tensor, "sqrt", sq)
    monkeypatch.setattr(torch.Tensor, "sqrt_", sq_)
    monkeypatch.setattr(torch, "sqrt", sq)


def _torch_steps(opt_cls, kw, p0, deltas):
    p = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    opt = opt_cls([p], foreach=False, **kw)
    for d in deltas:
        opt.zero_grad()
        p.grad = torch.tensor(-1.0 * d)  # fedopt.py:175
        opt.step()
    return p.detach().numpy().copy(), opt.state[p]


@pytest.mark.parametrize("name,kw", [
    ("Adam", dict(lr=1e-3)),
    ("Adam", dict(lr=1e-3, amsgrad=True)),
    ("AdamW", dict(lr=1e-3, weight_decay=1e-2)),
    ("NAdam", dict(lr=2e-3)),
    ("RAdam", dict(lr=1e-3)),
    ("Adagrad", dict(lr=0.1, lr_decay=0.05, eps=1e-8)),
    ("RMSprop", dict(lr=1e-3, centered=True, momentum=0.5)),
])
def test_optimizer_steps_bit_exact_with_amd_path_sqrt(oracle, ex_torch, here_rsqrtps, name, kw):
    from test_fedopt_oracle import nadam_mu_product

    rng = np.random.default_rng(21)
    n = 100_003
    p0 = rng.standard_normal(n).astype(np.float32)
    deltas = [(rng.standard_normal(n) * 0.01 * (0.05 if k == 2 else 1.0)).astype(np.float32) for k in range(7)]
    tp, st = _torch_steps(getattr(torch.optim, name), kw, p0, deltas)
    p, m, v, x3 = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    b1, b2 = kw.get("betas", (0.9, 0.999))
    mp = np.float32(1.0)
    for k, d in enumerate(deltas):
        common = dict(step=float(k + 1), torch_cpu_sqrt="torch_cpu_amd", rsqrtps=here_rsqrtps, lr=kw["lr"])
        if name in ("Adam", "AdamW"):
            oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p, m=m, v=v, vmax=x3, beta1=b1, beta2=b2, eps=1e-8,
                                  weight_decay=kw.get("weight_decay", 0.0), decoupled_weight_decay=int(name == "AdamW"),
                                  amsgrad=int(bool(kw.get("amsgrad"))), **common)
        elif name in ("NAdam", "RAdam"):
            oracle.epilogue_apply(d, oracle.EPI_NADAM if name == "NAdam" else oracle.EPI_RADAM, p=p, m=m, v=v,
                                  beta1=b1, beta2=b2, eps=1e-8, momentum_decay=4e-3, mu_product=float(mp), **common)
            mp = nadam_mu_product(mp, b1, 4e-3, k + 1)
        elif name == "Adagrad":
            oracle.epilogue_apply(d, oracle.EPI_ADAGRAD, p=p, m=m, lr_decay=kw["lr_decay"], eps=kw["eps"], **common)
        else:
            oracle.epilogue_apply(d, oracle.EPI_RMSPROP, p=p, m=m, v=v, vmax=x3, alpha=0.99, eps=1e-8,
                                  momentum=kw["momentum"], centered=1, **common)
    assert same_bits(p, tp), int(np.count_nonzero(p.view(np.uint32) != tp.view(np.uint32)))
    state = {"Adagrad": "sum", "RMSprop": "square_avg"}.get(name, "exp_avg")
    assert same_bits(m, st[state].numpy())
    # with the other sqrt modes the same run differs (the swap reached torch's optimizer)
    p2, m2, v2, x32 = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    if name in ("Adam", "AdamW"):
        for k, d in enumerate(deltas):
            oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p2, m=m2, v=v2, vmax=x32, beta1=b1, beta2=b2, eps=1e-8,
                                  weight_decay=kw.get("weight_decay", 0.0), decoupled_weight_decay=int(name == "AdamW"),
                                  amsgrad=int(bool(kw.get("amsgrad"))), step=float(k + 1), lr=kw["lr"],
                                  torch_cpu_sqrt="ieee")
        assert not same_bits(p2, tp)
