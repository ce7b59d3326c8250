"""The device epilogues' torch-CPU sqrt (fedavg_arith.h sqrt_torch_cpu / sqrt_mkl_rsqrtps; nvflare_amd/torch_sqrt.py)
on the GPU, both restated MKL vsSqrt paths: Intel hosts (AVX-512) and AMD hosts (SSE4.2 / AVX, e.g. this pool's).

* elementwise (fedavg_sqrt_f32), against the oracle's restatements (oracle_sqrt_torch_cpu, pinned against torch CPU
  by tests/test_torch_sqrt.py; oracle_sqrt_mkl_rsqrtps, pinned against MKL's kernel and the box's torch by
  tests/test_torch_sqrt_amd.py) over every mantissa of [1, 4), every subnormal and 1 in 61 of every other binade
  (tools/sqrt_probe.py's set, 59.8 M values) -- and against this host's torch.sqrt for whichever path
  torch_sqrt.detect() finds here;
* inside every epilogue that takes a sqrt (Adam, AdamW + amsgrad, Adagrad, RMSprop centered + momentum, NAdam,
  RAdam), kernel against oracle with the same sqrt, several rounds, bit-exact;
* the three sqrt modes really differ (the mode switch reaches the kernel)."""

import os
import sys

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ctx():
    from nvflare_amd.device import DeviceContext

    return DeviceContext.get(0)


def _probe_set():
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import sqrt_probe

    return sqrt_probe.probe_set().view(np.float32)


def _device_sqrt(ctx, x, torch_sqrt):
    buf = ctx.alloc(x.nbytes)
    out = ctx.alloc(x.nbytes)
    ctx.h2d_ptr(buf.ptr, x.ctypes.data, x.nbytes)
    ctx.sqrt_f32(buf.ptr, out.ptr, x.size, torch_sqrt)
    got = np.empty_like(x)
    ctx.d2h(got, out.ptr)
    buf.close()
    out.close()
    return got


def _same(a, b):
    return np.count_nonzero(~((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))))


def test_device_sqrt_matches_restatement_everywhere(ctx, oracle):
    import torch

    from nvflare_amd import torch_sqrt

    x = _probe_set()
    got = _device_sqrt(ctx, x, 1)
    exp = oracle.sqrt_torch_cpu(x)
    assert _same(got, exp) == 0
    amd = _device_sqrt(ctx, x, 2)
    with np.errstate(invalid="ignore"):
        assert _same(amd, oracle.sqrt_torch_cpu_amd(x)) == 0
    ieee = _device_sqrt(ctx, x, 0)
    with np.errstate(invalid="ignore"):
        assert _same(ieee, np.sqrt(x)) == 0
    assert _same(got, ieee) > 300_000  # the three sqrt modes are different functions
    assert _same(amd, ieee) > 3_000_000 and _same(amd, got) > 3_000_000
    here = torch_sqrt.detect()
    if here in ("torch_cpu", "torch_cpu_amd"):  # this host's torch computes one of them: compare with it too
        with np.errstate(invalid="ignore"):
            assert _same(got if here == "torch_cpu" else amd, torch.from_numpy(x.copy()).sqrt().numpy()) == 0


def test_device_sqrt_specials_every_mode(ctx, oracle):
    """Every positive and negative subnormal, zeros, the top 4096 finite values, inf, NaN and negatives through each
    mode's device sqrt against the oracle (NaN-aware).  Torch returns NaN for a negative subnormal (RMSprop's centered
    ``square_avg - grad_avg**2`` can round to one) where the raw v_sqrt_f32 the Intel-host form once used for its
    specials gave -0: tools/sqrt_device_exhaustive.py found those 8,388,607 inputs over all 2^32."""
    neg_sub = np.uint32(0x80000000) | np.arange(1, 1 << 23, dtype=np.uint32)
    pos_sub = np.arange(0, 1 << 23, dtype=np.uint32)
    top = np.arange(0x7F7FF000, 0x7F800001, dtype=np.uint32)
    misc = np.array([0x80000000, 0xFF800000, 0x7FC00000, 0xFFC00000, 0xBF800000, 0x80800000, 0xC0800000], np.uint32)
    x = np.concatenate([neg_sub, pos_sub, top, misc]).view(np.float32)
    for mode, fn in ((0, np.sqrt), (1, oracle.sqrt_torch_cpu), (2, oracle.sqrt_torch_cpu_amd)):
        with np.errstate(invalid="ignore"):
            assert _same(_device_sqrt(ctx, x, mode), fn(x)) == 0, mode


class _Dev:
    def __init__(self, ctx, rows, n):
        from nvflare_amd.device import TiledLayout

        self.ctx, self.n = ctx, n
        self.lay = TiledLayout(4096, len(rows))
        self.slab = ctx.alloc(self.lay.slab_elems(n) * 4)
        self.bases = [self.slab.ptr + self.lay.slot_offset_elems(k) * 4 for k in range(len(rows))]
        for b, r in zip(self.bases, rows):
            ctx.h2d_tiled(b, 4096 * 4, self.lay.tile_stride * 4, 0, r.ctypes.data, r.nbytes)
        self.n4 = (n + 3) // 4 * 4
        self.bufs = {}

    def buf(self, name, host):
        if name not in self.bufs:
            self.bufs[name] = self.ctx.alloc(self.n4 * 4 + 16)
        self.ctx.h2d_ptr(self.bufs[name].ptr, host.ctypes.data, host.nbytes)
        return self.bufs[name].ptr

    def get(self, name):
        out = np.empty(self.n, np.float32)
        self.ctx.d2h(out, self.bufs[name].ptr)
        return out

    def close(self):
        self.slab.close()
        for b in self.bufs.values():
            b.close()


KINDS = [
    ("adam", dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)),
    ("adamw_amsgrad", dict(lr=1e-3, beta1=0.5, beta2=0.9, eps=1e-8, weight_decay=1e-2, decoupled_weight_decay=1, amsgrad=1)),
    ("adagrad", dict(lr=1e-2, lr_decay=0.05, eps=1e-10, weight_decay=1e-3)),
    ("rmsprop", dict(lr=1e-3, alpha=0.99, eps=1e-8, momentum=0.5, centered=1)),
    ("nadam", dict(lr=2e-3, beta1=0.9, beta2=0.999, eps=1e-8, momentum_decay=4e-3)),
    ("radam", dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)),
]


@pytest.mark.parametrize("sqrt", ["torch_cpu", "torch_cpu_amd"])
@pytest.mark.parametrize("K", [5, 70])
@pytest.mark.parametrize("name,hp", KINDS, ids=[k for k, _ in KINDS])
def test_epilogues_with_torch_cpu_sqrt(ctx, oracle, name, hp, K, sqrt):
    from nvflare_amd import _native as N

    kind = {"adam": oracle.EPI_ADAM, "adamw_amsgrad": oracle.EPI_ADAM, "adagrad": oracle.EPI_ADAGRAD,
            "rmsprop": oracle.EPI_RMSPROP, "nadam": oracle.EPI_NADAM, "radam": oracle.EPI_RADAM}[name]
    rng = np.random.default_rng(31 + K)
    n = 3 * 4096 + 77
    p = rng.standard_normal(n).astype(np.float32)
    m, v, x3 = (np.zeros(n, np.float32) for _ in range(3))
    dev_p = dev_m = dev_v = dev_3 = None
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    count = None
    for w in ws:
        count = w if count is None else count + w
    mp = 1.0
    for step in range(1, 9):  # RAdam crosses into its rectified branch
        rows = [(rng.standard_normal(n) * 0.01 * (1.0 if step % 3 else 0.05)).astype(np.float32) for _ in range(K)]
        d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH)
        dev = _Dev(ctx, rows, n)
        if dev_p is None:
            dev_p, dev_m, dev_v, dev_3 = p.copy(), m.copy(), v.copy(), x3.copy()
        e = N.Epilogue()
        e.kind = kind
        for k_, val in hp.items():
            setattr(e, k_, val)
        e.step, e.mu_product = float(step), mp
        e.torch_sqrt = {"torch_cpu": N.FEDAVG_SQRT_TORCH_AVX512, "torch_cpu_amd": N.FEDAVG_SQRT_TORCH_AMD}[sqrt]
        e.param, e.state1 = dev.buf("p", dev_p), dev.buf("m", dev_m)
        e.state2, e.state3 = dev.buf("v", dev_v), dev.buf("x3", dev_3)
        ctx.accumulate_tiled_epi(dev.bases, ws, 4096, dev.lay.tile_stride, 0, dev.n4, None, N.FEDAVG_OP_TORCH,
                                 N.FEDAVG_FIN_DIV, count, e)
        dev_p, dev_m, dev_v, dev_3 = dev.get("p"), dev.get("m"), dev.get("v"), dev.get("x3")
        dev.close()
        oracle.epilogue_apply(d, kind, p=p, m=m, v=v, vmax=x3, step=float(step), mu_product=mp, torch_cpu_sqrt=sqrt, **hp)
        for nm, a, b in (("p", dev_p, p), ("m", dev_m, m), ("v", dev_v, v), ("x3", dev_3, x3)):
            assert same_bits(a, b), (name, step, nm, int(np.count_nonzero(a.view(np.uint32) != b.view(np.uint32))))
        if kind == oracle.EPI_NADAM:
            mu = hp["beta1"] * (1.0 - 0.5 * (0.96 ** (step * hp["momentum_decay"])))
            mp = float(np.float32(np.float32(mp) * np.float32(mu)))


def test_runtime_rsqrtps_table_on_the_box(ctx, oracle):
    """the RSQRTPS table FEDAVG_SQRT_TORCH_AMD uses is captured on the host at run time
    (fedavg_host_rsqrtps_table) and uploaded per context; on the GPU pool's EPYC 9575F it equals the table captured
    there in round 3 (tests/golden/rsqrtps_amd_epyc9575f.bin), and torch_sqrt.detect() must find the host's path --
    on this pool a silent fall-back to the correctly rounded sqrt would break Adam's 1-ulp parity."""
    from test_cpu_rsqrtps_table import BOX_CPU, cpu_model

    from nvflare_amd import torch_sqrt

    tab = torch_sqrt.host_rsqrtps_table()
    assert np.array_equal(tab, oracle.rsqrtps_table())
    if BOX_CPU in cpu_model():
        assert np.array_equal(tab, oracle.rsqrtps_table_box())
        assert torch_sqrt.detect() == "torch_cpu_amd"
    assert torch_sqrt.detect() != "unmatched", f"torch.sqrt on {cpu_model()!r} matches no restated path"
    # the device reads the uploaded table: a different table gives different roots, the host's gives the host's
    x = (1.0 + np.arange(1 << 16, dtype=np.float32) / (1 << 16)) * np.float32(2.0)
    ctx.load_rsqrtps(tab[::-1].copy())
    other = _device_sqrt(ctx, x, 2)
    ctx.load_rsqrtps(tab)
    mine = _device_sqrt(ctx, x, 2)
    assert _same(mine, oracle.sqrt_torch_cpu_amd(x, tab)) == 0
    assert _same(other, mine) > 1000


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_short_and_ragged_calls_match_the_hosts_torch(ctx, threads):
    """torch.sqrt on short tensors (1..67 elements) and on lengths that leave ragged chunk tails under
    at::parallel_for (grain 32768), at several intra-op thread counts, against the device sqrt in the mode this
    host's torch was detected as -- MKL's short-call and remainder paths, not only its long batches."""
    import torch

    from nvflare_amd import torch_sqrt

    mode = torch_sqrt.detect()
    if mode == "unmatched":
        pytest.fail("this host's torch.sqrt matches no restated path")
    flag = {"torch_cpu": 1, "torch_cpu_amd": 2, "ieee": 0}[mode]
    rng = np.random.default_rng(threads)
    sizes = list(range(1, 68)) + [32767, 32768, 32769, 65536 + 13, 3 * 32768 + 5, 100_003]
    saved = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        for n in sizes:
            x = np.abs(rng.standard_normal(n)).astype(np.float32) * np.float32(10.0) ** rng.integers(-30, 30, n).astype(np.float32)
            want = torch.from_numpy(x.copy()).sqrt().numpy()
            got = _device_sqrt(ctx, x, flag)
            assert _same(got, want) == 0, (n, threads, mode)
    finally:
        torch.set_num_threads(saved)


FROZEN_KINDS = [
    ("adam", dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)),  # (weight decay would make a frozen g non-zero)
    ("adagrad", dict(lr=1e-2, lr_decay=0.05, eps=1e-10)),
    ("rmsprop", dict(lr=1e-3, alpha=0.99, eps=1e-8, momentum=0.5)),
    ("nadam", dict(lr=2e-3, beta1=0.9, beta2=0.999, eps=1e-8, momentum_decay=4e-3)),
    ("radam", dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)),
]


@pytest.mark.parametrize("sqrt", ["ieee", "torch_cpu", "torch_cpu_amd"])
@pytest.mark.parametrize("K", [2, 70])
@pytest.mark.parametrize("name,hp", FROZEN_KINDS, ids=[k for k, _ in FROZEN_KINDS])
def test_frozen_parameters_and_signed_zero_states(ctx, oracle, name, hp, K, sqrt):
    """A frozen region (every client's update exactly 0: the states stay +0, the restated sqrt's and the quotients' +0
    inputs run their fast forms since round 6) beside -0 and subnormal states (still the rare path), through the
    LDS-DMA form (2 clients) and the burst form (70): p and every state bit for bit against the oracle, two steps."""
    from nvflare_amd import _native as N

    kind = {"adam": oracle.EPI_ADAM, "adagrad": oracle.EPI_ADAGRAD, "rmsprop": oracle.EPI_RMSPROP,
            "nadam": oracle.EPI_NADAM, "radam": oracle.EPI_RADAM}[name]
    rng = np.random.default_rng(77 + K)
    n = 6 * 4096 + 36
    frozen = 3 * 4096 + 1000  # tiles 0-2 whole and a piece of tile 3
    p = rng.standard_normal(n).astype(np.float32)
    m = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    v = (rng.random(n) * 1e-6).astype(np.float32)
    m[:frozen] = 0.0
    v[:frozen] = 0.0
    sel = rng.choice(np.arange(frozen, n), 200, replace=False)
    m[sel[:50]] = -0.0
    v[sel[50:100]] = -0.0 if name != "adagrad" else 0.0  # Adagrad's sum: -0 + g*g
    v[sel[100:150]] = np.float32(1e-40)  # subnormal
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    count = None
    for w in ws:
        count = w if count is None else count + w
    flag = {"ieee": N.FEDAVG_SQRT_IEEE, "torch_cpu": N.FEDAVG_SQRT_TORCH_AVX512, "torch_cpu_amd": N.FEDAVG_SQRT_TORCH_AMD}
    if sqrt == "torch_cpu_amd":
        ctx.load_rsqrtps(oracle.rsqrtps_table())
    for step in (1, 2):
        rows = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(K)]
        for r in rows:
            r[:frozen] = 0.0
        d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH)
        dev = _Dev(ctx, rows, n)
        try:
            e = N.Epilogue()
            e.kind = kind
            for k_, val in hp.items():
                setattr(e, k_, val)
            e.step, e.mu_product = float(step), 1.0
            e.torch_sqrt = flag[sqrt]
            e.param, e.state1 = dev.buf("p", p), dev.buf("m", m if name != "adagrad" and name != "rmsprop" else v)
            if name == "rmsprop":
                e.state2 = dev.buf("v", m)
            elif name != "adagrad":
                e.state2 = dev.buf("v", v)
            ctx.accumulate_tiled_epi(dev.bases, ws, 4096, dev.lay.tile_stride, 0, dev.n4, None, N.FEDAVG_OP_TORCH,
                                     N.FEDAVG_FIN_DIV, count, e)
            got = {nm: dev.get(nm) for nm in dev.bufs}
        finally:
            dev.close()
        if name == "adagrad":
            oracle.epilogue_apply(d, kind, p=p, m=v, step=float(step), torch_cpu_sqrt=sqrt, **hp)
            want = {"p": p, "m": v}
        elif name == "rmsprop":  # square_avg in state1, the momentum buffer in state2
            oracle.epilogue_apply(d, kind, p=p, m=v, v=m, step=float(step), torch_cpu_sqrt=sqrt, **hp)
            want = {"p": p, "m": v, "v": m}
        else:
            oracle.epilogue_apply(d, kind, p=p, m=m, v=v, step=float(step), mu_product=1.0, torch_cpu_sqrt=sqrt, **hp)
            want = {"p": p, "m": m, "v": v}
        for nm, w in want.items():
            assert same_bits(got[nm], w), (name, step, nm, int(np.count_nonzero(got[nm].view(np.uint32) !=
                                                                                 w.view(np.uint32))))
