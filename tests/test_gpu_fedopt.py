"""GPU parity of the fused server-optimizer epilogues (rows a9/a10) against the CPU oracle, bit-exact
(both use IEEE arithmetic; the oracle itself is pinned to torch CPU by tests/test_fedopt_oracle.py)."""

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

TILE = 4096


@pytest.fixture(scope="module")
def ctx():
    from nvflare_amd.device import DeviceContext

    return DeviceContext.get(0)


def _sum(ws):
    c = None
    for w in ws:
        c = w if c is None else c + w
    return c


class _Dev:
    """Slab of K client rows + flat p/m/v/base buffers on the device."""

    def __init__(self, ctx, rows, n):
        from nvflare_amd.device import TiledLayout

        self.ctx = ctx
        self.K = len(rows)
        self.n = n
        self.lay = TiledLayout(TILE, max(self.K, 1))
        self.slab = ctx.alloc(self.lay.slab_elems(n) * 4)
        self.bases = [self.slab.ptr + self.lay.slot_offset_elems(k) * 4 for k in range(self.K)]
        for b, r in zip(self.bases, rows):
            ctx.h2d_tiled(b, TILE * 4, self.lay.tile_stride * 4, 0, r.ctypes.data, r.nbytes)
        self.n4 = (n + 3) // 4 * 4
        self.bufs = {}

    def buf(self, name, host=None):
        if name not in self.bufs:
            self.bufs[name] = self.ctx.alloc(self.n4 * 4 + 16)
        if host is not None:
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


def _epi(kind, **kw):
    from nvflare_amd import _native as N

    e = N.Epilogue()
    e.kind = kind
    for k, v in kw.items():
        setattr(e, k, v)
    return e


@pytest.mark.parametrize("K", [5, 130])
@pytest.mark.parametrize("op,fin,mode", [(1, 2, 1), (0, 1, 0)])
def test_add_base_epilogue(ctx, oracle, K, op, fin, mode):
    rng = np.random.default_rng(K)
    n = 3 * TILE + 100
    rows = [rng.standard_normal(n).astype(np.float32) for _ in range(K)]
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    base = rng.standard_normal(n).astype(np.float32)
    dev = _Dev(ctx, rows, n)
    try:
        out = dev.buf("out", base)  # in place: out aliases base
        e = _epi(2 - 1, base=out)  # FEDAVG_EPI_ADD_BASE
        ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, out, op, fin, _sum(ws), e)
        d = oracle.fedavg_c(rows, ws, mode, fin=fin)
        assert same_bits(dev.get("out"), oracle.epilogue_apply(d, oracle.EPI_ADD_BASE, base=base))
    finally:
        dev.close()


SGD_CASES = [
    dict(lr=1.0),
    dict(lr=0.7, momentum=0.9),
    dict(lr=0.05, momentum=0.6, dampening=0.1),
    dict(lr=0.05, momentum=0.9, nesterov=1),
    dict(lr=0.1, momentum=0.9, weight_decay=1e-2),
    dict(lr=0.3, maximize=1, momentum=0.5),
]


@pytest.mark.parametrize("hp", SGD_CASES)
def test_sgd_epilogue_multi_round(ctx, oracle, hp):
    rng = np.random.default_rng(7)
    n, K = 2 * TILE + 44, 6
    p = rng.standard_normal(n).astype(np.float32)
    buf = np.zeros(n, np.float32)
    ws = [0.5 + k for k in range(K)]
    dev = None
    try:
        for rnd in range(3):
            rows = [(rng.standard_normal(n) * 0.1).astype(np.float32) for _ in range(K)]
            if dev is not None:
                for b, r in zip(dev.bases, rows):
                    ctx.h2d_tiled(b, TILE * 4, dev.lay.tile_stride * 4, 0, r.ctypes.data, r.nbytes)
            else:
                dev = _Dev(ctx, rows, n)
                dev.buf("p", p)
                dev.buf("m", buf)
            e = _epi(2, param=dev.buf("p"), state1=dev.buf("m"), first_step=int(rnd == 0), **hp)
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1, 2, _sum(ws), e)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH)
            oracle.epilogue_apply(d, oracle.EPI_SGD, p=p, m=buf, first_step=int(rnd == 0), **hp)
            assert same_bits(dev.get("p"), p), rnd
            if hp.get("momentum"):
                assert same_bits(dev.get("m"), buf), rnd
    finally:
        dev.close()


def test_sgd_epilogue_many_clients_no_out(ctx, oracle):
    """K > 128 with out=NULL: the chain's partial sum lives in a stream-ordered scratch."""
    rng = np.random.default_rng(11)
    n, K = TILE + 36, 131
    rows = [rng.standard_normal(n).astype(np.float32) for _ in range(K)]
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    p = rng.standard_normal(n).astype(np.float32)
    m = rng.standard_normal(n).astype(np.float32)
    dev = _Dev(ctx, rows, n)
    try:
        e = _epi(2, param=dev.buf("p", p), state1=dev.buf("m", m), lr=0.5, momentum=0.9)
        ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1, 2, _sum(ws), e)
        d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH)
        oracle.epilogue_apply(d, oracle.EPI_SGD, p=p, m=m, lr=0.5, momentum=0.9)
        assert same_bits(dev.get("p"), p)
        assert same_bits(dev.get("m"), m)
    finally:
        dev.close()


ADAM_CASES = [
    dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8),
    dict(lr=1e-2, beta1=0.8, beta2=0.99, eps=1e-6),
    dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2),
    dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, decoupled_weight_decay=1),
    dict(lr=1e-3, beta1=0.3, beta2=0.999, eps=1e-8),
    dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, maximize=1),
]


@pytest.mark.parametrize("hp", ADAM_CASES)
@pytest.mark.parametrize("K", [4, 129])
def test_adam_epilogue_multi_round(ctx, oracle, hp, K):
    rng = np.random.default_rng(11)
    n = 2 * TILE + 8
    p = rng.standard_normal(n).astype(np.float32)
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    ws = [float(1 + k % 7) for k in range(K)]
    dev = None
    try:
        for step in (1, 2, 3):
            rows = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(K)]
            if dev is None:
                dev = _Dev(ctx, rows, n)
                dev.buf("p", p)
                dev.buf("m", m)
                dev.buf("v", v)
            else:
                for b, r in zip(dev.bases, rows):
                    ctx.h2d_tiled(b, TILE * 4, dev.lay.tile_stride * 4, 0, r.ctypes.data, r.nbytes)
            e = _epi(3, param=dev.buf("p"), state1=dev.buf("m"), state2=dev.buf("v"), step=float(step), **hp)
            out = dev.buf("d") if K > 128 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, out, 1, 2, _sum(ws), e)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH)
            oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p, m=m, v=v, step=float(step), **hp)
            assert same_bits(dev.get("m"), m), step
            assert same_bits(dev.get("v"), v), step
            assert same_bits(dev.get("p"), p), step
    finally:
        dev.close()


def test_epilogue_on_precomputed_update(ctx, oracle):
    """k_rows = 0: the epilogue applied to an update already in HBM (the generator path: H2D of the
    aggregated diff, then the optimizer step on device)."""
    rng = np.random.default_rng(5)
    n = TILE + 4
    delta = rng.standard_normal(n).astype(np.float32)
    p = rng.standard_normal(n).astype(np.float32)
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    dev = _Dev(ctx, [], n)
    try:
        dp, dm, dv, dd = dev.buf("p", p), dev.buf("m", m), dev.buf("v", v), dev.buf("delta", delta)
        e = _epi(3, param=dp, state1=dm, state2=dv, step=1.0, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)
        ctx.accumulate_tiled_epi([], [], TILE, TILE, 0, dev.n4, None, 1, 0, 1.0, e, acc_in_ptr=dd)
        oracle.epilogue_apply(delta, oracle.EPI_ADAM, p=p, m=m, v=v, step=1.0, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)
        assert same_bits(dev.get("p"), p) and same_bits(dev.get("m"), m) and same_bits(dev.get("v"), v)
    finally:
        dev.close()


@pytest.mark.parametrize("variant", [0, 4])
@pytest.mark.parametrize("K,kind", [(6, 3), (2, 3), (1, 2), (5, 1), (0, 3)])
def test_epilogue_variants_multi_tile_per_block(ctx, oracle, variant, K, kind):
    """More tiles than blocks (every block walks several tiles), so the software-pipelined variant carries
    client loads across tiles; ragged client groups (K % 4 != 0), K = 1 and K = 0 (acc_in only)."""
    rng = np.random.default_rng(100 + K)
    n = 1100 * TILE + 12
    rows = [rng.standard_normal(n).astype(np.float32) for _ in range(K)]
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    acc0 = rng.standard_normal(n).astype(np.float32) if K == 0 else None
    p = rng.standard_normal(n).astype(np.float32)
    m = (rng.standard_normal(n) * 0.1).astype(np.float32)
    v = (rng.random(n) * 0.01).astype(np.float32)
    base = rng.standard_normal(n).astype(np.float32)
    hp = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, step=3.0) if kind == 3 else dict(lr=0.5, momentum=0.9)
    dev = _Dev(ctx, rows, n)
    ctx.set_variant(variant)
    try:
        if kind == 1:
            out = dev.buf("out")
            e = _epi(1, base=dev.buf("base", base))
        else:
            out = None
            e = _epi(kind, param=dev.buf("p", p), state1=dev.buf("m", m), state2=dev.buf("v", v), **hp)
        acc_ptr = dev.buf("acc", acc0) if K == 0 else None
        fin = 2 if K else 0
        count = _sum(ws) if K else 1.0
        ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, out, 1, fin, count, e,
                                 acc_in_ptr=acc_ptr)
        d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else acc0
        if kind == 1:
            assert same_bits(dev.get("out"), oracle.epilogue_apply(d, oracle.EPI_ADD_BASE, base=base))
        else:
            oracle.epilogue_apply(d, kind, p=p, m=m, v=v, **hp)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("m"), m)
            if kind == 3:
                assert same_bits(dev.get("v"), v)
    finally:
        ctx.set_variant(0)
        dev.close()


@pytest.mark.parametrize("K", [4, 5, 6, 7, 8, 9, 10, 11, 131, 133, 134])
def test_adam_burst_remainders(ctx, oracle, K):
    """The fused burst kernel's client loop (fedavg_arith.h tile_sum_rrem, round 4): groups of four, then the K mod 4
    remainder as one group chosen per tile; every remainder, one and two full groups before it, and chained launches
    (131 / 133 / 134: 128 clients, then 3 / 5 / 6 more on top of the partial sum, ACC_IN); more tiles than one launch
    covers (several launches, a short last one; the chained cases at one launch, 3.3 GB of rows), a ragged end; p, m
    and v bit for bit against the oracle."""
    n = (7000 if K <= 128 else 1500) * TILE + 12345
    cols = np.arange(n, dtype=np.uint64)
    rows = [oracle.synth_values(9, k, cols) for k in range(K)]
    ws = oracle.synth_weights(K)
    rng = np.random.default_rng(K)
    p = rng.standard_normal(n).astype(np.float32)
    m = (rng.standard_normal(n) * 0.1).astype(np.float32)
    v = (rng.random(n) * 0.01).astype(np.float32)
    hp = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, step=2.0)
    dev = _Dev(ctx, rows, n)
    try:
        e = _epi(3, param=dev.buf("p", p), state1=dev.buf("m", m), state2=dev.buf("v", v), **hp)
        out = dev.buf("d") if K > 128 else None
        ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, out, 1, 2, _sum(ws), e)
        d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8)
        oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p, m=m, v=v, **hp)
        assert same_bits(dev.get("p"), p) and same_bits(dev.get("m"), m) and same_bits(dev.get("v"), v)
    finally:
        dev.close()


@pytest.mark.parametrize("K,decoupled", [(7, 0), (3, 1), (0, 0)])
def test_adam_amsgrad_epilogue(ctx, oracle, K, decoupled):
    """Adam / AdamW with amsgrad: max_exp_avg_sq (state3) = torch.maximum(max_exp_avg_sq, exp_avg_sq) and the
    denominator uses it; four steps with shrinking updates so the running max and exp_avg_sq part ways.
    Bit-exact against the oracle (itself pinned to torch CPU by tests/test_fedopt_oracle.py)."""
    rng = np.random.default_rng(40 + K)
    n = 5 * TILE + 12
    p = rng.standard_normal(n).astype(np.float32)
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    vmax = np.zeros(n, np.float32)
    hp = dict(lr=1e-3, beta1=0.5, beta2=0.9, eps=1e-8, weight_decay=1e-2 if decoupled else 0.0,
              decoupled_weight_decay=decoupled)
    dev = None
    try:
        for step, scale in enumerate([1.0, 0.05, 1.0, 0.01]):
            rows = [(rng.standard_normal(n) * scale).astype(np.float32) for _ in range(K)]
            ws = [float(1 + (37 * k) % 100) for k in range(K)]
            delta = (rng.standard_normal(n) * scale).astype(np.float32) if K == 0 else None
            if dev is not None:
                kept = {name: dev.get(name) for name in ("p", "m", "v", "vmax")}
                dev.close()
            dev = _Dev(ctx, rows, n)
            if step == 0:
                kept = {"p": p, "m": m, "v": v, "vmax": vmax}
            ptrs = {name: dev.buf(name, kept[name]) for name in ("p", "m", "v", "vmax")}
            e = _epi(3, param=ptrs["p"], state1=ptrs["m"], state2=ptrs["v"], state3=ptrs["vmax"], amsgrad=1,
                     step=float(step + 1), **hp)
            acc_ptr = dev.buf("acc", delta) if K == 0 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1,
                                     2 if K else 0, _sum(ws) if K else 1.0, e, acc_in_ptr=acc_ptr)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else delta
            oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p, m=m, v=v, vmax=vmax, amsgrad=1, step=float(step + 1), **hp)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("m"), m), step
            assert same_bits(dev.get("v"), v) and same_bits(dev.get("vmax"), vmax), step
        assert np.count_nonzero(vmax != v) > n // 100
    finally:
        if dev is not None:
            dev.close()


@pytest.mark.parametrize("K,hp", [(5, dict(lr=0.1, lr_decay=0.05, eps=1e-10)),
                                  (2, dict(lr=1e-2, weight_decay=1e-3, eps=1e-8, maximize=1)),
                                  (0, dict(lr=0.5, eps=1e-10))])
def test_adagrad_epilogue(ctx, oracle, K, hp):
    """Adagrad (FedAdagrad): state_sum = fma(g, g, sum), p += (-clr * g) / (sqrt(sum) + eps) with
    clr = lr / (1 + (step - 1) * lr_decay); three steps from a non-zero initial sum, bit-exact vs the oracle
    (itself pinned to torch CPU by tests/test_fedopt_oracle.py)."""
    rng = np.random.default_rng(70 + K)
    n = 3 * TILE + 20
    p = rng.standard_normal(n).astype(np.float32)
    s = np.full(n, 0.1, np.float32)
    for step in range(3):
        rows = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        delta = (rng.standard_normal(n) * 0.05).astype(np.float32) if K == 0 else None
        dev = _Dev(ctx, rows, n)
        try:
            e = _epi(4, param=dev.buf("p", p), state1=dev.buf("s", s), step=float(step + 1), **hp)
            acc_ptr = dev.buf("acc", delta) if K == 0 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1,
                                     2 if K else 0, _sum(ws) if K else 1.0, e, acc_in_ptr=acc_ptr)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else delta
            oracle.epilogue_apply(d, oracle.EPI_ADAGRAD, p=p, m=s, step=float(step + 1), **hp)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("s"), s), step
        finally:
            dev.close()


@pytest.mark.parametrize("K,hp", [(5, dict(lr=2e-3, beta1=0.9, beta2=0.999, eps=1e-8)),
                                  (3, dict(lr=1e-2, beta1=0.8, beta2=0.95, eps=1e-6, weight_decay=1e-3, maximize=1)),
                                  (0, dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8))])
def test_adamax_epilogue(ctx, oracle, K, hp):
    """Adamax: exp_avg = lerp(m, g, 1-b1), exp_inf = maximum(u * b2, |g| + eps), p += (-clr * m) / u with
    clr = lr / (1 - b1^step).  Three steps, bit-exact vs the oracle (itself bit-exact vs torch CPU,
    tests/test_fedopt_oracle.py)."""
    rng = np.random.default_rng(110 + K)
    n = 3 * TILE + 36
    p = rng.standard_normal(n).astype(np.float32)
    m, u = np.zeros(n, np.float32), np.zeros(n, np.float32)
    for step in range(3):
        rows = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        delta = (rng.standard_normal(n) * 0.05).astype(np.float32) if K == 0 else None
        dev = _Dev(ctx, rows, n)
        try:
            e = _epi(6, param=dev.buf("p", p), state1=dev.buf("m", m), state2=dev.buf("u", u),
                     step=float(step + 1), **hp)
            acc_ptr = dev.buf("acc", delta) if K == 0 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1,
                                     2 if K else 0, _sum(ws) if K else 1.0, e, acc_in_ptr=acc_ptr)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else delta
            oracle.epilogue_apply(d, oracle.EPI_ADAMAX, p=p, m=m, v=u, step=float(step + 1), **hp)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("m"), m), step
            assert same_bits(dev.get("u"), u), step
        finally:
            dev.close()


@pytest.mark.parametrize("kind,K,hp", [
    (7, 5, dict(lr=2e-3, beta1=0.9, beta2=0.999, eps=1e-8, momentum_decay=4e-3)),
    (7, 3, dict(lr=1e-2, beta1=0.8, beta2=0.95, eps=1e-6, weight_decay=1e-3, momentum_decay=5e-3, maximize=1)),
    (7, 0, dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, decoupled_weight_decay=1,
                momentum_decay=4e-3)),
    (8, 5, dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)),
    (8, 2, dict(lr=1e-2, beta1=0.8, beta2=0.9, eps=1e-8, weight_decay=1e-3, maximize=1)),
    (8, 0, dict(lr=1e-3, beta1=0.9, beta2=0.99, eps=1e-8, weight_decay=1e-2, decoupled_weight_decay=1)),
])
def test_nadam_radam_epilogue(ctx, oracle, kind, K, hp):
    """NAdam (kind 7): denom = sqrt(v / bc2) + eps, two addcdiv_ with the mu / mu_product values; RAdam (kind 8):
    t = exp_avg / bc1 * lr, rectified by (bc2^.5 / (sqrt(v) + eps)) * rect once rho_t > 5.  Seven steps (RAdam
    crosses into the rectified branch), bit-exact vs the oracle (pinned to torch CPU in test_fedopt_oracle)."""
    from test_fedopt_oracle import nadam_mu_product

    rng = np.random.default_rng(130 + 10 * kind + K)
    n = 2 * TILE + 44
    p = rng.standard_normal(n).astype(np.float32)
    m, v = np.zeros(n, np.float32), np.zeros(n, np.float32)
    mp = np.float32(1.0)
    for step in range(7):
        rows = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        delta = (rng.standard_normal(n) * 0.05).astype(np.float32) if K == 0 else None
        dev = _Dev(ctx, rows, n)
        try:
            e = _epi(kind, param=dev.buf("p", p), state1=dev.buf("m", m), state2=dev.buf("v", v),
                     step=float(step + 1), mu_product=float(mp), **hp)
            acc_ptr = dev.buf("acc", delta) if K == 0 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1,
                                     2 if K else 0, _sum(ws) if K else 1.0, e, acc_in_ptr=acc_ptr)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else delta
            oracle.epilogue_apply(d, kind, p=p, m=m, v=v, step=float(step + 1), mu_product=float(mp), **hp)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("m"), m), step
            assert same_bits(dev.get("v"), v), step
        finally:
            dev.close()
        mp = nadam_mu_product(mp, hp["beta1"], hp.get("momentum_decay", 4e-3), step + 1)


@pytest.mark.parametrize("K,hp", [(5, dict(etaminus=0.5, etaplus=1.2, step_size_min=1e-6, step_size_max=50.0)),
                                  (2, dict(etaminus=0.3, etaplus=1.5, step_size_min=1e-3, step_size_max=0.08,
                                           maximize=1)),
                                  (0, dict(etaminus=0.5, etaplus=1.2, step_size_min=1e-6, step_size_max=50.0))])
def test_rprop_epilogue(ctx, oracle, K, hp):
    """Rprop: sign(g * prev) -> etaplus / etaminus / 1 scales the clamped step size, g is zeroed where the sign
    flipped, p = fma(-sign(g), step_size, p), prev = g.  Four steps from step_size = lr, with aggregates that
    flip sign on part of the elements, bit-exact vs the oracle (itself bit-exact vs torch CPU)."""
    rng = np.random.default_rng(150 + K)
    n = 3 * TILE + 52
    p = rng.standard_normal(n).astype(np.float32)
    prev, ss = np.zeros(n, np.float32), np.full(n, 0.01, np.float32)
    for step in range(4):
        rows = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        delta = (rng.standard_normal(n) * 0.05).astype(np.float32) if K == 0 else None
        if delta is not None and step == 2:
            delta[::5] = 0.0
        dev = _Dev(ctx, rows, n)
        try:
            e = _epi(9, param=dev.buf("p", p), state1=dev.buf("prev", prev), state2=dev.buf("ss", ss),
                     step=float(step + 1), **hp)
            acc_ptr = dev.buf("acc", delta) if K == 0 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1,
                                     2 if K else 0, _sum(ws) if K else 1.0, e, acc_in_ptr=acc_ptr)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else delta
            oracle.epilogue_apply(d, oracle.EPI_RPROP, p=p, m=prev, v=ss, step=float(step + 1), **hp)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("prev"), prev), step
            assert same_bits(dev.get("ss"), ss), step
        finally:
            dev.close()
    assert len(np.unique(ss)) > 3  # several step-size histories were exercised


@pytest.mark.parametrize("K,hp", [(5, dict(lambd=1e-4, alpha=0.75, t0=1e6)),
                                  (3, dict(lambd=1e-2, alpha=0.5, t0=1, weight_decay=1e-3, maximize=1)),
                                  (0, dict(lambd=1e-4, alpha=0.75, t0=0))])
def test_asgd_epilogue(ctx, oracle, K, hp):
    """ASGD: p = fma(g, -eta, p * (1 - lambd * eta)); ax = ax + (p - ax) * mu (or p when mu == 1).  Four steps
    with the host eta / mu sequence, bit-exact vs the oracle (itself bit-exact vs torch CPU)."""
    from test_fedopt_oracle import asgd_host_states

    rng = np.random.default_rng(170 + K)
    n = 3 * TILE + 12
    p = rng.standard_normal(n).astype(np.float32)
    ax = np.zeros(n, np.float32)
    lr = 1e-2
    eta, mu = np.float32(lr), np.float32(1.0)
    for step in range(4):
        rows = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        delta = (rng.standard_normal(n) * 0.05).astype(np.float32) if K == 0 else None
        dev = _Dev(ctx, rows, n)
        kw = dict(lambd=hp["lambd"], weight_decay=hp.get("weight_decay", 0.0), maximize=hp.get("maximize", 0))
        try:
            e = _epi(10, param=dev.buf("p", p), state1=dev.buf("ax", ax), eta=float(eta), mu=float(mu),
                     step=float(step + 1), **kw)
            acc_ptr = dev.buf("acc", delta) if K == 0 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1,
                                     2 if K else 0, _sum(ws) if K else 1.0, e, acc_in_ptr=acc_ptr)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else delta
            oracle.epilogue_apply(d, oracle.EPI_ASGD, p=p, m=ax, eta=float(eta), mu=float(mu),
                                  step=float(step + 1), **kw)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("ax"), ax), step
        finally:
            dev.close()
        eta, mu = asgd_host_states(lr, hp["lambd"], hp["alpha"], hp["t0"], step + 1)


@pytest.mark.parametrize("K,hp", [(6, dict(lr=1e-2, alpha=0.99, eps=1e-8)),
                                  (3, dict(lr=1e-2, alpha=0.9, eps=1e-6, momentum=0.9, weight_decay=1e-3)),
                                  (2, dict(lr=1e-3, alpha=0.95, eps=1e-8, centered=1, momentum=0.5, maximize=1)),
                                  (0, dict(lr=1e-3, alpha=0.99, eps=1e-8, centered=1))])
def test_rmsprop_epilogue(ctx, oracle, K, hp):
    """RMSprop: square_avg = fma((1-a) g, g, sq * a); centered grad_avg = lerp(ga, g, 1-a) and
    avg = sqrt(fma(-ga, ga, sq)) + eps; momentum buf = buf * m + g / avg, p = fma(buf, -lr, p), else
    p += (-lr g) / avg.  Three steps, bit-exact vs the oracle (pinned to torch CPU in test_fedopt_oracle)."""
    rng = np.random.default_rng(90 + K)
    n = 3 * TILE + 28
    p = rng.standard_normal(n).astype(np.float32)
    sq, buf, ga = (np.zeros(n, np.float32) for _ in range(3))
    for step in range(3):
        rows = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        delta = (rng.standard_normal(n) * 0.05).astype(np.float32) if K == 0 else None
        dev = _Dev(ctx, rows, n)
        try:
            e = _epi(5, param=dev.buf("p", p), state1=dev.buf("sq", sq), state2=dev.buf("buf", buf),
                     state3=dev.buf("ga", ga), step=float(step + 1), **hp)
            acc_ptr = dev.buf("acc", delta) if K == 0 else None
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, None, 1,
                                     2 if K else 0, _sum(ws) if K else 1.0, e, acc_in_ptr=acc_ptr)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8) if K else delta
            oracle.epilogue_apply(d, oracle.EPI_RMSPROP, p=p, m=sq, v=buf, vmax=ga, step=float(step + 1), **hp)
            assert same_bits(dev.get("p"), p) and same_bits(dev.get("sq"), sq), step
            assert same_bits(dev.get("buf"), buf) and same_bits(dev.get("ga"), ga), step
        finally:
            dev.close()


FEW_CASES = [  # (kind, hp, state names): every optimizer kind through the few-client fused form
    (1, dict(), ()),
    (2, dict(lr=0.5, momentum=0.9, nesterov=1, weight_decay=1e-3, dampening=0.1), ("m",)),
    (3, dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8), ("m", "v")),
    (3, dict(lr=1e-3, beta1=0.5, beta2=0.9, eps=1e-8, amsgrad=1, weight_decay=1e-2, decoupled_weight_decay=1),
     ("m", "v", "vmax")),
    (4, dict(lr=1e-2, weight_decay=1e-3, eps=1e-8, maximize=1), ("m",)),
    (5, dict(lr=1e-3, alpha=0.95, eps=1e-8, centered=1, momentum=0.5, maximize=1), ("m", "v", "vmax")),
    (6, dict(lr=1e-2, beta1=0.8, beta2=0.95, eps=1e-6, weight_decay=1e-3), ("m", "v")),
    (7, dict(lr=2e-3, beta1=0.9, beta2=0.999, eps=1e-8, momentum_decay=4e-3), ("m", "v")),
    (8, dict(lr=1e-2, beta1=0.8, beta2=0.9, eps=1e-8, weight_decay=1e-3), ("m", "v")),
    (9, dict(etaminus=0.5, etaplus=1.2, step_size_min=1e-6, step_size_max=50.0), ("m", "v")),
    (10, dict(lambd=1e-4, eta=1e-2, mu=0.5, weight_decay=1e-3), ("m",)),
]


def _dma_tiles_per_block(kind, K, amd=False, quad=False):
    """Tiles per block per launch of the LDS-DMA form (fedavg_epi.h EpiDmaGeom, N units per wave x W waves / 16): the
    Adam family and Adagrad 8 waves x 16 units at 2 reads, 4 x 32 at 3; Adamax / Rprop 4 x 24; the rest 4 x 40
    (x 32 at 3 reads)."""
    if quad:  # four operand streams (amsgrad, centered RMSprop with momentum): 4 waves x 24 (RMSprop at 3 x 16)
        return 4 if kind == 5 and K == 3 else 6
    if amd and K <= 2 and (kind in (5, 8) or (kind == 4 and K == 2)):  # AMD-host sqrt: 4 waves x 40 at 1-2 reads
        return 10
    if kind in (3, 4, 7, 8):
        return 8
    if kind in (6, 9):
        return 6
    return 8 if K == 3 else 10


@pytest.mark.parametrize("K", [2, 3])
@pytest.mark.parametrize("case", range(len(FEW_CASES)))
def test_few_client_fused_every_kind(ctx, oracle, K, case):
    """2-3 client reads through the fused few-client forms (the LDS-DMA form for ADD_BASE / SGD / Adam without amsgrad or
    an aggregate output, the per-tile form pipelined across tiles for the rest) for every optimizer kind and the Adam family's restated AMD-host sqrt: more tiles than blocks, a ragged end, states
    from a non-zero start, two steps; every output and state bit for bit against the oracle.  ADD_BASE writes out;
    one Adam case also asks for d in out.  (Round 5 also ran these against a register-held burst form of the fused
    kernel, fedavg_tiles_epi_few_f32x4 -- bit-exact, but 53 % of HBM peak against the per-tile form's 69 %, so it
    was dropped: DESIGN.md section 3.4.)"""
    from nvflare_amd import _native as N_

    kind, hp, names = FEW_CASES[case]
    rng = np.random.default_rng(300 + 10 * case + K)
    n = ctx.num_cus * 4 * 2 * TILE + 5 * TILE + 44
    p = rng.standard_normal(n).astype(np.float32)
    st = {"m": (rng.standard_normal(n) * 0.01).astype(np.float32),
          "v": (rng.random(n) * 1e-4 + 1e-6).astype(np.float32),
          "vmax": (rng.random(n) * 1e-4 + 1e-6).astype(np.float32)}
    if kind == 9:  # Rprop: prev gradient, step sizes
        st["v"] = np.full(n, 0.01, np.float32)
    if kind == 4:  # Adagrad: a positive sum
        st["m"] = np.abs(st["m"]) + np.float32(0.1)
    if kind == 5:  # RMSprop centered: square_avg above grad_avg^2
        st["m"] = (rng.random(n) * 1e-2 + 1e-3).astype(np.float32)
        st["vmax"] = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    if kind == 10:  # ASGD: ax
        st["m"] = p.copy()
    base = rng.standard_normal(n).astype(np.float32)
    sq = {"torch_sqrt": 2} if kind in (3, 4, 5, 7, 8) and case != 3 else {}
    for step in (1, 2):
        rows = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        dev = _Dev(ctx, rows, n)
        try:
            ptr = {"p": dev.buf("p", p)}
            for nm in names:
                ptr[nm] = dev.buf(nm, st[nm])
            out = None
            if kind == 1:
                e = _epi(1, base=dev.buf("base", base))
                out = dev.buf("out")
            else:
                kw = dict(param=ptr["p"], step=float(step), **hp)
                for nm, field in zip(names, ("state1", "state2", "state3")):
                    kw[field] = ptr[nm]
                if kind == 3 and case == 2:
                    out = dev.buf("out")
                if sq:
                    ctx.load_rsqrtps(oracle.rsqrtps_table())
                    kw.update(sq)
                e = _epi(kind, **kw)
            n_launch = ctx.launch_count()
            ctx.accumulate_tiled_epi(dev.bases, ws, TILE, dev.lay.tile_stride, 0, dev.n4, out, N_.FEDAVG_OP_TORCH,
                                     N_.FEDAVG_FIN_DIV, _sum(ws), e)
            ctx.sync()
            # Every kind takes the LDS-DMA few-client form (round 6) unless it asks for centered RMSprop without momentum or an aggregate
            # output: one launch per num_cus x tiles-per-block tiles; the rest the per-tile form: one persistent launch
            tiles = (dev.n4 - 1) // TILE + 1
            dma = (not (hp.get("centered") and not hp.get("momentum")) and (out is None or kind == 1)
                   and not (hp.get("amsgrad") and K < 3))
            tpb = _dma_tiles_per_block(kind, K, amd=bool(sq), quad=len(names) == 3)
            assert ctx.launch_count() - n_launch == (-(-tiles // (min(ctx.num_cus, tiles) * tpb)) if dma else 1)
            d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH, nthreads=8)
            if kind == 1:
                assert same_bits(dev.get("out"), oracle.epilogue_apply(d, oracle.EPI_ADD_BASE, base=base)), step
                continue
            if out is not None:
                assert same_bits(dev.get("out"), d), step
            kw = {k: st[nm] for k, nm in zip(("m", "v", "vmax"), names)}
            oracle.epilogue_apply(d, kind, p=p, step=float(step), torch_cpu_sqrt="torch_cpu_amd" if sq else False,
                                  **kw, **hp)
            assert same_bits(dev.get("p"), p), (step, "p")
            for nm in names:
                assert same_bits(dev.get(nm), st[nm]), (step, nm)
        finally:
            dev.close()
