"""GPU parity of the LDS-DMA few-client fused form (round 6, fedavg_epi.h fedavg_tiles_epi_dma_f32x4): 1-3 client reads
with a server-optimizer epilogue -- WEIGHT_DIFF apply (ADD_BASE), SGD (momentum buffer read or not), Adam (every sqrt
the epilogue knows) and the other kinds (RMSprop not centered) -- bit for bit against the oracle AND against the round-5 per-tile form (public variant bit 2, same
process), over the shapes the kernel's indexing has to get right: less than one tile, a range that starts and ends
inside a tile, operand buffers that exist only on [begin, end), more tiles than one launch, ragged last launches.
Reference arithmetic: weighted_aggregation_helper.py:181-236 then app_opt/pt/fedopt.py:157-182 (torch's single-tensor
SGD / Adam), restated by oracle/fedavg_oracle.c."""

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

TILE = 4096
ADAM = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)
ADAM_WD = dict(lr=1e-3, beta1=0.8, beta2=0.99, eps=1e-8, weight_decay=1e-2, decoupled_weight_decay=1)
SGD = dict(lr=0.5, momentum=0.9, nesterov=1, weight_decay=1e-3, dampening=0.1)


@pytest.fixture(scope="module")
def ctx():
    from nvflare_amd.device import DeviceContext

    c = DeviceContext.get(0)
    c.set_variant(0)
    return c


def _sum(ws):
    c = None
    for w in ws:
        c = w if c is None else c + w
    return c


def _epi(kind, **kw):
    from nvflare_amd import _native as N

    e = N.Epilogue()
    e.kind = kind
    for k, v in kw.items():
        setattr(e, k, v)
    return e


class _Case:
    """K client rows over global elements [begin, end) in a tiled slab; operand buffers allocated for exactly [begin, end)
    (the C-ABI indexes them by global element, so the device pointer passed is the buffer minus begin)."""

    def __init__(self, ctx, K, begin, end, seed):
        from nvflare_amd.device import TiledLayout

        self.ctx, self.K, self.begin, self.end = ctx, K, begin, end
        self.n = end - begin
        rng = np.random.default_rng(seed)
        self.rng = rng
        self.lay = TiledLayout(TILE, K)
        self.slab = ctx.alloc(self.lay.slab_elems(end) * 4)
        self.bases = [self.slab.ptr + self.lay.slot_offset_elems(k) * 4 for k in range(K)]
        self.rows = [(rng.standard_normal(end) * 0.05).astype(np.float32) for _ in range(K)]
        for b, r in zip(self.bases, self.rows):
            ctx.h2d_tiled(b, TILE * 4, self.lay.tile_stride * 4, 0, r.ctypes.data, r.nbytes)
        self.ws = [float(1 + (37 * k) % 100) for k in range(K)]
        self.bufs = {}

    def buf(self, name, host):
        """A device buffer holding host (n elements) for [begin, end); returns the global-element-indexed pointer."""
        b = self.bufs.get(name)
        if b is None:
            b = self.bufs[name] = self.ctx.alloc(self.n * 4)
        self.ctx.h2d_ptr(b.ptr, host.ctypes.data, host.nbytes)
        return b.ptr - 4 * self.begin

    def get(self, name):
        out = np.empty(self.n, np.float32)
        self.ctx.d2h(out, self.bufs[name].ptr)
        return out

    def d(self, oracle, op):
        rows = [r[self.begin:self.end] for r in self.rows]
        mode = oracle.MODE_TORCH if op == 1 else oracle.MODE_NUMPY
        return oracle.fedavg_c(rows, self.ws, mode, nthreads=8)

    def close(self):
        self.slab.close()
        for b in self.bufs.values():
            b.close()


def _diff(a, w):
    """Mismatch count and the first few (index, got bits, want bits) for an assertion message."""
    bad = np.flatnonzero((a.view(np.uint32) != w.view(np.uint32)) & ~(np.isnan(a) & np.isnan(w)))
    return int(bad.size), [(int(i), hex(int(a.view(np.uint32)[i])), hex(int(w.view(np.uint32)[i]))) for i in bad[:4]]


def _tiles_per_block(kind, K, rms_momentum=False, amd=False, quad=False):
    """Tiles per block per launch of the product geometry (fedavg_epi.h EpiDmaGeom: N units per wave x W waves / 16):
    Adam / NAdam / RAdam / Adagrad / RMSprop 1 / 2 clients 8 waves x 14 / 16 units, 3 clients 4 waves x 32 (RMSprop
    with momentum 14 / 14 / 24); Adamax / Rprop 4 waves x 24; ADD_BASE / SGD / ASGD 4 waves x 40 (x 32 at 3).  With
    the AMD-host sqrt: RAdam / RMSprop at 1-2 clients and Adagrad at 2 4 waves x 40, NAdam 8 x 16 at every count.
    Four operand streams (amsgrad, centered RMSprop with momentum): 4 waves x 24 (RMSprop at 3 clients x 16)."""
    if quad:
        return 4 if kind == 5 and K == 3 else 6
    if amd and K <= 2 and (kind in (5, 8) or (kind == 4 and K == 2)):
        return 10
    if amd and kind == 7:
        return 8
    if kind == 5 and rms_momentum:
        return {1: 7, 2: 7, 3: 6}[K]
    if kind in (3, 4, 5, 7, 8):
        return {1: 7, 2: 8, 3: 8}[K]
    if kind in (6, 9):
        return 6
    return 8 if K == 3 else 10


def _launches(ctx, begin, end, kind=3, K=2, rms_momentum=False, amd=False, quad=False):
    t_first, t_stop = begin // TILE, (end - 1) // TILE + 1
    per = min(ctx.num_cus, t_stop - t_first) * _tiles_per_block(kind, K, rms_momentum, amd, quad)  # one block per CU
    return -(-(t_stop - t_first) // per)


def _run(ctx, c, e, op, fin, out_ptr=None, variant=0):
    ctx.set_variant(variant)
    try:
        n0 = ctx.launch_count()
        ctx.accumulate_tiled_epi(c.bases, c.ws, TILE, c.lay.tile_stride, c.begin, c.end, out_ptr, op, fin,
                                 _sum(c.ws), e)
        ctx.sync()
        return ctx.launch_count() - n0
    finally:
        ctx.set_variant(0)


def _ranges(ctx):
    big = ctx.num_cus * 4 * TILE  # one launch's tiles
    return [
        (0, 8),  # two float4 columns of one tile
        (0, TILE),
        (3 * TILE + 100, 3 * TILE + 100 + 2 * TILE + 36),  # starts and ends inside tiles
        (TILE - 4, TILE + 4),  # straddles one tile boundary by a column each side
        (0, 2 * big + 5 * TILE + 44),  # three launches, the last one ragged
        (7 * TILE + 1024, 7 * TILE + 1024 + big + 12),
    ]


@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("rng_ix", range(6))
@pytest.mark.parametrize("sqrt", ["ieee", "torch_cpu_amd", "torch_cpu"])
def test_dma_adam_matches_oracle_and_per_tile(ctx, oracle, K, rng_ix, sqrt):
    from nvflare_amd import _native as N

    if sqrt != "torch_cpu_amd" and rng_ix not in (2, 4):
        pytest.skip("the other sqrt paths on two of the ranges")
    begin, end = _ranges(ctx)[rng_ix]
    c = _Case(ctx, K, begin, end, seed=1000 + 10 * rng_ix + K)
    try:
        n = c.n
        p = c.rng.standard_normal(n).astype(np.float32)
        m = (c.rng.standard_normal(n) * 0.01).astype(np.float32)
        v = (c.rng.random(n) * 1e-4 + 1e-6).astype(np.float32)
        flag = {"ieee": N.FEDAVG_SQRT_IEEE, "torch_cpu": N.FEDAVG_SQRT_TORCH_AVX512,
                "torch_cpu_amd": N.FEDAVG_SQRT_TORCH_AMD}[sqrt]
        if sqrt == "torch_cpu_amd":
            ctx.load_rsqrtps(oracle.rsqrtps_table())
        got = {}
        for variant in (0, 4):  # the LDS-DMA form, then the per-tile form on the same inputs
            hp = ADAM if rng_ix % 2 == 0 else ADAM_WD
            e = _epi(3, param=c.buf("p", p), state1=c.buf("m", m), state2=c.buf("v", v), step=3.0, torch_sqrt=flag, **hp)
            nl = _run(ctx, c, e, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, variant=variant)
            if variant == 0:
                assert nl == _launches(ctx, begin, end, 3, K)
            got[variant] = [c.get(x) for x in ("p", "m", "v")]
        pw, mw, vw = p.copy(), m.copy(), v.copy()
        oracle.epilogue_apply(c.d(oracle, 1), oracle.EPI_ADAM, p=pw, m=mw, v=vw, step=3.0, torch_cpu_sqrt=sqrt,
                              **(ADAM if rng_ix % 2 == 0 else ADAM_WD))
        for a, b, w, nm in zip(got[0], got[4], (pw, mw, vw), "pmv"):
            assert same_bits(a, w) and same_bits(b, w), (nm, _diff(a, w), _diff(b, w))
    finally:
        c.close()


@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("rng_ix", [0, 2, 4, 5])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_dma_sgd_two_steps(ctx, oracle, K, rng_ix, momentum):
    """SGD as the FedOpt generator's default (momentum 0.6-0.9): step 1 reads only p (the momentum buffer starts as g),
    step 2 reads p and the buffer -- both operand counts of the form; without momentum only p."""
    from nvflare_amd import _native as N

    begin, end = _ranges(ctx)[rng_ix]
    c = _Case(ctx, K, begin, end, seed=2000 + 10 * rng_ix + K)
    hp = dict(SGD, momentum=momentum)
    try:
        p = c.rng.standard_normal(c.n).astype(np.float32)
        buf = np.zeros(c.n, np.float32)
        pp, pb = c.buf("p", p), c.buf("m", buf)
        for step in (1, 2):
            e = _epi(2, param=pp, state1=pb, first_step=int(step == 1), **hp)
            nl = _run(ctx, c, e, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV)
            assert nl == _launches(ctx, begin, end, 2, K)
            oracle.epilogue_apply(c.d(oracle, 1), oracle.EPI_SGD, p=p, m=buf, first_step=int(step == 1), **hp)
            assert same_bits(c.get("p"), p), step
            if momentum:
                assert same_bits(c.get("m"), buf), step
    finally:
        c.close()


@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("rng_ix", [1, 2, 3, 4])
@pytest.mark.parametrize("op,fin", [(1, 2), (0, 1)])
def test_dma_add_base(ctx, oracle, K, rng_ix, op, fin):
    """WEIGHT_DIFF apply (full_model_shareable_generator.py:58-67): w = base + d into out, numpy and torch modes."""
    begin, end = _ranges(ctx)[rng_ix]
    c = _Case(ctx, K, begin, end, seed=3000 + 10 * rng_ix + K)
    try:
        base = c.rng.standard_normal(c.n).astype(np.float32)
        e = _epi(1, base=c.buf("base", base))
        outp = c.buf("out", np.zeros(c.n, np.float32))
        nl = _run(ctx, c, e, op, fin, out_ptr=outp)
        assert nl == _launches(ctx, begin, end, 1, K)
        want = oracle.epilogue_apply(c.d(oracle, op), oracle.EPI_ADD_BASE, base=base)
        assert same_bits(c.get("out"), want)
        assert same_bits(c.get("base"), base)  # the base is an input only
    finally:
        c.close()


OTHER_KINDS = [  # (kind, hyper-parameters, state names, restated AMD-host sqrt)
    (4, dict(lr=1e-2, weight_decay=1e-3, eps=1e-8, maximize=1), ("m",), True),  # Adagrad
    (5, dict(lr=1e-3, alpha=0.95, eps=1e-8, weight_decay=1e-3), ("m",), True),  # RMSprop: square_avg
    (5, dict(lr=1e-3, alpha=0.9, eps=1e-6, momentum=0.5, maximize=1), ("m", "v"), False),  # + momentum buffer
    (5, dict(lr=1e-3, alpha=0.95, eps=1e-8, momentum=0.5, centered=1), ("m", "v", "x"), True),  # + grad_avg
    (3, dict(lr=1e-3, beta1=0.5, beta2=0.9, eps=1e-8, amsgrad=1, weight_decay=1e-2, decoupled_weight_decay=1),
     ("m", "v", "x"), True),  # AdamW with amsgrad: max_exp_avg_sq
    (6, dict(lr=1e-2, beta1=0.8, beta2=0.95, eps=1e-6, weight_decay=1e-3), ("m", "v"), False),  # Adamax
    (7, dict(lr=2e-3, beta1=0.9, beta2=0.999, eps=1e-8, momentum_decay=4e-3), ("m", "v"), True),  # NAdam
    (8, dict(lr=1e-2, beta1=0.8, beta2=0.9, eps=1e-8, weight_decay=1e-3), ("m", "v"), True),  # RAdam
    (9, dict(etaminus=0.5, etaplus=1.2, step_size_min=1e-6, step_size_max=50.0), ("m", "v"), False),  # Rprop
    (10, dict(lambd=1e-4, eta=1e-2, mu=0.5, weight_decay=1e-3), ("m",), False),  # ASGD
]


@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("rng_ix", [2, 4])
@pytest.mark.parametrize("case", range(len(OTHER_KINDS)))
def test_dma_other_kinds(ctx, oracle, K, rng_ix, case):
    """The rest of the server optimizers on the LDS-DMA form (RMSprop not centered: with its momentum buffer or
    without): two steps from non-zero states (RAdam's second on its rectified branch), every output and state bit for
    bit against the oracle and against the per-tile form (public variant bit 2) on the same inputs."""
    from nvflare_amd import _native as N

    kind, hp, names, amd_sqrt = OTHER_KINDS[case]
    begin, end = _ranges(ctx)[rng_ix]
    c = _Case(ctx, K, begin, end, seed=4000 + 100 * case + 10 * rng_ix + K)
    try:
        n = c.n
        p = c.rng.standard_normal(n).astype(np.float32)
        st = {"m": (c.rng.standard_normal(n) * 0.01).astype(np.float32),
              "v": (c.rng.random(n) * 1e-4 + 1e-6).astype(np.float32)}
        if kind == 4:  # Adagrad: a positive sum
            st["m"] = np.abs(st["m"]) + np.float32(0.1)
        st["x"] = (c.rng.random(n) * 1e-4 + 1e-6).astype(np.float32)  # Adam's max_exp_avg_sq
        if kind == 5:  # RMSprop: square_avg, the momentum buffer, grad_avg (square_avg above grad_avg^2)
            st["m"], st["v"] = (c.rng.random(n) * 1e-2 + 1e-3).astype(np.float32), st["m"]
            st["x"] = (c.rng.standard_normal(n) * 1e-3).astype(np.float32)
        if kind == 9:  # Rprop: step sizes
            st["v"] = np.full(n, 0.01, np.float32)
        if kind == 10:  # ASGD: ax
            st["m"] = p.copy()
        if amd_sqrt:
            ctx.load_rsqrtps(oracle.rsqrtps_table())
        sq = dict(torch_sqrt=N.FEDAVG_SQRT_TORCH_AMD) if amd_sqrt else {}
        for step in (2.0, 10.0):
            got = {}
            for variant in (0, 4):  # the LDS-DMA form, then the per-tile form from the same states
                kw = dict(param=c.buf("p", p), step=step, **hp, **sq)
                for nm, field in zip(names, ("state1", "state2", "state3")):
                    kw[field] = c.buf(nm, st[nm])
                nl = _run(ctx, c, _epi(kind, **kw), N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, variant=variant)
                if variant == 0 and kind == 3 and K < 3:  # amsgrad under 3 reads: the per-tile form (epi_dma_nin)
                    assert nl == 1
                elif variant == 0:
                    assert nl == _launches(ctx, begin, end, kind, K, rms_momentum=len(names) == 2, amd=amd_sqrt,
                                           quad=len(names) == 3)
                got[variant] = [c.get(x) for x in ("p",) + names]
            kw = {k: st[nm] for k, nm in zip(("m", "v", "vmax"), names)}
            oracle.epilogue_apply(c.d(oracle, 1), kind, p=p, step=step,
                                  torch_cpu_sqrt="torch_cpu_amd" if amd_sqrt else False, **kw, **hp)
            for a, b, w, nm in zip(got[0], got[4], [p] + [st[x] for x in names], ("p",) + names):
                assert same_bits(a, w) and same_bits(b, w), (step, nm)
    finally:
        c.close()


def test_dma_route_leaves_others_on_the_per_tile_form(ctx, oracle):
    """A requested aggregate output, centered RMSprop without momentum (its grad_avg would be the third operand
    stream, where the form reads state2) and amsgrad under 3 reads (the per-tile form measured faster, s26) keep their
    round-5 route: one persistent per-tile launch.  (amsgrad at 3 reads and centered RMSprop with momentum -- four
    operand streams -- run the LDS-DMA form since round 6: test_dma_other_kinds.)"""
    from nvflare_amd import _native as N

    c = _Case(ctx, 2, 0, 3 * TILE + 8, seed=7)
    try:
        z = np.zeros(c.n, np.float32)
        e = _epi(3, param=c.buf("p", z + 1), state1=c.buf("m", z), state2=c.buf("v", z), step=1.0, **ADAM)
        assert _run(ctx, c, e, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, out_ptr=c.buf("d", z)) == 1
        want = c.d(oracle, 1)
        assert same_bits(c.get("d"), want)
        e = _epi(5, param=c.buf("p", z + 1), state1=c.buf("m", z + 1e-3), state3=c.buf("x", z),
                 lr=1e-3, alpha=0.9, eps=1e-8, centered=1)
        assert _run(ctx, c, e, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV) == 1
        e = _epi(3, param=c.buf("p", z + 1), state1=c.buf("m", z), state2=c.buf("v", z), state3=c.buf("x", z),
                 amsgrad=1, step=1.0, **ADAM)
        assert _run(ctx, c, e, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV) == 1  # amsgrad at 2 reads: the per-tile form
    finally:
        c.close()


def test_ab_probe_keeps_the_variant(ctx):
    """DeviceContext.ab_build() probes the library with variant bit 5 and restores the variant the context had (ADVICE
    r05: it used to reset it to 0): with public bit 2 set, the 2-client fused Adam call still takes the per-tile form."""
    from nvflare_amd import _native as N

    c = _Case(ctx, 2, 0, 5 * ctx.num_cus * 4 * TILE, seed=9)
    try:
        z = np.zeros(c.n, np.float32)
        e = _epi(3, param=c.buf("p", z + 1), state1=c.buf("m", z), state2=c.buf("v", z), step=1.0, **ADAM)
        ctx.set_variant(4)
        ctx.ab_build()
        n0 = ctx.launch_count()
        ctx.accumulate_tiled_epi(c.bases, c.ws, TILE, c.lay.tile_stride, c.begin, c.end, None, N.FEDAVG_OP_TORCH,
                                 N.FEDAVG_FIN_DIV, _sum(c.ws), e)
        ctx.sync()
        assert ctx.launch_count() - n0 == 1  # the per-tile form, not the LDS-DMA form's 3 launches
    finally:
        ctx.set_variant(0)
        c.close()
