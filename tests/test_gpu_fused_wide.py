"""The fused burst kernel's launch forms at one block per CU (64+ clients), bit-exact against the oracle over
more tiles than one launch holds (two launches, the second partial, ragged end): the default form for Adam (round 6:
the split epilogue, fedavg_tiles_epi_split_f32x4 -- 4 register- + 9 LDS-held tiles per block, waves 4-7 joining the
epilogue), round 5's burst form (variant bit 15; 8 register- + 9 LDS-held tiles, round 3), the 4-LDS-tile form (variant
bit 6) and the register-only form (bit 5; A/B builds),
with the correctly rounded and both restated torch-CPU sqrts (each stages its table in the same LDS: the Intel
hosts' 512-byte segments, the AMD hosts' 16 KiB RSQRTPS table -- 160 KiB in all at one block per CU).  64 and 70 clients read 4 distinct uploaded rows cyclically (the kernel sees 64 / 70 row pointers; the
oracle the same list), which keeps the host side small at 18 M elements per row."""

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

TILE = 4096
N = 4400 * TILE + 12  # > 256 blocks x 17 tiles: two launches of the default form at one block per CU


@pytest.fixture(scope="module")
def ctx():
    from nvflare_amd.device import DeviceContext

    return DeviceContext.get(0)


@pytest.fixture(scope="module")
def rows():
    rng = np.random.default_rng(4242)
    return [(rng.standard_normal(N, dtype=np.float32) * 0.01).astype(np.float32) for _ in range(4)]


@pytest.mark.parametrize("torch_sqrt", [0, 1, 2])
@pytest.mark.parametrize("variant", [0, 1 << 15, 64, 32])
@pytest.mark.parametrize("K", [64, 70])
def test_fused_adam_launch_forms(ctx, oracle, rows, K, variant, torch_sqrt):
    from nvflare_amd import _native as N_
    from nvflare_amd.device import TiledLayout

    if variant == 32 and not ctx.ab_build():
        pytest.skip("the register-only form is an A/B form (tools/build_rev_lib.py)")
    lay = TiledLayout(TILE, len(rows))
    n4 = (N + 3) // 4 * 4
    slab = ctx.alloc(lay.slab_elems(N) * 4)
    bufs = [ctx.alloc(n4 * 4 + 16) for _ in range(3)]
    rng = np.random.default_rng(K + variant + torch_sqrt)
    p = rng.standard_normal(N).astype(np.float32)
    m = (rng.standard_normal(N) * 0.01).astype(np.float32)
    v = (rng.random(N) * 1e-4).astype(np.float32)
    try:
        slots = [slab.ptr + lay.slot_offset_elems(j) * 4 for j in range(len(rows))]
        for b, r in zip(slots, rows):
            ctx.h2d_tiled(b, TILE * 4, lay.tile_stride * 4, 0, r.ctypes.data, r.nbytes)
        for b, h in zip(bufs, (p, m, v)):
            ctx.h2d_ptr(b.ptr, h.ctypes.data, h.nbytes)
        bases = [slots[k % len(rows)] for k in range(K)]
        ws = [float(1 + (37 * k) % 100) for k in range(K)]
        count = None
        for w in ws:
            count = w if count is None else count + w
        e = N_.Epilogue()
        e.kind = N_.FEDAVG_EPI_ADAM
        e.lr, e.beta1, e.beta2, e.eps, e.step = 1e-3, 0.9, 0.999, 1e-8, 2.0
        e.param, e.state1, e.state2 = bufs[0].ptr, bufs[1].ptr, bufs[2].ptr
        e.torch_sqrt = torch_sqrt
        ctx.set_variant(variant)
        n_launch = ctx.launch_count()
        ctx.accumulate_tiled_epi(bases, ws, TILE, lay.tile_stride, 0, n4, None, N_.FEDAVG_OP_TORCH, N_.FEDAVG_FIN_DIV,
                                 count, e)
        ctx.sync()
        launches = ctx.launch_count() - n_launch
        got = []
        for b in bufs:
            out = np.empty(N, np.float32)
            ctx.d2h(out, b.ptr)
            got.append(out)
    finally:
        ctx.set_variant(0)
        slab.close()
        for b in bufs:
            b.close()
    tiles = (N + TILE - 1) // TILE
    # variant 0: the split-epilogue form (round 6: 4 register- + 9 LDS-held tiles, 8 waves per block); 1 << 15: round 5's
    # burst form (8 + 9); 64: the 4-LDS-tile form; 32: register-held tiles only (A/B builds)
    per_launch = ctx.num_cus * {0: 4 + 9, 1 << 15: 8 + 9, 64: 8 + 4, 32: 8}[variant]
    assert launches == -(-tiles // per_launch)  # the form that ran is the one asked for
    d = oracle.fedavg_c([rows[k % len(rows)] for k in range(K)], ws, oracle.MODE_TORCH, nthreads=8)
    oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p, m=m, v=v, step=2.0, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                          torch_cpu_sqrt=["ieee", "torch_cpu", "torch_cpu_amd"][torch_sqrt])
    for name, a, b in (("p", got[0], p), ("m", got[1], m), ("v", got[2], v)):
        assert same_bits(a, b), (name, int(np.count_nonzero(a.view(np.uint32) != b.view(np.uint32))))
