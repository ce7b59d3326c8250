"""The few-client kernels' tile-PAIR forms with storage that starts exactly at begin's tile: the fp32
1-read form and the 16-bit 1- and 3-read forms deal units of two consecutive tiles, so when begin's tile index is odd a
unit's first tile is the one BEFORE begin's.  The C-ABI (include/nvflare_amd_fedavg.h) only requires client storage for
the tiles [begin, end) touches; the kernels clamp a unit's tiles to [begin's tile, end's tile].  Here the client slab
is allocated from begin's tile on (every base pointer is the allocation minus the tiles before it), and the result
must equal the same aggregation over a slab allocated from tile 0, bit for bit, on [begin, end)."""

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

TILE = 4096


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


def _run(ctx, elem, K, begin, end, from_tile, fmt=None):
    """Aggregate rows over [begin, end) from a slab whose storage starts at tile `from_tile`; returns the result."""
    from nvflare_amd import _native as N
    from nvflare_amd.device import TiledLayout

    rng = np.random.default_rng(K * 1000 + begin)
    n = (end + TILE - 1) // TILE * TILE
    lay = TiledLayout(TILE, K)
    if elem == 4:
        rows = [rng.standard_normal(n).astype(np.float32) for _ in range(K)]
    else:
        rows = [(rng.standard_normal(n) * 4).astype(np.float32).astype(np.float16).view(np.uint16) if fmt == "f16" else
                ((rng.standard_normal(n) * 4).astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
                for _ in range(K)]
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    skip = from_tile * lay.tile_stride * elem  # bytes of slab before the allocation
    slab = ctx.alloc(lay.slab_elems(n) * elem - skip)
    out = ctx.alloc(n * elem)
    try:
        bases = [slab.ptr - skip + lay.slot_offset_elems(k) * elem for k in range(K)]
        lo = from_tile * TILE
        for b, r in zip(bases, rows):  # logical bytes [lo, n) only: nothing is written before the allocation
            ctx.h2d_tiled(b, TILE * elem, lay.tile_stride * elem, lo * elem, r[lo:].ctypes.data, r[lo:].nbytes)
        if elem == 4:
            ctx.accumulate_tiled(bases, ws, TILE, lay.tile_stride, begin, end, out.ptr, N.FEDAVG_OP_TORCH,
                                 N.FEDAVG_FIN_DIV, _sum(ws))
            got = np.empty(n, np.float32)
        else:
            code = N.FEDAVG_BF16 if fmt == "bf16" else N.FEDAVG_F16
            ctx.accumulate_tiled16(code, bases, ws, TILE, lay.tile_stride, begin, end, out.ptr, N.FEDAVG_OP_TORCH,
                                   N.FEDAVG_FIN_DIV, _sum(ws))
            got = np.empty(n, np.uint16)
        ctx.d2h(got, out.ptr)
        return got[begin:end]
    finally:
        slab.close()
        out.close()


@pytest.mark.parametrize("begin_tile", [7, 13])
@pytest.mark.parametrize("elem,K,fmt", [(4, 1, None), (2, 1, "bf16"), (2, 3, "bf16"), (2, 1, "f16"), (2, 3, "f16")])
def test_pair_forms_read_nothing_before_begin(ctx, elem, K, fmt, begin_tile):
    begin = begin_tile * TILE + 40  # multiples of 8 (the 16-bit entry's granule)
    end = begin + 9 * TILE + 24  # several pair units, a ragged end
    full = _run(ctx, elem, K, begin, end, 0, fmt)
    own = _run(ctx, elem, K, begin, end, begin_tile, fmt)
    assert same_bits(own, full)
