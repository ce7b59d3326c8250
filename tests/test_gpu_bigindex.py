"""Keys longer than 2^31 elements (an 8.6 GB fp32 tensor): every index and byte offset on the path must be
64-bit.  Client values come from the device generator, so the oracle regenerates them at sampled positions
(both sides of 2^31 and of 2^32 bytes, tile edges, the ragged tail) and aggregates those element by element.
Checked on the engine's tiled layout and on the contiguous-rows entry point (whole tiles on the streaming
kernel, the ragged tail on the scalar kernel)."""

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

K = 3
P = (1 << 31) + 3 * 4096 + 5
SEED = 77


def _sample_idx():
    rng = np.random.default_rng(9)
    idx = rng.integers(0, P, 4000, dtype=np.int64)
    marks = np.array([0, 1, (1 << 30) - 1, 1 << 30, (1 << 31) - 1, 1 << 31, (1 << 31) + 1, P - 6, P - 5, P - 1])
    around = np.concatenate([marks + d for d in (-4097, -4096, -1, 0, 4095, 4096)])
    idx = np.concatenate([idx, marks, around, (idx // 4096) * 4096])
    return np.unique(np.clip(idx, 0, P - 1)).astype(np.uint64)


def _room(ctx, nbytes):
    import torch

    torch.cuda.empty_cache()
    free, _ = ctx.mem_info()
    if free < nbytes + (4 << 30):
        pytest.skip(f"needs {nbytes / 2**30:.0f} GiB free, device has {free / 2**30:.0f}")


@pytest.mark.parametrize("layout", ["tiled", "rows"])
def test_key_longer_than_2pow31(oracle, layout):
    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext, TiledLayout

    ctx = DeviceContext.get(0)
    ws = [1.0, 37.0, 5.5]
    count = ws[0] + ws[1] + ws[2]
    idx = _sample_idx()
    exp = oracle.fedavg_c([oracle.synth_values(SEED, k, idx) for k in range(K)], ws, oracle.MODE_TORCH)
    if layout == "tiled":
        lay = TiledLayout(4096, K)
        _room(ctx, (lay.slab_elems(P) + P) * 4)
        slab = ctx.alloc(lay.slab_elems(P) * 4)
        bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]
        for k, b in enumerate(bases):
            ctx.fill_synthetic_f32(b, P, SEED, k, 0, lay.tile, lay.tile_stride)
        end = (P + 3) // 4 * 4
        out = ctx.alloc(end * 4)
        ctx.accumulate_tiled(bases, ws, lay.tile, lay.tile_stride, 0, end, out.ptr, N.FEDAVG_OP_TORCH,
                             N.FEDAVG_FIN_DIV, count)
        bufs = [slab]
    else:
        _room(ctx, (K + 1) * P * 4)
        bufs = [ctx.alloc(P * 4) for _ in range(K)]
        for k, b in enumerate(bufs):
            ctx.fill_synthetic_f32(b.ptr, P, SEED, k, 0, 4096, 4096)  # tile == stride: a contiguous row
        out = ctx.alloc(P * 4)
        ctx.accumulate([b.ptr for b in bufs], ws, P, out.ptr, N.FEDAVG_F32, N.FEDAVG_F32, N.FEDAVG_OP_TORCH,
                       N.FEDAVG_FIN_DIV, count)
    got = ctx.gather_f32(out.ptr, idx)
    out.close()
    for b in bufs:
        b.close()
    assert same_bits(got, exp), f"{np.count_nonzero(got.view(np.uint32) != exp.view(np.uint32))} of {idx.size} differ"
