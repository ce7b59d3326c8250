"""Parity at BASELINE.json's full size: 64 clients x 1e9 fp32 params (config 3, 256 GB of client updates in
HBM) and the fused FedOpt-Adam step on it (config 5).  The oracle cannot redo 64e9 multiply-adds in a test,
so the size-independent property checked is a SAMPLED bit-exact comparison: the device generator's host twin
(``oracle.synth_values``) regenerates the client values at 20 000 random positions plus both ends and every
tile edge near them, and the C oracle aggregates (and steps) them element by element.

The workload must run at its full size: if the device cannot hold 64 x 1e9 params (plus out, p, m, v) next to
what earlier tests left allocated, the fixture FAILS and names the P that would have fit -- it never shrinks
quietly."""

import gc

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

K = 64
P_FULL = 1_000_000_000
SEED = 4242


def _sample_idx(P, rng):
    idx = rng.integers(0, P, 20_000, dtype=np.int64)
    edges = (idx // 4096) * 4096
    idx = np.concatenate([idx, edges, np.maximum(edges - 1, 0), [0, 1, P - 2, P - 1]])
    return np.unique(np.clip(idx, 0, P - 1)).astype(np.uint64)


@pytest.fixture(scope="module")
def full():
    import torch

    from nvflare_amd.device import DeviceContext, TiledLayout

    gc.collect()
    torch.cuda.empty_cache()
    ctx = DeviceContext.get(0)
    free, total = ctx.mem_info()
    per_param = 4 * (K + 4)  # slab + out + p, m, v
    fits = int((free - (2 << 30)) // per_param) // 4096 * 4096
    if fits < P_FULL:
        pytest.fail(f"config 3 / 5 need {P_FULL * per_param / 1e9:.0f} GB; the device has {free / 1e9:.1f} GB free of "
                    f"{total / 1e9:.1f} (would fit P = {fits}): the full-size test does not run at a reduced size")
    P = P_FULL
    lay = TiledLayout(4096, K)
    slab = ctx.alloc(lay.slab_elems(P) * 4)
    bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]
    for k, b in enumerate(bases):
        ctx.fill_synthetic_f32(b, P, SEED, k, 0, lay.tile, lay.tile_stride)
    ctx.sync()
    yield ctx, lay, slab, bases, P
    slab.close()


@pytest.mark.parametrize("mode", ["torch", "numpy"])
def test_full_size_aggregation_sampled(full, oracle, mode):
    from nvflare_amd import _native as N

    ctx, lay, slab, bases, P = full
    ws = oracle.synth_weights(K)
    count = None
    for w in ws:
        count = w if count is None else count + w
    op, fin, omode = ((N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, oracle.MODE_TORCH) if mode == "torch"
                      else (N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE, oracle.MODE_NUMPY))
    end = (P + 3) // 4 * 4
    out = ctx.alloc(end * 4)
    ctx.accumulate_tiled(bases, ws, lay.tile, lay.tile_stride, 0, end, out.ptr, op, fin, count)
    idx = _sample_idx(P, np.random.default_rng(1 if mode == "torch" else 2))
    rows = [oracle.synth_values(SEED, k, idx) for k in range(K)]
    exp = oracle.fedavg_c(rows, ws, omode)
    got = ctx.gather_f32(out.ptr, idx)
    out.close()
    assert same_bits(got, exp), f"{np.count_nonzero(got.view(np.uint32) != exp.view(np.uint32))} of {idx.size} differ"


def _sqrt_modes():
    """The product's sqrt first (``torch_sqrt.mode()``: on the GPU pool's AMD hosts ``torch_cpu_amd``), then the
    other two restated forms."""
    from nvflare_amd import torch_sqrt

    first = torch_sqrt.mode()
    return [first] + [m for m in torch_sqrt.MODES if m != first]


@pytest.mark.parametrize("sqrt_idx", [0, 1, 2], ids=["product", "other1", "other2"])
def test_full_size_fused_adam_sampled(full, oracle, sqrt_idx):
    """Config 5: aggregation + Adam (step 1 then step 2) in one launch per step, sampled against the oracle
    aggregation followed by the oracle Adam epilogue -- in every sqrt the epilogue knows, the one the product
    ships on this host (``torch_sqrt.mode()``, the bench's config-5 line) first (nvflare/app_opt/pt/fedopt.py:157-182
    steps with torch CPU's sqrt)."""
    from nvflare_amd import _native as N
    from nvflare_amd import torch_sqrt

    sqrt_mode = _sqrt_modes()[sqrt_idx]

    ctx, lay, slab, bases, P = full
    ws = oracle.synth_weights(K)
    count = None
    for w in ws:
        count = w if count is None else count + w
    end = (P + 3) // 4 * 4
    p, m, v = (ctx.alloc(end * 4) for _ in range(3))
    ctx.fill_synthetic_f32(p.ptr, end, SEED + 7, 0, 0)
    ctx.memset(m.ptr, 0, end * 4)
    ctx.memset(v.ptr, 0, end * 4)
    idx = _sample_idx(P, np.random.default_rng(3))
    rows = [oracle.synth_values(SEED, k, idx) for k in range(K)]
    d = oracle.fedavg_c(rows, ws, oracle.MODE_TORCH)
    hp = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)
    p_h = oracle.synth_values(SEED + 7, 0, idx)
    m_h = np.zeros_like(p_h)
    v_h = np.zeros_like(p_h)
    for step in (1, 2):
        e = N.Epilogue()
        e.kind = N.FEDAVG_EPI_ADAM
        e.step = float(step)
        e.param, e.state1, e.state2 = p.ptr, m.ptr, v.ptr
        e.torch_sqrt = torch_sqrt.epilogue_flag(sqrt_mode)
        for k, val in hp.items():
            setattr(e, k, val)
        ctx.accumulate_tiled_epi(bases, ws, lay.tile, lay.tile_stride, 0, end, None, N.FEDAVG_OP_TORCH,
                                 N.FEDAVG_FIN_DIV, count, e)
        oracle.epilogue_apply(d, oracle.EPI_ADAM, p=p_h, m=m_h, v=v_h, step=float(step), torch_cpu_sqrt=sqrt_mode,
                              **hp)
        for name, buf, host in (("p", p, p_h), ("exp_avg", m, m_h), ("exp_avg_sq", v, v_h)):
            got = ctx.gather_f32(buf.ptr, idx)
            assert same_bits(got, host), f"sqrt {sqrt_mode} step {step} {name}"
    for b in (p, m, v):
        b.close()
