"""GPU parity for float16 / bfloat16 / integer / bool client arrays.

1. The drop-in helper on the reference's own outputs (tests/golden/dtype_cases.*): bit-exact on every element
   of every case -- numpy float16, every integer / bool case (numpy and torch), and torch float16 / bfloat16
   including torch's scalar-loop tail, which the engine recomputes with that loop's two roundings
   (nvflare_amd/torch16.py, fedavg_accumulate_tiled16_tails) for the one torch thread the fixtures were made
   with.
2. The 16-bit kernel through the C-ABI against the oracle, bit-exact on EVERY element: both formats, all
   ops, K up to 131 (chained launches), ragged n, unaligned rows (per-element path), acc_in continuation.
3. Device-resident bfloat16 tensors in, device tensor out."""

import numpy as np
import pytest
import torch

from golden_util import (
    as_f32_values,
    dtype_case_inputs,
    dtype_case_weights,
    load_dtype_golden,
    same_bits,
)
from oracle import fedavg_oracle as orc

pytestmark = pytest.mark.gpu

META, ARRAYS = load_dtype_golden()
CASES = sorted(META["cases"].items())


@pytest.mark.parametrize("name,case", CASES, ids=[n for n, _ in CASES])
def test_helper_dtype_golden(name, case):
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    rows = dtype_case_inputs(case, ARRAYS)
    ws = dtype_case_weights(case)
    h = WeightedAggregationHelper(weigh_by_local_iter=case["weighted"])
    for k, (r, w) in enumerate(zip(rows, ws)):
        h.add({"w": r}, w, f"site-{k}", 0)
    threads = torch.get_num_threads()
    torch.set_num_threads(1)  # the fixtures' torch thread count (the tails follow this process's setting)
    try:
        got = h.get_result()["w"]
    finally:
        torch.set_num_threads(threads)
    dt = case["dtype"]
    exp_bits = ARRAYS[case["expected"]]
    if case["container"] == "torch":
        assert isinstance(got, torch.Tensor)
        assert str(got.dtype).replace("torch.", "") == case["expected_dtype"]
    else:
        assert str(np.asarray(got).dtype) == case["expected_dtype"]
    if case["container"] != "torch" or dt not in ("float16", "bfloat16"):
        g = got.numpy() if isinstance(got, torch.Tensor) else np.asarray(got)
        assert same_bits(g, exp_bits), name
        return
    g, exp = as_f32_values(got, dt), as_f32_values(exp_bits, dt)
    assert same_bits(g, exp), name


@pytest.fixture(scope="module")
def ctx():
    from nvflare_amd.device import DeviceContext

    return DeviceContext.get(0)


def _bits(x_f32, fmt):
    if fmt == "bfloat16":
        return orc.f32_to_bf16_bits(x_f32)
    return x_f32.astype(np.float16).view(np.uint16)


def _vals(bits, fmt):
    if fmt == "bfloat16":
        return orc.bf16_bits_to_f32(bits)
    return bits.view(np.float16).astype(np.float32)


def _kernel16(ctx, rows_bits, weights, fmt, op, fin, count, acc_in_bits=None, offset=0):
    """fedavg_accumulate with (fmt, fmt) dtypes on device buffers; rows at `offset` elements past 16 B."""
    from nvflare_amd import _native as N

    code = N.FEDAVG_BF16 if fmt == "bfloat16" else N.FEDAVG_F16
    n = rows_bits[0].size if rows_bits else acc_in_bits.size
    bufs, ptrs = [], []
    for r in rows_bits:
        b = ctx.alloc((n + offset) * 2 + 16)
        bufs.append(b)
        p = b.ptr + offset * 2
        ctx.h2d_ptr(p, r.ctypes.data, r.nbytes)
        ptrs.append(p)
    ob = ctx.alloc((n + offset) * 2 + 16)
    optr = ob.ptr + offset * 2
    acc_ptr = None
    if acc_in_bits is not None:
        ctx.h2d_ptr(optr, acc_in_bits.ctypes.data, acc_in_bits.nbytes)
        acc_ptr = optr
    ctx.accumulate(ptrs, weights, n, optr, code, code, op, fin, count, acc_in_ptr=acc_ptr)
    out = np.empty(n, dtype=np.uint16)
    ctx.d2h(out, optr)
    for b in bufs + [ob]:
        b.close()
    return out


def _count(ws):
    c = None
    for w in ws:
        c = w if c is None else c + w
    return c


CONFIGS = [("bfloat16", "torch"), ("float16", "torch"), ("float16", "numpy"), ("bfloat16", "unweighted"),
           ("float16", "unweighted_numpy")]


@pytest.mark.parametrize("fmt,mode", CONFIGS)
@pytest.mark.parametrize("K,n,offset", [(1, 1, 0), (3, 7, 0), (5, 4099, 0), (5, 4099, 1), (131, 1000, 0), (8, 65536 + 24, 3)])
def test_kernel16_vs_oracle(ctx, fmt, mode, K, n, offset):
    from nvflare_amd import _native as N

    rng = np.random.default_rng(K * 1000 + n + offset)
    rows = [_bits((rng.standard_normal(n) * 4).astype(np.float32), fmt) for _ in range(K)]
    ws = [float(rng.random() * 20 + 1e-3) for _ in range(K)]
    vals = [_vals(r, fmt) for r in rows]
    if mode == "torch":
        op, fin = N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV
        exp = orc.torch16_vector_reference(vals, ws, fmt)
    elif mode == "unweighted":
        op, fin = N.FEDAVG_OP_UNWEIGHTED, N.FEDAVG_FIN_DIV
        exp = orc.torch16_vector_reference(vals, ws, fmt, weighted=False)
    elif mode == "numpy":
        op, fin = N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE
        exp = orc.numpy_mode_reference([r.view(np.float16) for r in rows], ws).astype(np.float32)
    else:
        op, fin = N.FEDAVG_OP_UNWEIGHTED, N.FEDAVG_FIN_SCALE
        exp = orc.numpy_mode_reference([r.view(np.float16) for r in rows], ws, weighted=False).astype(np.float32)
    got = _vals(_kernel16(ctx, rows, ws, fmt, op, fin, _count(ws), offset=offset), fmt)
    assert same_bits(got, exp)
    if K >= 3:  # split the clients over two calls: partial sum in 16 bits, continued through acc_in
        part = _kernel16(ctx, rows[:2], ws[:2], fmt, op, N.FEDAVG_FIN_NONE, 1.0, offset=offset)
        full = _kernel16(ctx, rows[2:], ws[2:], fmt, op, fin, _count(ws), acc_in_bits=part, offset=offset)
        assert same_bits(_vals(full, fmt), exp)


def test_device_bf16_tensors_through_helper():
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    rng = np.random.default_rng(7)
    rows = [torch.from_numpy(rng.standard_normal(10_000).astype(np.float32)).to(torch.bfloat16) for _ in range(6)]
    ws = [float(1 + k) for k in range(6)]
    h = WeightedAggregationHelper()
    for k, r in enumerate(rows):
        h.add({"w": r.to("cuda:0"), "h": r.to(torch.float16).to("cuda:0")}, ws[k], f"s{k}", 0)
    out = h.get_result()
    assert out["w"].device.type == "cuda" and out["w"].dtype == torch.bfloat16
    assert out["h"].device.type == "cuda" and out["h"].dtype == torch.float16
    # the reference's ops as torch-ROCm runs them on device tensors: alpha kept in fp32, div_ as a product with
    # the fp32 reciprocal (FEDAVG_OP_TORCH_DEVICE / FEDAVG_FIN_RECIP)
    exp = orc.torch_mode_reference([r.to("cuda:0") for r in rows], ws)
    assert torch.equal(out["w"].view(torch.int16), exp.view(torch.int16))
    exp_h = orc.torch_mode_reference([r.to(torch.float16).to("cuda:0") for r in rows], ws)
    assert torch.equal(out["h"].view(torch.int16), exp_h.view(torch.int16))
    # and it differs from torch CPU's arithmetic on the same values (alpha rounded, true division)
    cpu = orc.torch_mode_reference([r.clone() for r in rows], ws)
    assert not torch.equal(out["w"].cpu().view(torch.int16), cpu.view(torch.int16))


# ---------------------------------------------------------------------------------------------------
# the tiled 16-bit kernel (engine slabs for float16 / bfloat16 keys) against the oracle, every element
# ---------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("fmt,mode", CONFIGS)
@pytest.mark.parametrize("K,slots,begin,end", [(1, 1, 0, 8), (5, 8, 0, 3 * 4096 + 8), (7, 16, 4096 - 8, 2 * 4096 + 64),
                                               (131, 131, 0, 4096 + 16)])
def test_tiled16_vs_oracle(ctx, fmt, mode, K, slots, begin, end):
    from nvflare_amd import _native as N
    from nvflare_amd.device import TiledLayout

    n = (end + 4095) // 4096 * 4096
    rng = np.random.default_rng(K + begin + end)
    rows = [_bits((rng.standard_normal(n) * 4).astype(np.float32), fmt) for _ in range(K)]
    ws = [float(rng.random() * 20 + 1e-3) for _ in range(K)]
    vals = [_vals(r[begin:end], fmt) for r in rows]
    if mode in ("torch", "unweighted"):
        op = N.FEDAVG_OP_TORCH if mode == "torch" else N.FEDAVG_OP_UNWEIGHTED
        fin = N.FEDAVG_FIN_DIV
        exp = orc.torch16_vector_reference(vals, ws, fmt, weighted=mode == "torch")
    else:
        op = N.FEDAVG_OP_NUMPY if mode == "numpy" else N.FEDAVG_OP_UNWEIGHTED
        fin = N.FEDAVG_FIN_SCALE
        exp = orc.numpy_mode_reference([r[begin:end].view(np.float16) for r in rows], ws,
                                       weighted=mode == "numpy").astype(np.float32)
    code = N.FEDAVG_BF16 if fmt == "bfloat16" else N.FEDAVG_F16
    lay = TiledLayout(4096, slots)
    slab = ctx.alloc(lay.slab_elems(n) * 2)
    bases = [slab.ptr + lay.slot_offset_elems(k) * 2 for k in range(K)]
    for b, r in zip(bases, rows):
        ctx.h2d_tiled(b, 4096 * 2, lay.tile_stride * 2, 0, r.ctypes.data, r.nbytes)
    out = ctx.alloc(n * 2)
    ctx.accumulate_tiled16(code, bases, ws, 4096, lay.tile_stride, begin, end, out.ptr, op, fin, _count(ws))
    got = np.empty(n, np.uint16)
    ctx.d2h(got, out.ptr)
    assert same_bits(_vals(got[begin:end], fmt), exp)
    if K >= 3:  # first two clients, then the rest continuing through acc_in
        ctx.accumulate_tiled16(code, bases[:2], ws[:2], 4096, lay.tile_stride, begin, end, out.ptr, op,
                               N.FEDAVG_FIN_NONE, 1.0)
        ctx.accumulate_tiled16(code, bases[2:], ws[2:], 4096, lay.tile_stride, begin, end, out.ptr, op, fin,
                               _count(ws), acc_in_ptr=out.ptr)
        ctx.d2h(got, out.ptr)
        assert same_bits(_vals(got[begin:end], fmt), exp)
    slab.close()
    out.close()


@pytest.mark.parametrize("fmt", ["bfloat16", "float16"])
@pytest.mark.parametrize("K", [5, 131])
def test_tiled16_tails_vs_oracle(ctx, fmt, K):
    """fedavg_accumulate_tiled16_tails: listed elements take torch's scalar-loop step (recomputed before the
    tile kernel, written over its results after it), chained past 128 clients and through acc_in in place."""
    from nvflare_amd import _native as N
    from nvflare_amd.device import TiledLayout

    begin, end = 8 * 37, 3 * 4096 + 8 * 11
    n = (end + 4095) // 4096 * 4096
    rng = np.random.default_rng(K)
    rows = [_bits((rng.standard_normal(n) * 40).astype(np.float32), fmt) for _ in range(K)]
    ws = [float(rng.random() * 20 + 1e-3) for _ in range(K)]
    vals = [_vals(r[begin:end], fmt) for r in rows]
    mask = np.zeros(end - begin, bool)
    mask[rng.choice(end - begin, 200, replace=False)] = True
    mask[-31:] = True
    mask[4096 - begin - 5:4096 - begin + 9] = True  # across a tile boundary
    tails = np.concatenate([[0, begin - 8], np.nonzero(mask)[0] + begin, [end, n - 1]]).astype(np.int64)  # out of range ignored
    exp = orc.torch16_reference(vals, ws, fmt, mask=mask)
    assert not same_bits(exp, orc.torch16_vector_reference(vals, ws, fmt))  # the tails matter here
    code = N.FEDAVG_BF16 if fmt == "bfloat16" else N.FEDAVG_F16
    lay = TiledLayout(4096, 8)
    slab = ctx.alloc(lay.slab_elems(n) * 2 * -(-K // 8))
    per = lay.slab_elems(n)
    bases = [slab.ptr + ((k // 8) * per + lay.slot_offset_elems(k % 8)) * 2 for k in range(K)]
    for b, r in zip(bases, rows):
        ctx.h2d_tiled(b, 4096 * 2, lay.tile_stride * 2, 0, r.ctypes.data, r.nbytes)
    out = ctx.alloc(n * 2)
    ctx.accumulate_tiled16(code, bases, ws, 4096, lay.tile_stride, begin, end, out.ptr, N.FEDAVG_OP_TORCH,
                           N.FEDAVG_FIN_DIV, _count(ws), tails=tails)
    got = np.empty(n, np.uint16)
    ctx.d2h(got, out.ptr)
    assert same_bits(_vals(got[begin:end], fmt), exp)
    ctx.accumulate_tiled16(code, bases[:2], ws[:2], 4096, lay.tile_stride, begin, end, out.ptr, N.FEDAVG_OP_TORCH,
                           N.FEDAVG_FIN_NONE, 1.0, tails=tails)
    ctx.accumulate_tiled16(code, bases[2:], ws[2:], 4096, lay.tile_stride, begin, end, out.ptr, N.FEDAVG_OP_TORCH,
                           N.FEDAVG_FIN_DIV, _count(ws), acc_in_ptr=out.ptr, tails=tails)
    ctx.d2h(got, out.ptr)
    assert same_bits(_vals(got[begin:end], fmt), exp)
    slab.close()
    out.close()


@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.bfloat16, torch.float16, torch.int32])
@pytest.mark.parametrize("weighted", [True, False])
def test_device_tensors_match_torch_rocm(dt, weighted):
    """Device-resident tensors: the helper's torch ops as torch-ROCm runs them on the GPU (probe:
    tools/torch_gpu_semantics_probe.py) -- alpha in fp32 for every dtype, div_ by a scalar as a product with the
    opmath reciprocal -- bit for bit, for ragged sizes, a 0-d key and 130 clients (chained launches)."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    if dt == torch.int32 and not weighted:
        pytest.skip("an integer total's div_ raises (tests/test_cpu_boundary.py)")
    rng = np.random.default_rng(5)
    # float16: below one 2048-element block torch-ROCm runs every element through its unrolled (single-rounding)
    # path, whole blocks through its vector path, the last partial block unrolled again (nvflare_amd/torch16.py)
    sizes = {"a": (4097 * 3 + 5,), "b": (33, 7), "c": (), "d": (3072,), "e": (2048,)}
    for K in (6, 130):
        clients = []
        for _ in range(K):
            c = {}
            for k, s in sizes.items():
                x = torch.from_numpy(np.asarray(rng.standard_normal(s) * 20, dtype=np.float32))
                c[k] = (x.round() if dt == torch.int32 else x).to(dt).to("cuda:0")
            clients.append(c)
        ws = [float(rng.random() * 4 + 0.05) for _ in range(K)]
        h = WeightedAggregationHelper(weigh_by_local_iter=weighted)
        for k, (c, w) in enumerate(zip(clients, ws)):
            h.add(c, w, f"s{k}", 0)
        out = h.get_result()
        for key in sizes:
            exp = orc.torch_mode_reference([c[key].clone() for c in clients], ws, weighted=weighted)
            got = out[key]
            assert got.device.type == "cuda" and got.dtype == exp.dtype and got.shape == exp.shape, key
            if got.dtype in (torch.bfloat16, torch.float16):
                got, exp = got.view(torch.int16), exp.view(torch.int16)
            assert torch.equal(got, exp), (key, K)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_helper_torch16_matches_torch_cpu(dt, threads):
    """The drop-in helper against torch CPU itself (mul / add_(alpha) / div_ run by torch, as the reference's
    helper runs them) on 16-bit tensors whose scalar-loop elements depend on torch's thread ranges: sizes
    below and above the 32768-element grain, ragged against the 32-element vector blocks."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rng = np.random.default_rng(threads)
        sizes = {"a": (33000 + 7,), "b": (3, 23339), "c": (1031,), "d": (100003,), "e": (64, 512)}
        K = 6
        clients = [{k: torch.from_numpy((rng.standard_normal(s) * 30).astype(np.float32)).to(dt) for k, s in sizes.items()}
                   for _ in range(K)]
        ws = [float(rng.random() * 5 + 0.1) for _ in range(K)]
        h = WeightedAggregationHelper()
        for k, (c, w) in enumerate(zip(clients, ws)):
            h.add(c, w, f"site-{k}", 0)
        got = h.get_result()
        for key in sizes:
            exp = orc.torch_mode_reference([c[key].clone() for c in clients], ws)
            assert got[key].dtype == dt and got[key].shape == exp.shape
            assert torch.equal(got[key].view(torch.int16), exp.view(torch.int16)), (key, threads)
    finally:
        torch.set_num_threads(old)


@pytest.mark.parametrize("budget", [None, 1])
def test_engine_mixed_fp32_bf16_model(budget):
    """An fp32 + bf16 + fp16 + int64 model through the helper: 16-bit keys in their own tiled arenas, partial
    keys, several slab geometries (40 clients), folding under a 1-byte budget -- bit-exact vs the oracle."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    rng = np.random.default_rng(9)
    K = 40
    shapes = {"a.w": (64, 129), "a.b": (64,), "emb": (5000, 3), "ln": (7,)}
    clients = []
    for k in range(K):
        c = {"a.w": torch.from_numpy(rng.standard_normal(shapes["a.w"]).astype(np.float32)),
             "a.b": torch.from_numpy(rng.standard_normal(shapes["a.b"]).astype(np.float32)).to(torch.bfloat16),
             "emb": torch.from_numpy(rng.standard_normal(shapes["emb"]).astype(np.float32)).to(torch.bfloat16),
             "ln": torch.from_numpy(rng.standard_normal(shapes["ln"]).astype(np.float16)),
             "steps": torch.tensor(k, dtype=torch.int64)}
        if k == 3:
            del c["emb"]  # a partial contribution
        clients.append(c)
    ws = [float(1 + (37 * k) % 11) for k in range(K)]
    h = WeightedAggregationHelper(max_resident_bytes=budget)
    for k, (c, w) in enumerate(zip(clients, ws)):
        h.add(c, w, f"s{k}", 0)
    out = h.get_result()
    for key in ("a.b", "emb", "ln"):  # torch CPU itself (mul / add_ / div_), scalar-loop tails included
        seq = [(c[key], w) for c, w in zip(clients, ws) if key in c]
        exp = orc.torch_mode_reference([t.clone() for t, _ in seq], [w for _, w in seq])
        assert torch.equal(out[key].view(torch.int16), exp.view(torch.int16)), key
    exp_w = orc.torch_mode_reference([c["a.w"].clone() for c in clients], ws)
    assert same_bits(out["a.w"].numpy(), exp_w.numpy())
    if budget == 1:
        assert h.engine.stats["folds"] >= 1


@pytest.mark.parametrize("mode", ["numpy", "torch", "unweighted"])
@pytest.mark.parametrize("K,slots,begin,end", [(1, 1, 0, 4096), (3, 4, 64, 3 * 4096 + 130), (130, 131, 8, 2 * 4096)])
def test_tiled64_vs_oracle(ctx, mode, K, slots, begin, end):
    """fp64 arena kernel (fedavg_accumulate_tiled64) against the C oracle's fp64 restatement: numpy
    (v*w then add, T * (1.0/count)), torch (fma, T / count), unweighted; partial ranges, more clients than one
    launch holds (chained through out), and a continuation through acc_in."""
    from nvflare_amd import _native as N
    from nvflare_amd.device import TiledLayout

    n = (end + 4095) // 4096 * 4096
    rng = np.random.default_rng(K + begin + end)
    rows = [rng.standard_normal(n) * 4 for _ in range(K)]
    ws = [float(rng.random() * 20 + 1e-3) for _ in range(K)]
    weighted = mode != "unweighted"
    omode = orc.MODE_TORCH if mode == "torch" else orc.MODE_NUMPY
    op = {"numpy": N.FEDAVG_OP_NUMPY, "torch": N.FEDAVG_OP_TORCH, "unweighted": N.FEDAVG_OP_UNWEIGHTED}[mode]
    fin = N.FEDAVG_FIN_DIV if mode == "torch" else N.FEDAVG_FIN_SCALE
    exp = orc.fedavg_c([r[begin:end].copy() for r in rows], ws, omode, weighted=weighted, fin=fin,
                       count=_count(ws) if weighted else float(K))
    lay = TiledLayout(4096, slots)
    slab = ctx.alloc(lay.slab_elems(n) * 8)
    bases = [slab.ptr + lay.slot_offset_elems(k) * 8 for k in range(K)]
    for b, r in zip(bases, rows):
        ctx.h2d_tiled(b, 4096 * 8, lay.tile_stride * 8, 0, r.ctypes.data, r.nbytes)
    out = ctx.alloc(n * 8)
    count = _count(ws) if weighted else float(K)
    ctx.accumulate_tiled64(bases, ws, 4096, lay.tile_stride, begin, end, out.ptr, op, fin, count)
    got = np.empty(n, np.float64)
    ctx.d2h(got, out.ptr)
    assert same_bits(got[begin:end], exp)
    if K >= 3:
        ctx.accumulate_tiled64(bases[:2], ws[:2], 4096, lay.tile_stride, begin, end, out.ptr, op, N.FEDAVG_FIN_NONE, 1.0)
        ctx.accumulate_tiled64(bases[2:], ws[2:], 4096, lay.tile_stride, begin, end, out.ptr, op, fin, count,
                               acc_in_ptr=out.ptr)
        ctx.d2h(got, out.ptr)
        assert same_bits(got[begin:end], exp)
    slab.close()
    out.close()


@pytest.mark.parametrize("fmt,mode", [("bfloat16", "torch"), ("float16", "torch"), ("float16", "numpy"),
                                      ("bfloat16", "unweighted")])
@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("form", [0, 1, 2, 3, 4])
def test_tiled16_few_client_forms(ctx, fmt, mode, K, form):
    """The 16-bit few-client burst kernel (fedavg_narrow.hip fedavg_tiles_narrow_few; 1-3 client reads, no chained
    sum): several launches and a short last one (13 001 tiles), unconditional loads (a launch's slots past its last
    tile re-read that tile, nothing past it is stored), tiles of zeros, of huge and of tiny values (FIN_DIV's per-tile
    rare-case branch), a sub-range starting and ending inside tiles with a sentinel around it; bit for bit.  Forms 1-4
    (launch variant bits 9-11) are the A/B geometries (fedavg_internal.h kNarrowFewAB), in -DFEDAVG_AB_FEW builds."""
    from nvflare_amd import _native as N
    from nvflare_amd.device import TiledLayout

    if form:
        try:
            ctx.set_variant(form << 9)
        except N.FedAvgError:
            pytest.skip("an A/B form: tools/build_rev_lib.py --product -D FEDAVG_AB_FEW builds the library carrying it")
        ctx.set_variant(0)
    n_tiles = 13_001
    n = n_tiles * 4096
    rng = np.random.default_rng(K * 10 + form)
    rows = []
    for _ in range(K):
        x = (rng.standard_normal(n) * 4).astype(np.float32)
        x[4096 * 5:4096 * 6] = 0.0  # a tile of zeros: the exact division's rare case
        x[4096 * 9:4096 * 9 + 700] *= 1e30 if fmt == "bfloat16" else 1.0
        x[4096 * 11:4096 * 11 + 300] *= 1e-30 if fmt == "bfloat16" else 1e-4
        rows.append(_bits(x, fmt))
    ws = [float(rng.random() * 20 + 1e-3) for _ in range(K)]
    if mode in ("torch", "unweighted"):
        op = N.FEDAVG_OP_TORCH if mode == "torch" else N.FEDAVG_OP_UNWEIGHTED
        fin = N.FEDAVG_FIN_DIV
    else:
        op, fin = N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE

    def expected(b, e):
        if fin == N.FEDAVG_FIN_DIV:
            return orc.torch16_vector_reference([_vals(r[b:e], fmt) for r in rows], ws, fmt, weighted=mode == "torch")
        return orc.numpy_mode_reference([r[b:e].view(np.float16) for r in rows], ws).astype(np.float32)

    code = N.FEDAVG_BF16 if fmt == "bfloat16" else N.FEDAVG_F16
    lay = TiledLayout(4096, K)
    slab = ctx.alloc(lay.slab_elems(n) * 2)
    out = ctx.alloc(n * 2)
    try:
        bases = [slab.ptr + lay.slot_offset_elems(k) * 2 for k in range(K)]
        for b, r in zip(bases, rows):
            ctx.h2d_tiled(b, 4096 * 2, lay.tile_stride * 2, 0, r.ctypes.data, r.nbytes)
        got = np.empty(n, np.uint16)
        ctx.set_variant(form << 9)
        n0 = ctx.launch_count()
        ctx.accumulate_tiled16(code, bases, ws, 4096, lay.tile_stride, 0, n, out.ptr, op, fin, _count(ws))
        assert ctx.launch_count() - n0 >= 2  # several launches, the last partial
        ctx.d2h(got, out.ptr)
        assert same_bits(_vals(got, fmt), expected(0, n)), (fmt, mode, K, form)
        lo, hi = 4096 * 7 + 40, n - 4096 * 3 - 104
        sentinel = np.full(n, 0x7E00, np.uint16)
        ctx.h2d_ptr(out.ptr, sentinel.ctypes.data, sentinel.nbytes)
        ctx.accumulate_tiled16(code, bases, ws, 4096, lay.tile_stride, lo, hi, out.ptr, op, fin, _count(ws))
        ctx.d2h(got, out.ptr)
        assert same_bits(_vals(got[lo:hi], fmt), expected(lo, hi))
        assert np.all(got[:lo] == 0x7E00) and np.all(got[hi:] == 0x7E00)
    finally:
        ctx.set_variant(0)
        slab.close()
        out.close()


@pytest.mark.parametrize("mode", ["numpy", "torch", "unweighted"])
@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("form", [0, 1, 2, 3, 4])
def test_tiled64_few_client_forms(ctx, mode, K, form):
    """The fp64 few-client burst kernel (fedavg_kernels.hip fedavg_tiles_f64x2_few; 1-3 client reads, no chained sum):
    several launches and a short last one (4001 tiles), unconditional loads (a launch's slots past its last tile
    re-read that tile, nothing past it is stored), zeros, huge, tiny and subnormal values, a sub-range starting and
    ending inside tiles with a sentinel around it; bit for bit against the C oracle's fp64 restatement.  Forms 1-4
    (launch variant bits 9-11) are the A/B geometries (fedavg_internal.h kF64FewAB), in -DFEDAVG_AB_FEW builds."""
    from nvflare_amd import _native as N
    from nvflare_amd.device import TiledLayout

    if form:
        try:
            ctx.set_variant(form << 9)
        except N.FedAvgError:
            pytest.skip("an A/B form: tools/build_rev_lib.py --product -D FEDAVG_AB_FEW builds the library carrying it")
        ctx.set_variant(0)
    n = 4001 * 4096
    rng = np.random.default_rng(K * 10 + form)
    rows = []
    for _ in range(K):
        x = rng.standard_normal(n) * 4
        x[4096 * 5:4096 * 6] = 0.0
        x[4096 * 9:4096 * 9 + 700] *= 1e300
        x[4096 * 11:4096 * 11 + 300] *= 1e-310
        rows.append(x)
    ws = [float(rng.random() * 20 + 1e-3) for _ in range(K)]
    weighted = mode != "unweighted"
    omode = orc.MODE_TORCH if mode == "torch" else orc.MODE_NUMPY
    op = {"numpy": N.FEDAVG_OP_NUMPY, "torch": N.FEDAVG_OP_TORCH, "unweighted": N.FEDAVG_OP_UNWEIGHTED}[mode]
    fin = N.FEDAVG_FIN_DIV if mode == "torch" else N.FEDAVG_FIN_SCALE
    count = _count(ws) if weighted else float(K)

    def expected(b, e):
        return orc.fedavg_c([r[b:e].copy() for r in rows], ws, omode, weighted=weighted, fin=fin, count=count,
                            nthreads=8)

    lay = TiledLayout(4096, K)
    slab = ctx.alloc(lay.slab_elems(n) * 8)
    out = ctx.alloc(n * 8)
    try:
        bases = [slab.ptr + lay.slot_offset_elems(k) * 8 for k in range(K)]
        for b, r in zip(bases, rows):
            ctx.h2d_tiled(b, 4096 * 8, lay.tile_stride * 8, 0, r.ctypes.data, r.nbytes)
        got = np.empty(n, np.float64)
        ctx.set_variant(form << 9)
        n0 = ctx.launch_count()
        ctx.accumulate_tiled64(bases, ws, 4096, lay.tile_stride, 0, n, out.ptr, op, fin, count)
        assert ctx.launch_count() - n0 >= 2  # several launches, the last partial
        ctx.d2h(got, out.ptr)
        assert same_bits(got, expected(0, n)), (mode, K, form)
        lo, hi = 4096 * 7 + 42, n - 4096 * 3 - 106
        sentinel = np.full(n, -7.0)
        ctx.h2d_ptr(out.ptr, sentinel.ctypes.data, sentinel.nbytes)
        ctx.accumulate_tiled64(bases, ws, 4096, lay.tile_stride, lo, hi, out.ptr, op, fin, count)
        ctx.d2h(got, out.ptr)
        assert same_bits(got[lo:hi], expected(lo, hi))
        assert np.all(got[:lo] == -7.0) and np.all(got[hi:] == -7.0)
    finally:
        ctx.set_variant(0)
        slab.close()
        out.close()
