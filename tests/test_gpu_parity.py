"""GPU parity: the HIP path (through the C-ABI and the drop-in classes) against the reference's golden
vectors and the pinned CPU oracle.  Bit-exact is the bar (NaN payloads excepted; see golden_util).

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""

import numpy as np
import pytest
import torch

from golden_util import helper_cases, intime_cases, same_bits

pytestmark = pytest.mark.gpu

HCASES, ARRAYS = helper_cases()
ICASES, _ = intime_cases()


def _container(arr, container, device=None):
    if container == "torch":
        t = torch.from_numpy(np.array(arr, copy=True))
        return t.to(device) if device is not None else t
    return np.array(arr, copy=True)


def _as_numpy(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return np.asarray(v)


@pytest.fixture(scope="module")
def ctx():
    from nvflare_amd.device import DeviceContext

    return DeviceContext.get(0)


# ---------------------------------------------------------------------------------------------------
# golden vectors (produced by the reference itself) through the drop-in helper
# ---------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", HCASES, ids=[c["name"] for c in HCASES])
def test_helper_golden_bitexact(case):
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    h = WeightedAggregationHelper(exclude_vars=case["exclude_vars"], weigh_by_local_iter=case["weigh_by_local_iter"])
    for c in case["contributions"]:
        data = {k: _container(ARRAYS[name], case["container"]) for k, name in c["data"].items()}
        h.add(data, c["weight"], c["name"], 0)
    out = h.get_result()
    assert set(out) == set(case["expected"])
    for k, name in case["expected"].items():
        exp = ARRAYS[name]
        got = out[k]
        if case["container"] == "torch":
            assert isinstance(got, torch.Tensor)
        got = _as_numpy(got)
        assert str(got.dtype) == case["expected_dtype"][k], k
        assert same_bits(got.reshape(exp.shape), exp), f"{case['name']}:{k}"
    assert h.last_aggregation_stats == case["stats"]


@pytest.mark.parametrize("case", HCASES[:6], ids=[c["name"] for c in HCASES[:6]])
def test_helper_golden_bitexact_with_folding(case):
    """A tiny HBM budget forces the staged contributions to be folded every step: same bits."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    h = WeightedAggregationHelper(exclude_vars=case["exclude_vars"], weigh_by_local_iter=case["weigh_by_local_iter"],
                                  max_resident_bytes=1)
    for c in case["contributions"]:
        h.add({k: _container(ARRAYS[n], case["container"]) for k, n in c["data"].items()}, c["weight"], c["name"], 0)
    out = h.get_result()
    for k, name in case["expected"].items():
        assert same_bits(_as_numpy(out[k]).reshape(ARRAYS[name].shape), ARRAYS[name]), k
    if len(case["contributions"]) > 1:
        assert h.engine.stats["folds"] >= 1


@pytest.mark.parametrize("case", [c for c in HCASES if "partial" in c["name"] or "many_keys" in c["name"]
                                  or "k64" in c["name"] or "special" in c["name"]],
                         ids=[c["name"] for c in HCASES if "partial" in c["name"] or "many_keys" in c["name"]
                              or "k64" in c["name"] or "special" in c["name"]])
def test_helper_golden_bitexact_sharded(case):
    """Parameter-bucket sharding over 3 engines (here all on device 0): same bits as one device."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    h = WeightedAggregationHelper(exclude_vars=case["exclude_vars"], weigh_by_local_iter=case["weigh_by_local_iter"],
                                  devices=[0, 0, 0])
    for c in case["contributions"]:
        h.add({k: _container(ARRAYS[n], case["container"]) for k, n in c["data"].items()}, c["weight"], c["name"], 0)
    out = h.get_result()
    assert set(out) == set(case["expected"])
    for k, name in case["expected"].items():
        got = _as_numpy(out[k])
        assert str(got.dtype) == case["expected_dtype"][k]
        assert same_bits(got.reshape(ARRAYS[name].shape), ARRAYS[name]), k
    h.engine.release()


def oracle_mod():
    from oracle import fedavg_oracle

    return fedavg_oracle


@pytest.mark.parametrize("case", [c for c in HCASES if c["container"] == "torch"][:4],
                         ids=[c["name"] for c in HCASES if c["container"] == "torch"][:4])
def test_helper_device_tensors(case):
    """torch tensors already on the GPU: staged D2D, result returned as a device tensor -- bit for bit what the
    reference helper's torch ops (mul / add_(alpha) / div_) give when torch-ROCm runs them on those tensors
    (FEDAVG_OP_TORCH_DEVICE / FEDAVG_FIN_RECIP: div_ by a scalar is a product with the fp32 reciprocal there)."""
    import re

    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    h = WeightedAggregationHelper(exclude_vars=case["exclude_vars"], weigh_by_local_iter=case["weigh_by_local_iter"])
    seqs = {}
    for c in case["contributions"]:
        data = {k: _container(ARRAYS[n], "torch", "cuda:0") for k, n in c["data"].items()}
        h.add(data, c["weight"], c["name"], 0)
        for k, v in data.items():
            if not (case["exclude_vars"] and re.search(case["exclude_vars"], k)):
                seqs.setdefault(k, []).append((v.clone(), c["weight"]))
    out = h.get_result()
    assert set(out) == set(seqs)
    for k, seq in seqs.items():
        exp = oracle_mod().torch_mode_reference([v for v, _ in seq], [w for _, w in seq],
                                                weighted=case["weigh_by_local_iter"])
        assert out[k].device.type == "cuda" and out[k].dtype == exp.dtype
        assert same_bits(_as_numpy(out[k]), _as_numpy(exp)), k


@pytest.mark.parametrize("case", ICASES, ids=[c["name"] for c in ICASES])
def test_intime_golden_bitexact(case):
    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import (
        InTimeAccumulateWeightedAggregator,
    )
    from nvflare_amd.compat import DXO, AppConstants, DataKind, FLContext, MetaKey, ReservedKey, Shareable, from_shareable

    edk = case["expected_data_kind"]
    agg = InTimeAccumulateWeightedAggregator(
        exclude_vars=case["exclude_vars"], aggregation_weights=case["aggregation_weights"], expected_data_kind=edk
    )
    agg._initialize(agg.aggregation_weights, agg.exclude_vars, agg.expected_data_kind)
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0)
    for cl in case["clients"]:
        def mk(d):
            return DXO(d["kind"], data={k: _container(ARRAYS[n], case["container"]) for k, n in d["data"].items()},
                       meta={MetaKey.NUM_STEPS_CURRENT_ROUND: d["n_iter"]})
        if "" in cl["dxos"]:
            dxo = mk(cl["dxos"][""])
        else:
            dxo = DXO(DataKind.COLLECTION, data={dk: mk(d) for dk, d in cl["dxos"].items()})
        s = Shareable()
        s.set_peer_props({ReservedKey.IDENTITY_NAME: cl["name"]})
        s.add_cookie(AppConstants.CONTRIBUTION_ROUND, 0)
        assert agg.accept(dxo.update_shareable(s), fl_ctx) == cl["accepted"]
    res = from_shareable(agg.aggregate(fl_ctx))
    if "" in case["expected"]:
        got = {"": res}
    else:
        assert res.data_kind == DataKind.COLLECTION
        got = res.data
    for dk, exp in case["expected"].items():
        assert got[dk].data_kind == exp["kind"]
        for k, name in exp["data"].items():
            assert same_bits(_as_numpy(got[dk].data[k]).reshape(ARRAYS[name].shape), ARRAYS[name]), (dk, k)
    assert fl_ctx.get_prop(AppConstants.AGGREGATION_STATS) == case["stats"]


# ---------------------------------------------------------------------------------------------------
# the kernel through the C-ABI against the C oracle
# ---------------------------------------------------------------------------------------------------
def _run_kernel(ctx, rows, weights, op, fin, count, acc_in=None, offset_elems=0, out_dtype=None):
    from nvflare_amd import _native as N
    from nvflare_amd.device import fedavg_dtype

    in_np = rows[0].dtype if rows else acc_in.dtype
    acc_np = np.dtype(out_dtype) if out_dtype is not None else (acc_in.dtype if acc_in is not None else in_np)
    n = rows[0].size if rows else acc_in.size
    isz = np.dtype(in_np).itemsize
    bufs = []
    ptrs = []
    for r in rows:
        b = ctx.alloc((n + offset_elems) * isz + 16)
        bufs.append(b)
        p = b.ptr + offset_elems * isz
        ctx.h2d_ptr(p, r.ctypes.data, r.nbytes)
        ptrs.append(p)
    asz = acc_np.itemsize
    ob = ctx.alloc((n + offset_elems) * asz + 16)
    optr = ob.ptr + offset_elems * asz
    acc_ptr = None
    if acc_in is not None:
        ctx.h2d_ptr(optr, acc_in.ctypes.data, acc_in.nbytes)
        acc_ptr = optr
    ctx.accumulate(ptrs, weights, n, optr, fedavg_dtype(in_np), fedavg_dtype(acc_np), op, fin, count, acc_in_ptr=acc_ptr)
    out = np.empty(n, dtype=acc_np)
    ctx.d2h(out, optr)
    for b in bufs + [ob]:
        b.close()
    return out


def _sum(ws):
    c = None
    for w in ws:
        c = w if c is None else c + w
    return c


OPS = [("numpy", 0, 1), ("torch", 1, 2), ("unweighted", 2, 1)]


@pytest.mark.parametrize("K", [1, 2, 7, 8, 9, 17, 64, 129, 200])
@pytest.mark.parametrize("n", [1, 3, 4, 5, 257, 65539])
@pytest.mark.parametrize("opname,op,fin", OPS, ids=[o[0] for o in OPS])
def test_kernel_f32_vs_oracle(ctx, oracle, K, n, opname, op, fin):
    rng = np.random.default_rng(K * 1000 + n)
    rows = [rng.standard_normal(n).astype(np.float32) for _ in range(K)]
    ws = [float(rng.random() * rng.integers(1, 50)) for _ in range(K)]
    omode = oracle.MODE_TORCH if op == 1 else oracle.MODE_NUMPY
    exp = oracle.fedavg_c(rows, ws, omode, weighted=(op != 2), fin=fin, count=_sum(ws))
    got = _run_kernel(ctx, rows, ws, op, fin, _sum(ws))
    assert same_bits(got, exp)


@pytest.mark.parametrize("offset", [1, 2, 3])
def test_kernel_unaligned_rows_use_generic_path(ctx, oracle, offset):
    rng = np.random.default_rng(offset)
    rows = [rng.standard_normal(1001).astype(np.float32) for _ in range(5)]
    ws = [0.5, 1.5, 2.25, 3.0, 0.125]
    for op, fin, mode in ((0, 1, oracle.MODE_NUMPY), (1, 2, oracle.MODE_TORCH)):
        exp = oracle.fedavg_c(rows, ws, mode, fin=fin)
        got = _run_kernel(ctx, rows, ws, op, fin, _sum(ws), offset_elems=offset)
        assert same_bits(got, exp)


def test_kernel_acc_in_continuation(ctx, oracle):
    rng = np.random.default_rng(5)
    rows = [rng.standard_normal(10007).astype(np.float32) for _ in range(140)]
    ws = [float(1 + (37 * k) % 100) for k in range(140)]
    for op, fin, mode in ((0, 1, oracle.MODE_NUMPY), (1, 2, oracle.MODE_TORCH)):
        full = oracle.fedavg_c(rows, ws, mode, fin=fin)
        part = _run_kernel(ctx, rows[:50], ws[:50], op, 0, 0.0)
        got = _run_kernel(ctx, rows[50:], ws[50:], op, fin, _sum(ws), acc_in=part)
        assert same_bits(got, full)
        # pure finalisation (k_rows = 0) of a folded sum
        acc = _run_kernel(ctx, rows, ws, op, 0, 0.0)
        got = _run_kernel(ctx, [], [], op, fin, _sum(ws), acc_in=acc)
        assert same_bits(got, full)


@pytest.mark.parametrize("in_dt,acc_dt", [(np.float64, np.float64), (np.float32, np.float64), (np.int64, np.float64),
                                          (np.int32, np.float64), (np.int64, np.float32), (np.int32, np.float32)])
def test_kernel_generic_dtypes(ctx, oracle, in_dt, acc_dt):
    rng = np.random.default_rng(11)
    if np.dtype(in_dt).kind == "i":
        rows = [rng.integers(-(2 ** 40) if in_dt == np.int64 else -(2 ** 30), 2 ** 30, 999).astype(in_dt) for _ in range(6)]
    else:
        rows = [rng.standard_normal(999).astype(in_dt) for _ in range(6)]
    ws = [0.3, 1.7, 2.0, 5.5, 0.01, 9.0]
    conv = [r.astype(acc_dt) for r in rows]
    for op, fin, mode in ((0, 1, oracle.MODE_NUMPY), (1, 2, oracle.MODE_TORCH)):
        exp = oracle.fedavg_c(conv, ws, mode, fin=fin)
        got = _run_kernel(ctx, rows, ws, op, fin, _sum(ws), out_dtype=acc_dt)
        assert same_bits(got, exp)


PRODUCT_VARIANTS = (0, 4, 16, 64, 20, 80)  # fedavg_internal.h kVariantProductMask: bits 2, 4 and 6


def _product_form(variant=0, unroll=0, tile=4096):
    return (variant & ~84) == 0 and unroll in (0, 4) and tile == 4096


@pytest.fixture(scope="module")
def ab(ctx):
    """Whether the library is an A/B build (tools/build_rev_lib.py): the product library carries only routed forms."""
    return ctx.ab_build()


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 8, 16, 32])
@pytest.mark.parametrize("bpc,unroll,tile", [(1, 4, 1024), (2, 8, 2048), (4, 4, 4096), (8, 8, 8192), (2, 4, 4096),
                                             (0, 0, 4096), (1, 8, 4096)])
def test_launch_variants_same_bits(ctx, oracle, ab, bpc, unroll, tile, variant):
    if not ab and not _product_form(variant, unroll, tile):
        pytest.skip("an A/B form: tools/build_rev_lib.py builds the library that carries it")
    rng = np.random.default_rng(21)
    n = 300_001 + variant  # whole tiles on the streaming kernel + a ragged tail on the scalar kernel
    rows = [rng.standard_normal(n).astype(np.float32) for _ in range(33)]
    ws = [float(1 + (37 * k) % 100) for k in range(33)]
    for op, fin, mode in ((1, 2, oracle.MODE_TORCH), (0, 1, oracle.MODE_NUMPY)):
        exp = oracle.fedavg_c(rows, ws, mode, fin=fin, nthreads=4)
        ctx.set_launch(bpc, unroll)
        ctx.set_variant(variant)
        ctx.set_tile(tile)
        try:
            got = _run_kernel(ctx, rows, ws, op, fin, _sum(ws))
        finally:
            ctx.set_launch(0, 0)
            ctx.set_variant(0)
            ctx.set_tile(0)
        assert same_bits(got, exp)


@pytest.mark.parametrize("K,bpc,variant", [(20, 0, 0), (7, 0, 0), (20, 3, 0), (131, 0, 0), (1, 0, 0), (2, 0, 0),
                                           (129, 0, 0), (1, 0, 256), (2, 0, 256), (3, 0, 256), (3, 0, 384), (4, 0, 0),
                                           (5, 0, 0), (8, 0, 0), (8, 0, 128), (9, 0, 0), (130, 0, 256), (136, 0, 0)])
def test_burst_many_launches(ctx, oracle, ab, K, bpc, variant):
    """The default (burst) kernel issues one launch per grid x 8 tiles: more tiles than one launch covers,
    a last launch with fewer tiles than blocks, a sub-range starting and ending inside tiles, more than
    128 clients (chained through the output), against the oracle bit for bit.  One and two clients, and a
    chained last chunk of one client (129), take the per-tile-store kernel (fedavg_capi.cpp kBurstMinClients);
    variant bit 8 keeps them on the burst form.  1-8 clients per launch (a chained last chunk of 1-8: 129-136) take
    the burst kernel with the client count built in (tile_sum_kc, round 4); bit 7 the runtime-K loop."""
    if not ab and not _product_form(variant):
        pytest.skip("an A/B form: tools/build_rev_lib.py builds the library that carries it")
    n = 2048 * 4096 * 2 + 12345
    rows = [oracle.synth_values(5, k, np.arange(n, dtype=np.uint64)) for k in range(K)]
    ws = oracle.synth_weights(K)
    ctx.set_launch(bpc, 0)
    ctx.set_variant(variant)
    try:
        for op, fin, mode in ((1, 2, oracle.MODE_TORCH), (0, 1, oracle.MODE_NUMPY)):
            exp = oracle.fedavg_c(rows, ws, mode, fin=fin, nthreads=8)
            got = _run_kernel(ctx, rows, ws, op, fin, _sum(ws))
            assert same_bits(got, exp)
        # a sub-range [lo, hi) through the tiled entry point (contiguous rows: tile stride == tile): only it
        # is written, the sentinel around it stays
        lo, hi = 4096 * 3 + 100, (n - 4096 * 5 - 36) // 4 * 4
        n_alloc = (n + 4095) // 4096 * 4096
        bufs = [ctx.alloc(n_alloc * 4) for _ in rows]
        for b, r in zip(bufs, rows):
            ctx.h2d_ptr(b.ptr, r.ctypes.data, r.nbytes)
        out = ctx.alloc(n_alloc * 4)
        sentinel = np.full(n, -7.0, np.float32)
        ctx.h2d_ptr(out.ptr, sentinel.ctypes.data, sentinel.nbytes)
        ctx.accumulate_tiled([b.ptr for b in bufs], ws, 4096, 4096, lo, hi, out.ptr, 1, 2, _sum(ws))
        got = np.empty(n, np.float32)
        ctx.d2h(got, out.ptr)
        exp = oracle.fedavg_c([r[lo:hi] for r in rows], ws, oracle.MODE_TORCH, fin=2, nthreads=8)
        assert same_bits(got[lo:hi], exp)
        assert np.all(got[:lo] == -7.0) and np.all(got[hi:] == -7.0)
        for b in bufs + [out]:
            b.close()
    finally:
        ctx.set_launch(0, 0)
        ctx.set_variant(0)


def test_large_k64(ctx, oracle):
    """64 clients x (4M + 3) params: the bench's K at a size the oracle finishes in seconds."""
    K, n = 64, (1 << 22) + 3
    rows = [oracle.synth_values(3, k, np.arange(n, dtype=np.uint64)) for k in range(K)]
    ws = oracle.synth_weights(K)
    for op, fin, mode in ((1, 2, oracle.MODE_TORCH), (0, 1, oracle.MODE_NUMPY)):
        exp = oracle.fedavg_c(rows, ws, mode, fin=fin, nthreads=8)
        got = _run_kernel(ctx, rows, ws, op, fin, _sum(ws))
        assert same_bits(got, exp)


def test_synthetic_generator_matches_host(ctx, oracle):
    n = 1_000_003
    b = ctx.alloc(n * 4)
    ctx.fill_synthetic_f32(b.ptr, n, 9, 5, 123)
    dev = np.empty(n, dtype=np.float32)
    ctx.d2h(dev, b.ptr)
    host = oracle.synth_values(9, 5, np.arange(123, 123 + n, dtype=np.uint64))
    assert np.array_equal(dev.view(np.uint32), host.view(np.uint32))
    idx = np.array([0, 7, n - 1, 4242], dtype=np.uint64)
    assert np.array_equal(ctx.gather_f32(b.ptr, idx), host[idx.astype(np.int64)])
    b.close()


def test_timing_events(ctx):
    n = 1 << 20
    bufs = [ctx.alloc(n * 4) for _ in range(4)]
    for i, b in enumerate(bufs):
        ctx.fill_synthetic_f32(b.ptr, n, 1, i, 0)
    ctx.set_timing(True)
    try:
        ctx.accumulate([b.ptr for b in bufs[:3]], [1.0, 2.0, 3.0], n, bufs[3].ptr, 0, 0, 1, 2, 6.0)
        ms = ctx.last_kernel_ms()
    finally:
        ctx.set_timing(False)
    assert 0.0 < ms < 1000.0
    for b in bufs:
        b.close()


@pytest.mark.parametrize("tile", [1024, 2048, 4096, 8192])
@pytest.mark.parametrize("K,slots", [(13, 16), (16, 16), (24, 24), (130, 130)])
@pytest.mark.parametrize("begin,end", [(0, None), (64, None), (4096 + 128, 3 * 4096 - 64), (8, 12)])
def test_tiled_slab_vs_oracle(ctx, oracle, ab, tile, K, slots, begin, end):
    """Tiled slab (clients interleaved per tile), permuted arrival order, sub-ranges that start and end
    mid-tile (only [begin, end) of the flat output is written), >128 clients chained through the output."""
    from nvflare_amd.device import TiledLayout

    if not ab and not _product_form(tile=tile):
        pytest.skip("tile widths other than 4096 are A/B forms (tools/build_rev_lib.py)")

    n = 7 * 4096 + 1024 + 12  # ragged last tile
    end = n if end is None else end
    lay = TiledLayout(tile, slots)
    slab = ctx.alloc(lay.slab_elems(n) * 4)
    for s_ in range(slots):
        ctx.fill_synthetic_f32(slab.ptr + lay.slot_offset_elems(s_) * 4, n, 77, s_, 5, tile, lay.tile_stride)
    order = [int(x) for x in np.random.default_rng(tile + K).permutation(slots)[:K]]
    ws = [0.25 + 1.5 * j for j in range(K)]
    rows = [oracle.synth_values(77, s_, np.arange(5, 5 + n, dtype=np.uint64)) for s_ in order]
    bases = [slab.ptr + lay.slot_offset_elems(s_) * 4 for s_ in order]
    out = ctx.alloc(n * 4 + 64)
    sentinel = np.full(n, 12345.0, np.float32)
    try:
        for op, fin, mode in ((1, 2, oracle.MODE_TORCH), (0, 1, oracle.MODE_NUMPY), (2, 1, oracle.MODE_NUMPY)):
            ctx.h2d_ptr(out.ptr, sentinel.ctypes.data, sentinel.nbytes)
            e4 = (end + 3) // 4 * 4
            ctx.accumulate_tiled(bases, ws, tile, lay.tile_stride, begin, e4, out.ptr, op, fin, _sum(ws))
            got = np.empty(n, np.float32)
            ctx.d2h(got, out.ptr)
            exp = oracle.fedavg_c(rows, ws, mode, weighted=(op != 2), fin=fin, nthreads=4)
            assert same_bits(got[begin:e4], exp[begin:e4]), (op, fin)
            assert np.all(got[:begin] == 12345.0) and np.all(got[e4:] == 12345.0)
    finally:
        slab.close()
        out.close()


@pytest.mark.parametrize("tile", [1024, 4096])
def test_h2d_tiled_staging(ctx, oracle, ab, tile):
    """Host arrays staged into tiled slots at arbitrary (4-aligned) logical offsets, pageable and pinned."""
    from nvflare_amd.device import TiledLayout

    if not ab and not _product_form(tile=tile):
        pytest.skip("tile widths other than 4096 are A/B forms (tools/build_rev_lib.py)")

    K, slots, n = 5, 8, 3 * tile + 100
    lay = TiledLayout(tile, slots)
    slab = ctx.alloc(lay.slab_elems(n) * 4)
    rng = np.random.default_rng(tile)
    rows = [rng.standard_normal(n).astype(np.float32) for _ in range(K)]
    cuts = [0, 4, tile - 4, tile + 36, 2 * tile, n]
    for k, r in enumerate(rows):
        base = slab.ptr + lay.slot_offset_elems(k) * 4
        for a, b in zip(cuts[:-1], cuts[1:]):  # staged piecewise, like several keys of one client
            piece = np.ascontiguousarray(r[a:b])
            if k % 2:
                piece = torch.from_numpy(piece).pin_memory().numpy()
            ctx.h2d_tiled(base, tile * 4, lay.tile_stride * 4, a * 4, piece.ctypes.data, piece.nbytes)
    ws = [1.0, 2.5, 0.125, 7.0, 3.0]
    out = ctx.alloc(n * 4 + 64)
    e4 = (n + 3) // 4 * 4
    ctx.accumulate_tiled([slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)], ws, tile, lay.tile_stride, 0, e4,
                         out.ptr, 1, 2, _sum(ws))
    got = np.empty(n, np.float32)
    ctx.d2h(got, out.ptr)
    assert same_bits(got, oracle.fedavg_c(rows, ws, oracle.MODE_TORCH))
    slab.close()
    out.close()


def test_d2d_tiled_staging_from_torch(ctx, oracle):
    from nvflare_amd.device import TiledLayout

    tile, K, n = 4096, 3, 2 * 4096 + 8
    lay = TiledLayout(tile, K)
    slab = ctx.alloc(lay.slab_elems(n) * 4)
    rows = [torch.randn(n, generator=torch.Generator().manual_seed(k)) for k in range(K)]
    for k, r in enumerate(rows):
        t = r.to("cuda:0")
        torch.cuda.synchronize()
        ctx.d2d_tiled(slab.ptr + lay.slot_offset_elems(k) * 4, tile * 4, lay.tile_stride * 4, 0, t.data_ptr(), t.numel() * 4)
    ws = [0.5, 1.5, 2.0]
    out = ctx.alloc(n * 4)
    ctx.accumulate_tiled([slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)], ws, tile, lay.tile_stride, 0, n,
                         out.ptr, 0, 1, _sum(ws))
    got = np.empty(n, np.float32)
    ctx.d2h(got, out.ptr)
    assert same_bits(got, oracle.fedavg_c([r.numpy() for r in rows], ws, oracle.MODE_NUMPY))
    slab.close()
    out.close()


@pytest.mark.parametrize("slots", [1, 2, 3])
def test_engine_multi_slab_chaining(oracle, slots):
    """Few slots per slab: a round spans several slabs (launches chained through the accumulator) and the
    next round is consolidated into one slab -- bits unchanged either way."""
    from nvflare_amd.engine import DeviceFedAvg

    rng = np.random.default_rng(slots)
    K = 7
    eng = DeviceFedAvg(slab_slots=slots)
    for rnd in range(2):
        rows = [rng.standard_normal(10_000 + 3).astype(np.float32) for _ in range(K)]
        ws = [float(1 + k) for k in range(K)]
        for k in range(K):
            eng.add([("w", rows[k])], ws[k], True)
        got = eng.result()["w"]
        eng.reset()
        assert same_bits(got, oracle.fedavg_c(rows, ws, oracle.MODE_NUMPY))
    assert eng.stats["slabs_allocated"] >= 1
    eng.release()


def test_h2d_tiled_multi_many_keys_split_across_slots(ctx, oracle):
    """~240 MB per client in 211 keys: pieces split at every 64 MiB ring-slot boundary, the remainder opening
    the next slot with later keys packed behind it; bit-exact aggregation of every key."""
    from nvflare_amd.device import TiledLayout

    tile, K = 4096, 2
    sizes = [300_017 - 13 * (j % 7) for j in range(211)]
    offs, off = [], 0
    for n in sizes:
        offs.append(off)
        off += (n + 63) // 64 * 64
    n_total = off
    lay = TiledLayout(tile, K)
    slab = ctx.alloc(lay.slab_elems(n_total) * 4)
    rng = np.random.default_rng(4)
    flat = [rng.standard_normal(sum(sizes)).astype(np.float32) for _ in range(K)]
    clients = []
    for k in range(K):
        parts, o = [], 0
        for n in sizes:
            parts.append(flat[k][o:o + n])
            o += n
        clients.append(parts)
        ctx.h2d_tiled_multi(slab.ptr + lay.slot_offset_elems(k) * 4, tile * 4, lay.tile_stride * 4,
                            [(oo * 4, a.ctypes.data, a.nbytes) for oo, a in zip(offs, parts)])
    ws = [3.0, 1.5]
    out = ctx.alloc(n_total * 4)
    ctx.accumulate_tiled([slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)], ws, tile, lay.tile_stride, 0,
                         n_total, out.ptr, 1, 2, _sum(ws))
    got = np.empty(n_total, np.float32)
    ctx.d2h(got, out.ptr)
    exp = oracle.fedavg_c([np.concatenate(c) for c in clients], ws, oracle.MODE_TORCH, nthreads=4)
    o = 0
    for oo, n in zip(offs, sizes):
        assert same_bits(got[oo:oo + n], exp[o:o + n]), oo
        o += n
    slab.close()
    out.close()


def test_h2d_tiled_multi_packs_keys(ctx, oracle):
    """Many keys of one client staged in one call: pieces spanning ring-slot boundaries (> 64 MiB),
    zero-length pieces, gaps, pageable and pinned sources."""
    from nvflare_amd.device import TiledLayout

    tile, K = 4096, 3
    sizes = [5, 0, 4096, 17 * 1024 * 1024 + 3, 64, 1, 3 * 4096 + 7]  # one piece larger than a ring slot
    offs, off = [], 0
    for n in sizes:
        offs.append(off)
        off += (n + 63) // 64 * 64
    n_total = off
    lay = TiledLayout(tile, K)
    slab = ctx.alloc(lay.slab_elems(n_total) * 4)
    rng = np.random.default_rng(3)
    clients = [[rng.standard_normal(n).astype(np.float32) for n in sizes] for _ in range(K)]
    for k, arrs in enumerate(clients):
        srcs = [a if k != 1 else torch.from_numpy(a).pin_memory().numpy() for a in arrs]
        ctx.h2d_tiled_multi(slab.ptr + lay.slot_offset_elems(k) * 4, tile * 4, lay.tile_stride * 4,
                            [(o * 4, a.ctypes.data, a.nbytes) for o, a in zip(offs, srcs)])
    ws = [0.5, 2.0, 1.25]
    out = ctx.alloc(n_total * 4)
    ctx.accumulate_tiled([slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)], ws, tile, lay.tile_stride, 0,
                         n_total, out.ptr, 0, 1, _sum(ws))
    got = np.empty(n_total, np.float32)
    ctx.d2h(got, out.ptr)  # > 8 MiB: drained through the pinned ring
    for j, (o, n) in enumerate(zip(offs, sizes)):
        if n:
            exp = oracle.fedavg_c([clients[k][j] for k in range(K)], ws, oracle.MODE_NUMPY)
            assert same_bits(got[o:o + n], exp), j
    slab.close()
    out.close()


@pytest.mark.parametrize("K", [1, 2, 3, 4])
@pytest.mark.parametrize("form", [0, 1, 2, 3, 4, 5, 6, 7])
def test_few_client_burst_forms(ctx, oracle, ab, K, form):
    """The few-client burst kernel (fedavg_tiles.h fedavg_tiles_few_f32x4; 1-3 client reads, no chained sum): several
    launches and a short last one (15 001 tiles against 6144 per launch at the default form), every load unconditional
    (a launch's slots past its last tile re-read that tile, nothing past it is stored), a ragged end, a sub-range
    starting and ending inside tiles with a sentinel around it; numpy and torch modes, bit for bit.  Forms 1-7 (launch
    variant bits 9-11, A/B builds) are the sweeps' geometries (fedavg_internal.h kFewAB, kFewAB34; 4 reads only there)
    and, at 3-4 clients, the burst form's built-in count (6) and remainder form (7)."""
    if K == 4 and form == 0:
        pytest.skip("4 client reads take the burst form (test_burst_many_launches)")
    if K <= 2 and form == 7:
        pytest.skip("no seventh few-client geometry at 1-2 reads")
    if form:
        from nvflare_amd._native import FedAvgError

        try:  # A/B builds, or a product build with -DFEDAVG_AB_FEW (tools/build_rev_lib.py --product)
            ctx.set_variant(form << 9)
        except FedAvgError:
            pytest.skip("an A/B form: tools/build_rev_lib.py builds the library that carries it")
        ctx.set_variant(0)
    n = 15_001 * 4096 - 4092
    cols = np.arange(n, dtype=np.uint64)
    rows = [oracle.synth_values(17, k, cols) for k in range(K)]
    ws = oracle.synth_weights(K)
    n_alloc = (n + 4095) // 4096 * 4096
    bufs = [ctx.alloc(n_alloc * 4) for _ in rows]
    out = ctx.alloc(n_alloc * 4)
    ctx.set_variant(form << 9)
    try:
        for b, r in zip(bufs, rows):
            ctx.h2d_ptr(b.ptr, r.ctypes.data, r.nbytes)
        got = np.empty(n, np.float32)
        for op, fin, mode in ((1, 2, oracle.MODE_TORCH), (0, 1, oracle.MODE_NUMPY)):
            exp = oracle.fedavg_c(rows, ws, mode, fin=fin, nthreads=8)
            n0 = ctx.launch_count()
            ctx.accumulate_tiled([b.ptr for b in bufs], ws, 4096, 4096, 0, (n + 3) // 4 * 4, out.ptr, op, fin, _sum(ws))
            assert ctx.launch_count() - n0 >= 2  # several launches, the last partial
            ctx.d2h(got, out.ptr)
            assert same_bits(got, exp), (K, form, mode)
        lo, hi = 4096 * 7 + 36, n - 4096 * 3 - 100
        sentinel = np.full(n, -7.0, np.float32)
        ctx.h2d_ptr(out.ptr, sentinel.ctypes.data, sentinel.nbytes)
        ctx.accumulate_tiled([b.ptr for b in bufs], ws, 4096, 4096, lo, hi, out.ptr, 1, 2, _sum(ws))
        ctx.d2h(got, out.ptr)
        exp = oracle.fedavg_c([r[lo:hi] for r in rows], ws, oracle.MODE_TORCH, fin=2, nthreads=8)
        assert same_bits(got[lo:hi], exp)
        assert np.all(got[:lo] == -7.0) and np.all(got[hi:] == -7.0)
    finally:
        ctx.set_variant(0)
        for b in bufs + [out]:
            b.close()


def test_product_library_refuses_ab_forms(ctx, ab):
    """The product library carries only the routed kernel forms (round 5): the A/B launch variants, unroll 8 and other
    tile widths are refused with an error, not run on some other form."""
    from nvflare_amd._native import FedAvgError

    if ab:
        pytest.skip("an A/B build accepts them")
    for v in (1, 2, 8, 32, 128, 256, 1 << 9, 3 << 9):
        with pytest.raises(FedAvgError, match="A/B"):
            ctx.set_variant(v)
    for v in PRODUCT_VARIANTS:
        ctx.set_variant(v)
    ctx.set_variant(0)
    with pytest.raises(FedAvgError, match="A/B"):
        ctx.set_launch(0, 8)
    for t in (1024, 2048, 8192):
        with pytest.raises(FedAvgError, match="A/B"):
            ctx.set_tile(t)
    ctx.set_launch(0, 0)
    ctx.set_tile(0)
