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
    assert h.engine.stats["folds"] >= 1


@pytest.mark.parametrize("case", [c for c in HCASES if c["container"] == "torch"][:4],
                         ids=[c["name"] for c in HCASES if c["container"] == "torch"][:4])
def test_helper_device_tensors(case):
    """torch tensors already on the GPU: staged D2D, result returned as a device tensor."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    h = WeightedAggregationHelper(exclude_vars=case["exclude_vars"], weigh_by_local_iter=case["weigh_by_local_iter"])
    for c in case["contributions"]:
        h.add({k: _container(ARRAYS[n], "torch", "cuda:0") for k, n in c["data"].items()}, c["weight"], c["name"], 0)
    out = h.get_result()
    for k, name in case["expected"].items():
        assert out[k].device.type == "cuda"
        assert same_bits(_as_numpy(out[k]).reshape(ARRAYS[name].shape), ARRAYS[name]), k


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


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("bpc,unroll", [(1, 4), (2, 8), (4, 16), (8, 8), (16, 4)])
def test_launch_variants_same_bits(ctx, oracle, bpc, unroll, variant):
    rng = np.random.default_rng(21)
    n = 300_001 + variant  # ragged tiles for the 2-column variants too
    rows = [rng.standard_normal(n).astype(np.float32) for _ in range(33)]
    ws = [float(1 + (37 * k) % 100) for k in range(33)]
    for op, fin, mode in ((1, 2, oracle.MODE_TORCH), (0, 1, oracle.MODE_NUMPY)):
        exp = oracle.fedavg_c(rows, ws, mode, fin=fin, nthreads=4)
        ctx.set_launch(bpc, unroll)
        ctx.set_variant(variant)
        try:
            got = _run_kernel(ctx, rows, ws, op, fin, _sum(ws))
        finally:
            ctx.set_launch(0, 0)
            ctx.set_variant(0)
        assert same_bits(got, exp)


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
    ctx.fill_synthetic_f32(b.ptr, n, seed=9, row=5, col0=123)
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
        ctx.fill_synthetic_f32(b.ptr, n, 1, i)
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
@pytest.mark.parametrize("variant", [0, 2, 4, 6])
@pytest.mark.parametrize("K,unroll", [(13, 8), (16, 4), (16, 8), (24, 8)])
@pytest.mark.parametrize("seg_pad,tile_pad", [(0, 0), (64, 1040)])
def test_tiled_slab_vs_oracle(ctx, oracle, tile, variant, K, unroll, seg_pad, tile_pad):
    """Tiled slab layout (client segments interleaved per tile) with a permuted arrival order; variants 4/6
    take the software-pipelined kernel when K % unroll == 0 (and include grid-stride tile reuse)."""
    from nvflare_amd.device import TiledLayout

    n = 7 * 4096 + 1024 + 12  # ragged last tile
    lay = TiledLayout(tile, 24, seg_pad, tile_pad)
    k_max = lay.k_max
    slab = ctx.alloc(lay.slab_elems(n) * 4)
    ctx.fill_synthetic_tiled_f32(slab.ptr, lay, n, 77, 5)
    order = [int(x) for x in np.random.default_rng(tile).permutation(k_max)[:K]]
    ws = [0.25 + 1.5 * j for j in range(K)]
    rows = [oracle.synth_values(77, s, np.arange(5, 5 + n, dtype=np.uint64)) for s in order]
    out = ctx.alloc(n * 4)
    ctx.set_variant(variant)
    ctx.set_launch(1 if variant & 4 else 0, unroll)  # few blocks: several tiles per block
    try:
        for op, fin, mode in ((1, 2, oracle.MODE_TORCH), (0, 1, oracle.MODE_NUMPY), (2, 1, oracle.MODE_NUMPY)):
            ctx.accumulate_tiled(slab.ptr, lay, order, ws, n, out.ptr, op, fin, _sum(ws))
            got = np.empty(n, np.float32)
            ctx.d2h(got, out.ptr)
            exp = oracle.fedavg_c(rows, ws, mode, weighted=(op != 2), fin=fin)
            assert same_bits(got, exp), (op, fin)
    finally:
        ctx.set_variant(0)
        ctx.set_launch(0, 0)
        slab.close()
        out.close()
