"""Dequantisation on the GPU (row f4): the kernel vs the oracle for every format, the drop-in filter vs the
reference's own AdaQuantizer round trips, and quantized contributions staged lazily through the
aggregator (compressed bytes over PCIe, dequantized into the slab slot) vs the eager path -- bit-exact."""

import bz2

import numpy as np
import pytest
import torch

from golden_util import adaquant_state, load_quant_golden, same_bits
from nvflare_amd import _native as N
from nvflare_amd.app_common.aggregators import InTimeAccumulateWeightedAggregator
from nvflare_amd.app_opt.pt.quantization import ModelDequantizer
from nvflare_amd.compat import DXO, AppConstants, DataKind, EventType, FLContext, MetaKey, ReservedKey, Shareable
from nvflare_amd.device import DeviceContext, TiledLayout
from nvflare_amd.quantized import QuantizedPayload

pytestmark = pytest.mark.gpu
QM, QA = load_quant_golden()


@pytest.fixture(scope="module")
def ctx():
    return DeviceContext.get(0)


def _random_payload(rng, qt, n, bs=64):
    nb = (n + bs - 1) // bs
    kw = {}
    if qt == N.FEDAVG_Q_F16:
        q = rng.standard_normal(n).astype(np.float16).view(np.uint16)
    elif qt == N.FEDAVG_Q_BF16:
        q = (rng.standard_normal(n).astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
    elif qt == N.FEDAVG_Q_BLOCKWISE8:
        q = rng.integers(0, 256, n).astype(np.uint8)
        kw = dict(absmax=(rng.random(nb) * 2).astype(np.float32), code=np.sort(rng.standard_normal(256)).astype(np.float32),
                  blocksize=bs)
    elif qt in (N.FEDAVG_Q_FP4, N.FEDAVG_Q_NF4):
        q = rng.integers(0, 256, (n + 1) // 2).astype(np.uint8)
        kw = dict(absmax=(rng.random(nb) * 2).astype(np.float32), blocksize=bs)
    elif qt == N.FEDAVG_Q_ADA_U8:
        q = rng.integers(0, 256, n).astype(np.uint8)
        kw = dict(norm=6.25, level=255.0, offset=3.1)
    else:
        q = rng.integers(0, 4096, n).astype(np.uint16)
        kw = dict(norm=2205.77, level=4095.0, offset=1054.18)
    return q, kw


QTYPES = [N.FEDAVG_Q_F16, N.FEDAVG_Q_BF16, N.FEDAVG_Q_BLOCKWISE8, N.FEDAVG_Q_FP4, N.FEDAVG_Q_NF4,
          N.FEDAVG_Q_ADA_U8, N.FEDAVG_Q_ADA_U16]


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("n", [1, 7, 4096, 100_003])
def test_kernel_matches_oracle_flat(oracle, qt, n):
    rng = np.random.default_rng(qt * 1000 + n)
    q, kw = _random_payload(rng, qt, n)
    p = QuantizedPayload(qt, q, (n,), "numpy", **kw)
    got = p.materialize()
    ref = oracle.dequantize(qt, q, n, **kw)
    assert same_bits(got, ref)


@pytest.mark.parametrize("qt", [N.FEDAVG_Q_BLOCKWISE8, N.FEDAVG_Q_NF4, N.FEDAVG_Q_ADA_U16])
def test_kernel_tiled_slot_with_offset(ctx, oracle, qt):
    """Into slot 2 of a 3-client slab at logical offset 4100 -- the aggregation staging path."""
    rng = np.random.default_rng(qt)
    n, off, S = 9000, 4100, 3
    lay = TiledLayout(4096, S)
    total = off + n
    slab = ctx.alloc(lay.slab_elems(total) * 4)
    try:
        ctx.memset(slab.ptr, 0, lay.slab_elems(total) * 4)
        q, kw = _random_payload(rng, qt, n, bs=128)
        p = QuantizedPayload(qt, q, (n,), "numpy", **kw)
        from nvflare_amd.quantized import stager

        base = slab.ptr + lay.slot_offset_elems(2) * 4
        stager().dequantize_into(ctx, p, base, lay.tile, lay.tile_stride, off)
        host = np.empty(lay.slab_elems(total), np.float32)
        ctx.d2h(host, slab.ptr)
        idx = np.arange(off, off + n)
        phys = lay.slot_offset_elems(2) + (idx // 4096) * lay.tile_stride + idx % 4096
        assert same_bits(host[phys], oracle.dequantize(qt, q, n, **kw))
        mask = np.ones(host.size, bool)
        mask[phys] = False
        assert not host[mask].any()  # nothing else written
    finally:
        slab.close()


@pytest.mark.parametrize("container", ["numpy", "torch"])
def test_filter_adaquant_matches_reference(container):
    f = ModelDequantizer()
    params, qstate, srcdt, expect = {}, {}, {}, {}
    for c in QM["cases"]:
        q = QA[c["quantized"]]
        params[c["name"]] = torch.from_numpy(q.copy()) if container == "torch" else q.copy()
        st = adaquant_state(c, QA)
        if container == "torch" and "compressed_tensor" in st:
            st["compressed_tensor"] = st["compressed_tensor"]  # numpy in either case (ada_quant.py:61)
        qstate[c["name"]] = st
        srcdt[c["name"]] = "float32"
        expect[c["name"]] = QA[c["expected"]]
    dxo = DXO(DataKind.WEIGHTS, data=params, meta={MetaKey.PROCESSED_ALGORITHM: "adaquant", "quant_state": qstate,
                                                   "source_datatype": srcdt, "quantized_flag": True})
    out = f.process_dxo(dxo, dxo.to_shareable(), FLContext()).data
    for k, ref in expect.items():
        got = out[k]
        if container == "torch":
            assert isinstance(got, torch.Tensor) and got.dtype == torch.float32
            got = got.numpy()
        else:
            assert isinstance(got, np.ndarray) and got.dtype == np.float32
        assert same_bits(got, ref), k


def _client_shareables(rng, n_clients, qtype, container):
    """Quantized WEIGHT_DIFF results as clients would send them (several keys, ragged sizes)."""
    sizes = {"conv.weight": (64, 3, 3, 3), "fc.weight": (1000, 37), "fc.bias": (1000,), "big": (70_001,)}
    out = []
    for c in range(n_clients):
        params, qstate, srcdt = {}, {}, {}
        for k, shp in sizes.items():
            n = int(np.prod(shp))
            if qtype == "float16":
                v = rng.standard_normal(shp).astype(np.float16)
                st = {}
            elif qtype == "blockwise8":
                v = rng.integers(0, 256, shp).astype(np.uint8)
                st = {"absmax": (rng.random((n + 4095) // 4096) + 0.5).astype(np.float32),
                      "code": np.sort(rng.standard_normal(256)).astype(np.float32)}
            else:  # normfloat4
                v = rng.integers(0, 256, ((n + 1) // 2, 1)).astype(np.uint8)
                st = {"absmax": (rng.random((n + 63) // 64) + 0.5).astype(np.float32), "blocksize": 64,
                      "quant_map": np.zeros(16, np.float32), "dtype": "float32", "shape": list(shp), "quant_type": "nf4"}
            params[k] = torch.from_numpy(v) if container == "torch" else v
            qstate[k], srcdt[k] = st, "float32"
        dxo = DXO(DataKind.WEIGHT_DIFF, data=params, meta={MetaKey.PROCESSED_ALGORITHM: qtype, "quant_state": qstate,
                                                          "source_datatype": srcdt, "quantized_flag": True,
                                                          "NUM_STEPS_CURRENT_ROUND": 1 + 3 * c})
        s = dxo.to_shareable()
        s.set_peer_props({ReservedKey.IDENTITY_NAME: f"site-{c}"})
        s.add_cookie(AppConstants.CONTRIBUTION_ROUND, 0)
        out.append(s)
    return out


def _aggregate(shareables, lazy):
    import copy

    f = ModelDequantizer(lazy=lazy)
    agg = InTimeAccumulateWeightedAggregator(expected_data_kind=DataKind.WEIGHT_DIFF, device=0)
    ctx = FLContext()
    ctx.set_prop(AppConstants.CURRENT_ROUND, 0)
    agg.handle_event(EventType.START_RUN, ctx)
    for s in shareables:
        s2 = f.process(copy.deepcopy(s), ctx)
        assert agg.accept(s2, ctx)
    from nvflare_amd.compat import from_shareable

    return from_shareable(agg.aggregate(ctx)).data


@pytest.mark.parametrize("qtype", ["float16", "blockwise8", "normfloat4"])
@pytest.mark.parametrize("container", ["numpy", "torch"])
def test_lazy_staging_equals_eager(qtype, container):
    rng = np.random.default_rng(7)
    sh = _client_shareables(rng, 5, qtype, container)
    eager = _aggregate(sh, lazy=False)
    lazy = _aggregate(sh, lazy=True)
    assert set(eager) == set(lazy)
    for k in eager:
        a, b = eager[k], lazy[k]
        if container == "torch":
            assert isinstance(b, torch.Tensor)
            a, b = a.numpy(), b.numpy()
        assert same_bits(a, b), k
