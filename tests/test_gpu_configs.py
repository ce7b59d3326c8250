"""Parity at the sizes of BASELINE.json configs 2 and 4 (configs[1], configs[3]).

* Config 2 -- 8 clients x 125M fp32 on one GPU -- runs end to end through the drop-in
  ``InTimeAccumulateWeightedAggregator`` (DXO accept -> engine staging -> burst kernel -> D2H), numpy and torch
  containers, and EVERY one of the 125M results is compared with the C oracle (multi-threaded, same per-element
  sequence: weighted_aggregation_helper.py:181-236).
* Config 4 -- 256 clients x 350M split over 8 GPUs -- one GPU's share is 256 clients x 43.75M params: the kernel
  chains two 128-client launches through the fp32 accumulator.  Sampled bit-exact check (the oracle cannot redo
  11.2e9 multiply-adds in a test) at 20 000 random positions plus every tile edge near them, on the first and on a
  middle bucket of the global model (the generator's column offset).
* The in-process parameter-bucket split over 8 engines (``WeightedAggregationHelper(devices=[0] * 8)``,
  sharding.ShardedFedAvg) at 256 clients, every element against the oracle.
"""

import gc

import numpy as np
import pytest

from golden_util import same_bits

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16  # the GPU box's CPU share


def _weights(K):
    return [1.0 * float(1 + (37 * k) % 100) for k in range(K)]


@pytest.fixture(scope="module")
def config2_rows():
    P, K = 125_000_000, 8
    rows = [np.random.default_rng(2000 + k).standard_normal(P, dtype=np.float32) for k in range(K)]
    yield rows
    del rows
    gc.collect()


@pytest.mark.parametrize("container", ["numpy", "torch"])
def test_config2_full_size_every_element(config2_rows, oracle, container):
    import torch

    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import (
        InTimeAccumulateWeightedAggregator,
    )
    from nvflare_amd.compat import DXO, AppConstants, DataKind, EventType, FLContext, MetaKey, ReservedKey, from_shareable

    rows = config2_rows
    K, P = len(rows), rows[0].size
    n_iter = [1 + (37 * k) % 100 for k in range(K)]
    agg = InTimeAccumulateWeightedAggregator(expected_data_kind=DataKind.WEIGHTS)
    fl_ctx = FLContext()
    agg.handle_event(EventType.START_RUN, fl_ctx)
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 3)
    for k in range(K):
        v = rows[k] if container == "numpy" else torch.from_numpy(rows[k])
        s = DXO(DataKind.WEIGHTS, data={"model.w": v}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: n_iter[k]}).to_shareable()
        s.set_peer_props({ReservedKey.IDENTITY_NAME: f"site-{k}"})
        s.add_cookie(AppConstants.CONTRIBUTION_ROUND, 3)
        assert agg.accept(s, fl_ctx)
    got = from_shareable(agg.aggregate(fl_ctx)).data["model.w"]
    if container == "torch":
        assert isinstance(got, torch.Tensor)
        got = got.numpy()
    assert got.dtype == np.float32 and got.size == P
    mode = oracle.MODE_TORCH if container == "torch" else oracle.MODE_NUMPY
    exp = oracle.fedavg_c(rows, [float(n) for n in n_iter], mode, nthreads=ORACLE_THREADS)
    diff = np.count_nonzero(got.view(np.uint32) != exp.view(np.uint32))
    assert diff == 0, f"{diff} of {P} results differ from the oracle"
    stats = fl_ctx.get_prop(AppConstants.AGGREGATION_STATS)
    assert stats is not None


def _sample_idx(P, rng, n=20_000):
    idx = rng.integers(0, P, n, dtype=np.int64)
    edges = (idx // 4096) * 4096
    idx = np.concatenate([idx, edges, np.maximum(edges - 1, 0), [0, 1, P - 2, P - 1]])
    return np.unique(np.clip(idx, 0, P - 1)).astype(np.uint64)


@pytest.fixture(scope="module")
def config4_share():
    """One GPU's share of config 4 at 8 GPUs: 256 clients x bucket_ranges(350M, 8)[b] params in one slab."""
    import torch

    from nvflare_amd.device import DeviceContext, TiledLayout
    from nvflare_amd.sharding import bucket_ranges

    torch.cuda.empty_cache()
    gc.collect()
    ctx = DeviceContext.get(0)
    K = 256
    lo, hi = bucket_ranges(350_000_000, 8)[0]
    P = hi - lo
    lay = TiledLayout(4096, K)
    slab = ctx.alloc(lay.slab_elems(P) * 4)
    yield ctx, lay, slab, K, P
    slab.close()


@pytest.mark.parametrize("bucket", [0, 5])
@pytest.mark.parametrize("mode", ["torch", "numpy"])
def test_config4_gpu_share_sampled(config4_share, oracle, bucket, mode):
    from nvflare_amd import _native as N
    from nvflare_amd.sharding import bucket_ranges

    ctx, lay, slab, K, P0 = config4_share
    lo, hi = bucket_ranges(350_000_000, 8)[bucket]
    P = hi - lo
    assert P <= P0 and abs(P - 43_750_000) < 4096
    seed = 4400 + bucket
    bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]
    for k, b in enumerate(bases):
        ctx.fill_synthetic_f32(b, P, seed, k, lo, lay.tile, lay.tile_stride)
    ws = _weights(K)
    count = None
    for w in ws:
        count = w if count is None else count + w
    op, fin, omode = ((N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, oracle.MODE_TORCH) if mode == "torch"
                      else (N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE, oracle.MODE_NUMPY))
    end = (P + 3) // 4 * 4
    out = ctx.alloc(end * 4)
    n0 = ctx.launch_count()
    ctx.accumulate_tiled(bases, ws, lay.tile, lay.tile_stride, 0, end, out.ptr, op, fin, count)
    ctx.sync()
    launches = ctx.launch_count() - n0
    idx = _sample_idx(P, np.random.default_rng(40 + bucket))
    rows = [oracle.synth_values(seed, k, idx + np.uint64(lo)) for k in range(K)]
    exp = oracle.fedavg_c(rows, ws, omode)
    got = ctx.gather_f32(out.ptr, idx)
    out.close()
    assert same_bits(got, exp), f"{np.count_nonzero(got.view(np.uint32) != exp.view(np.uint32))} of {idx.size} differ"
    # 256 clients = two chains of 128 (the kernel-argument table): every tile range is launched twice
    tiles = (P + 4095) // 4096
    assert launches >= 2 * -(-tiles // (ctx.num_cus * 18))


@pytest.mark.parametrize("container", ["numpy", "torch"])
def test_sharded_eight_buckets_256_clients(oracle, container):
    """WeightedAggregationHelper(devices=[0] * 8): every key cut into 8 parameter buckets, one engine each (all on
    the test GPU), 256 contributions; same bits as the one-device aggregation, every element."""
    import torch

    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    K = 256
    sizes = {"big": 600_011, "mid": 8 * 4096 + 17, "tiny": 5}
    rng = np.random.default_rng(256)
    data = [{k: rng.standard_normal(n, dtype=np.float32) for k, n in sizes.items()} for _ in range(K)]
    ws = [float(1 + (37 * k) % 100) * (0.5 if k % 3 else 1.0) for k in range(K)]
    h = WeightedAggregationHelper(devices=[0] * 8)
    try:
        assert len(h.engine.engines) == 8
        for k in range(K):
            d = data[k] if container == "numpy" else {n: torch.from_numpy(v) for n, v in data[k].items()}
            h.add(d, ws[k], f"site-{k}", 0)
        out = h.get_result()
    finally:
        h.engine.release()
    mode = oracle.MODE_TORCH if container == "torch" else oracle.MODE_NUMPY
    for name in sizes:
        got = out[name].numpy() if container == "torch" else out[name]
        exp = oracle.fedavg_c([d[name] for d in data], ws, mode, nthreads=ORACLE_THREADS)
        assert same_bits(got, exp), name
