"""Multi-process (gloo, world_size 2) checks of the parameter-bucket sharding on CPU.

The HIP kernel cannot run here, so each rank computes its bucket with the CPU oracle (test
infrastructure) from the host twin of the bench's synthetic generator; rank 0 reassembles and compares
bit-for-bit with a single-process aggregation of the whole model.  This is the partition the bench's
torchrun path and sharding.ShardedFedAvg use: per-element order is unchanged, so no collective is needed
and the bits cannot change."""

import os
import socket

import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nvflare_amd.sharding import BUCKET_ALIGN, bucket_ranges


@pytest.mark.parametrize("total", [0, 1, 4095, 4096, 4097, 10 * 4096 + 3, 1_000_000])
@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_bucket_ranges_partition(total, parts):
    r = bucket_ranges(total, parts)
    assert len(r) == parts
    assert r[0][0] == 0 and r[-1][1] == total
    for (a0, a1), (b0, b1) in zip(r[:-1], r[1:]):
        assert a1 == b0 and a0 <= a1
        assert a1 % BUCKET_ALIGN == 0 or a1 == total
    sizes = [b - a for a, b in r]
    assert max(sizes) - min(sizes) <= BUCKET_ALIGN


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, P, K, q, scaling="weak"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from oracle import fedavg_oracle as orc

        col0, n = bench.rank_span(scaling, rank, world, P)
        rows = [orc.synth_values(1000, k, np.arange(col0, col0 + n, dtype=np.uint64)) for k in range(K)]
        ws = orc.synth_weights(K)
        part = orc.fedavg_c(rows, ws, orc.MODE_TORCH)
        gathered = [None] * world if rank == 0 else None
        dist.gather_object(part, gathered, dst=0)
        t = bench.max_over_ranks(world, float(rank + 1))
        sums = bench.sum_over_ranks(world, [rank, 1])  # the spot-check counts' reduction
        if rank == 0:
            q.put((np.concatenate(gathered), (t, sums)))
    finally:
        dist.destroy_process_group()


def test_weak_scaling_buckets_gloo(oracle):
    world, P, K = 2, 12_345, 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, (tmax, sums) = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rows = [oracle.synth_values(1000, k, np.arange(world * P, dtype=np.uint64)) for k in range(K)]
    full = oracle.fedavg_c(rows, oracle.synth_weights(K), oracle.MODE_TORCH)
    assert np.array_equal(res.view(np.uint32), full.view(np.uint32))
    assert tmax == 2.0  # max over ranks
    assert sums == [1, 2]  # sum over ranks


@pytest.mark.parametrize("world", [2, 3])
def test_strong_scaling_buckets_gloo(oracle, world):
    """bench.py --scaling strong (BASELINE configs 4 and 5): one P-param model split by bucket_ranges over the
    ranks; the ranks' buckets, reassembled, are the one-process aggregation of the whole model, bit for bit."""
    P, K = 3 * 4096 * 5 + 77, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, K, q, "strong")) for r in range(world)]
    for p in procs:
        p.start()
    res, (tmax, sums) = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rows = [oracle.synth_values(1000, k, np.arange(P, dtype=np.uint64)) for k in range(K)]
    full = oracle.fedavg_c(rows, oracle.synth_weights(K), oracle.MODE_TORCH)
    assert res.size == P and np.array_equal(res.view(np.uint32), full.view(np.uint32))
    assert tmax == float(world) and sums == [sum(range(world)), world]


def test_bench_presets_follow_baseline():
    """bench.py --config N fills K, P, the epilogue and the scaling from BASELINE.json configs[1..4]; the default run
    (config 3) also measures config 2 device-resident, configs 5 and 4 under strong scaling, config 2 host-resident and
    config 4 through the client-sharded exchange;
    explicit overrides turn that off."""
    import bench

    a = bench.parse([])
    assert (a.clients, a.params, a.epilogue, a.scaling, a.also) == \
        (64, 10**9, "none", "weak", [2, 5, 4, bench.HOST_RESIDENT, bench.HOST_SHARDED, bench.CLIENT_SHARDED])
    assert bench.parse(["--also", "4x,5"]).also == [bench.CLIENT_SHARDED, 5]
    assert bench.parse(["--also", "2h"]).also == [bench.HOST_RESIDENT]
    assert bench.parse(["--also", "2s,2h"]).also == [bench.HOST_SHARDED, bench.HOST_RESIDENT]
    assert (lambda c: (c.clients, c.params, c.epilogue, c.scaling))(bench.parse(["--config", "2"])) == \
        (8, 125_000_000, "none", "weak")
    assert (lambda c: (c.clients, c.params, c.epilogue, c.scaling))(bench.parse(["--config", "4"])) == \
        (256, 350_000_000, "none", "strong")
    assert (lambda c: (c.clients, c.params, c.epilogue, c.scaling))(bench.parse(["--config", "5"])) == \
        (64, 10**9, "adam", "strong")
    b = bench.parse(["--clients", "8", "--params", "1.25e8"])
    assert b.also == [] and not b.preset_exact and b.scaling == "weak"
    c = bench.parse(["--global-params", "3.5e8", "--clients", "256"])
    assert c.scaling == "strong" and c.params == 350_000_000
    # config 4 per GPU at 8 GPUs: 256 clients x 43.75 M (bucket_ranges in whole tiles)
    spans = [bench.rank_span("strong", r, 8, 350_000_000) for r in range(8)]
    assert sum(n for _, n in spans) == 350_000_000 and all(abs(n - 43_750_000) < 4096 for _, n in spans)
    assert spans[0][0] == 0 and all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(7))


def test_sharded_pieces_reassemble(oracle):
    """ShardedFedAvg's slicing and reassembly (host side), checked with the oracle per bucket."""
    from nvflare_amd.sharding import ShardedFedAvg

    rng = np.random.default_rng(0)
    shapes = {"a": (3, 5000), "b": (7,), "c": (), "d": (0,), "e": (2, 4096)}
    K = 4
    data = [{k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()} for _ in range(K)]
    ws = [1.0, 2.0, 0.5, 3.0]
    sh = ShardedFedAvg.__new__(ShardedFedAvg)  # host-side methods only (no device engines)
    sh.engines = [types.SimpleNamespace(key_spans={}) for _ in range(3)]
    pieces = [dict(sh._pieces(b, list(data[0].items()))) for b in range(3)]
    for b, eng in enumerate(sh.engines):  # each bucket's place in its whole key, for the 16-bit torch loops
        assert set(eng.key_spans) == set(pieces[b])
        for sub, (lo, n) in eng.key_spans.items():
            assert sub.endswith(f"\x00{lo}") and n == (int(np.prod(shapes[sub.split(chr(0))[0]])) or 0)
    covered = {}
    for b, pc in enumerate(pieces):
        for sub, arr in pc.items():
            k, off = sub.split("\x00")
            covered.setdefault(k, []).append((int(off), arr.size))
    for k, s in shapes.items():
        n = int(np.prod(s)) if s else 1
        spans = sorted(covered[k])
        assert spans[0][0] == 0 and sum(x for _, x in spans) == n
    # bucket-wise oracle == whole-key oracle
    for k, s in shapes.items():
        n = int(np.prod(s)) if s else 1
        if n == 0:
            continue
        whole = oracle.fedavg_c([d[k].reshape(-1) for d in data], ws, oracle.MODE_NUMPY)
        parts = []
        for lo, hi in bucket_ranges(n, 3):
            if hi > lo:
                parts.append(oracle.fedavg_c([d[k].reshape(-1)[lo:hi] for d in data], ws, oracle.MODE_NUMPY))
        assert np.array_equal(np.concatenate(parts).view(np.uint32), whole.view(np.uint32))


def _fake_sharded(n_dev=3):
    import threading
    from concurrent.futures import ThreadPoolExecutor

    from fake_device import fake_engine
    from nvflare_amd.sharding import ShardedFedAvg

    sh = ShardedFedAvg.__new__(ShardedFedAvg)  # engines on tests/fake_device (host memory)
    sh.devices = list(range(n_dev))
    sh.engines = [fake_engine() for _ in range(n_dev)]
    sh.lock = threading.RLock()
    sh._pool = ThreadPoolExecutor(max_workers=n_dev)
    sh._shapes = {}
    return sh


def test_sharded_rejects_reshaped_contribution(oracle):
    """A later contribution with the first one's element count but another shape raises the single-device
    engine's ValueError, and stages nothing on any shard (sharding.py shape check)."""
    sh = _fake_sharded()
    rng = np.random.default_rng(1)
    a0 = rng.standard_normal((64, 7)).astype(np.float32)
    b0 = rng.standard_normal(9000).astype(np.float32)
    sh.add([("a", a0), ("b", b0)], 1.0, True)
    staged = [len(e.ctx.launches) for e in sh.engines], [dict(e.stats) for e in sh.engines]
    bad = rng.standard_normal((7, 64)).astype(np.float32)
    with pytest.raises(ValueError, match="shape"):
        sh.add([("b", b0), ("a", bad)], 2.0, True)  # the good item first: it must not be staged either
    assert ([len(e.ctx.launches) for e in sh.engines], [dict(e.stats) for e in sh.engines]) == staged
    with pytest.raises(ValueError, match="shape"):
        sh.add([("c", b0), ("c", b0.reshape(90, 100))], 2.0, True)  # two shapes for a new key in one call
    assert "c" not in sh._shapes
    sh.add([("a", a0 * 2), ("b", b0)], 3.0, True)
    res = sh.result()
    assert res["a"].shape == (64, 7)
    exp = oracle.fedavg_c([a0.reshape(-1), (a0 * 2).reshape(-1)], [1.0, 3.0], oracle.MODE_NUMPY)
    assert np.array_equal(res["a"].reshape(-1).view(np.uint32), exp.view(np.uint32))
    sh._pool.shutdown()


def test_sharded_keys_with_nul_bytes(oracle):
    """Keys holding NUL bytes (the SCAFFOLD control prefix) survive the bucket sub-key round trip."""
    sh = _fake_sharded()
    rng = np.random.default_rng(2)
    keys = ["w", "\x00scaffold_ctrl\x00w", "a\x00b\x001"]
    rows = [{k: rng.standard_normal(9000).astype(np.float32) for k in keys} for _ in range(3)]
    for i, r in enumerate(rows):
        sh.add(list(r.items()), 1.0 + i, True)
    assert sh.keys == set(keys)
    res = sh.result()
    assert set(res) == set(keys)
    for k in keys:
        exp = oracle.fedavg_c([r[k] for r in rows], [1.0, 2.0, 3.0], oracle.MODE_NUMPY)
        assert np.array_equal(res[k].view(np.uint32), exp.view(np.uint32))
    sh._pool.shutdown()



def test_sharded_deferred_rounds_match_eager():
    """ShardedFedAvg.result_deferred: every fp32 key comes back as a ShardedDeferredAggregate whose pieces are
    the buckets' DeferredAggregates (one per engine); materialised, it equals the eager sharded result bit
    for bit, also after the next round has settled the previous one; fp64 keys stay eager."""
    import torch

    from nvflare_amd.deferred import DeferredAggregate, ShardedDeferredAggregate, materialize_deferred

    rng = np.random.default_rng(7)
    shapes = {"a": (3, 5000), "b": (7,), "c": (), "e": (2, 4096), "big": (3 * 4096 + 5,)}
    sh_def, sh_eager = _fake_sharded(3), _fake_sharded(3)
    kept = []
    for rnd in range(2):
        ws = [1.0 + rnd, 2.5, 0.75, 3.0]
        for k, w in enumerate(ws):
            items = [(n, rng.standard_normal(s).astype(np.float32)) for n, s in shapes.items()]
            items.append(("d64", rng.standard_normal(10)))  # numpy's default fp64: the fp64 arena, eager
            items.append(("t", torch.from_numpy(rng.standard_normal(9000).astype(np.float32))))
            sh_def.add(items, w, True)
            sh_eager.add(items, w, True)
        got, exp = sh_def.result_deferred(), sh_eager.result()
        sh_def.reset()
        sh_eager.reset()
        assert isinstance(got["d64"], np.ndarray)
        for n in list(shapes) + ["t"]:
            v = got[n]
            assert isinstance(v, ShardedDeferredAggregate), n
            assert v.shape == tuple(exp[n].shape) and v.container == ("torch" if n == "t" else "numpy")
            assert all(isinstance(d, DeferredAggregate) for _, _, d in v.pieces)
            assert sum(hi - lo for lo, hi, _ in v.pieces) == v.size
        kept.append((got, exp))
    for got, exp in kept:  # round 0's values materialise after round 1 settled them
        for n in exp:
            g = materialize_deferred(got[n])
            g = g.numpy() if isinstance(g, torch.Tensor) else np.asarray(g)
            e_ = exp[n].numpy() if isinstance(exp[n], torch.Tensor) else np.asarray(exp[n])
            assert g.shape == e_.shape and g.dtype == e_.dtype
            assert np.array_equal(g.reshape(-1).view(np.uint8), e_.reshape(-1).view(np.uint8)), n
    for s_ in (sh_def, sh_eager):
        s_._pool.shutdown()


def test_sharded_result_lands_in_one_host_array(oracle):
    """ShardedFedAvg.result: every device copies its buckets straight to their place in one host array per
    element format (fedavg_d2h_multi, one call per device and format) -- no host concatenation; keys with a
    bucket outside an arena (integer side buffers, empty keys) are still reassembled per key.  Same bits."""
    import torch

    sh = _fake_sharded(3)
    rng = np.random.default_rng(9)
    shapes = {"a": (3, 5000), "b": (7,), "c": (), "e": (2, 4096), "z": (0,)}
    rows = []
    for i in range(4):
        r = {k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()}
        r["d64"] = rng.standard_normal(9000)
        r["n"] = np.arange(5000, dtype=np.int64) * i
        rows.append(r)
        sh.add(list(r.items()), 1.0 + i, True)
    res = sh.result()
    ws = [1.0, 2.0, 3.0, 4.0]
    base32 = None
    for k in ("a", "b", "c", "e"):
        v = res[k]
        assert np.shape(v) == shapes[k]
        exp = oracle.fedavg_c([r[k].reshape(-1) for r in rows], ws, oracle.MODE_NUMPY)
        assert np.array_equal(np.asarray(v, dtype=np.float32).reshape(-1).view(np.uint32), exp.view(np.uint32)), k
        if k != "c":  # 0-d results are numpy scalars, as the reference's
            owner = v.base if v.base is not None else v
            while getattr(owner, "base", None) is not None and isinstance(owner.base, np.ndarray):
                owner = owner.base
            base32 = base32 if base32 is not None else owner
            assert np.shares_memory(v, base32), k  # one host array for every fp32 key
    exp64 = oracle.fedavg_c([r["d64"] for r in rows], ws, oracle.MODE_NUMPY)
    assert res["d64"].dtype == np.float64 and np.array_equal(res["d64"].view(np.uint64), exp64.view(np.uint64))
    assert res["z"].shape == (0,) and res["n"].dtype == np.float64
    assert sum(getattr(e.ctx, "d2h_multi_calls", 0) for e in sh.engines) >= 3
    sh._pool.shutdown()
