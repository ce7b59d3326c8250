"""Pipelined egress on the GPU: final launches split at EGRESS_CHUNK boundaries with readiness marks, the D2H
of finished chunks overlapping the launches still running (fedavg_mark / fedavg_d2h_marked).  The result
must be bit-identical to the one-shot path and to the oracle, with chunk boundaries inside keys, between
keys, inside multi-slab chains and for keys a client left out."""

import numpy as np
import pytest
import torch

from golden_util import same_bits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("container", ["numpy", "torch"])
def test_pipelined_egress_matches_one_shot(monkeypatch, oracle, container):
    import nvflare_amd.engine as E
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    rng = np.random.default_rng(5)
    sizes = {"k0": 400_000, "k1": 3, "k2": 700_001, "k3": 163_840}
    K = 20  # first round: slabs of 16 then 32 slots -> chained launches
    clients = [{k: rng.standard_normal(n).astype(np.float32) for k, n in sizes.items()} for _ in range(K)]
    clients[2].pop("k1")
    ws = [float(1 + (37 * k) % 11) for k in range(K)]

    def run(chunk):
        monkeypatch.setattr(E, "EGRESS_CHUNK", chunk)
        h = WeightedAggregationHelper()
        for k, (c, w) in enumerate(zip(clients, ws)):
            h.add({n: torch.from_numpy(a.copy()) if container == "torch" else a for n, a in c.items()}, w, f"s{k}", 0)
        out = h.get_result()
        return {n: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)).copy() for n, v in out.items()}

    piped = run(256 << 10)  # 64 Ki fp32 elements per chunk: ~20 chunks over the 5 MB layout
    whole = run(1 << 40)
    mode = oracle.MODE_TORCH if container == "torch" else oracle.MODE_NUMPY
    for key in sizes:
        seq = [(c[key], w) for c, w in zip(clients, ws) if key in c]
        exp = oracle.fedavg_c([a for a, _ in seq], [w for _, w in seq], mode)
        assert same_bits(piped[key], exp), key
        assert same_bits(whole[key], exp), key


def test_registered_host_arrays_copy_and_unregister_on_free():
    """Pool arrays of >= 16 MiB are page-locked for direct D2H; each is unregistered when its memory is freed,
    so a new array at the same address registers again (hipHostRegister refuses a range registered twice)."""
    import gc

    from nvflare_amd.device import DeviceContext, HostArenaPool

    ctx = DeviceContext.get(0)
    n = (HostArenaPool.PIN_MIN_BYTES // 4) + 12345
    src = np.random.default_rng(5).standard_normal(n).astype(np.float32)
    buf = ctx.alloc(n * 4)
    ctx.h2d_ptr(buf.ptr, src.ctypes.data, src.nbytes)
    for _ in range(4):
        pool = HostArenaPool(depth=1)
        a = pool.take(n, np.float32, pin=ctx)
        ctx.d2h(a, buf.ptr)
        assert np.array_equal(a.view(np.uint32), src.view(np.uint32))
        b = pool.take(n, np.float32, pin=ctx)  # `a` is referenced: a new (registered) array, `a` dropped by the pool
        assert b is not a
        ctx.d2h(b, buf.ptr)
        assert np.array_equal(b.view(np.uint32), src.view(np.uint32))
        del a, b, pool
        gc.collect()
    buf.close()
