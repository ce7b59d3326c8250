"""A contribution is staged all or nothing (engine.DeviceFedAvg.add, sharding.ShardedFedAvg.add).

The reference keeps a key's sum and its weight count together (weighted_aggregation_helper.py:201,216: the
count moves with the key's sum).  On the device a contribution takes a slot per element format, side buffers
and DMAs; if any of them fails (an allocation in a second arena, an H2D error) nothing of it may stay behind: the
next aggregation must equal the oracle over the contributions that were accepted.  The device is
tests/fake_device.FakeDeviceContext with failures injected into its allocator and copy entry points."""

import numpy as np
import pytest
import torch

from fake_device import FakeDeviceContext, fake_engine
from golden_util import as_f32_values, same_bits
from nvflare_amd import _native as N
from nvflare_amd.sharding import ShardedFedAvg


class _Fail:
    """Arms a failure on the n-th call (1-based) of a context method after ``arm``."""

    def __init__(self, ctx, method, when=lambda *a: True):
        self.ctx, self.method, self.when = ctx, method, when
        self.orig = getattr(ctx, method)
        self.left = None
        setattr(ctx, method, self._call)

    def arm(self, nth=1):
        self.left = nth

    def _call(self, *a, **kw):
        if self.left is not None and self.when(*a):
            self.left -= 1
            if self.left == 0:
                self.left = None
                raise N.FedAvgError(f"injected {self.method} failure")
        return self.orig(*a, **kw)


def _client(rng, k, late=False):
    c = {"w": rng.standard_normal(9000).astype(np.float32),
         "b": torch.from_numpy(rng.standard_normal(300).astype(np.float32)).to(torch.bfloat16),
         "n": torch.tensor(k, dtype=torch.int64)}
    if late:
        c["late"] = rng.standard_normal(50).astype(np.float32)
    return c


def _expect(clients, ws, key):
    vals = [(c[key], w) for c, w in zip(clients, ws) if key in c]
    v0 = vals[0][0]
    is_t = isinstance(v0, torch.Tensor)
    fmt = "bfloat16" if is_t and v0.dtype == torch.bfloat16 else None
    rows = [(as_f32_values(v, fmt) if fmt else (v.numpy() if is_t else v).astype(np.float32)).reshape(-1)
            for v, _ in vals]
    wl = [w for _, w in vals]
    count = None
    for w in wl:
        count = w if count is None else count + w
    if fmt:
        from oracle import fedavg_oracle as orc

        scalar = orc.torch16_scalar_mask(rows[0].size, torch.get_num_threads())
        return FakeDeviceContext._agg(rows, wl, N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV, count, None, fmt=fmt, scalar=scalar)
    op, fin = (N.FEDAVG_OP_TORCH, N.FEDAVG_FIN_DIV) if is_t else (N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE)
    return FakeDeviceContext._agg(rows, wl, op, fin, count, None)


def _check(out, clients, ws):
    assert set(out) == set().union(*[set(c) for c in clients])
    for key in out:
        exp = _expect(clients, ws, key)
        v = out[key]
        got = as_f32_values(v, "bfloat16") if isinstance(v, torch.Tensor) and v.dtype == torch.bfloat16 else \
            (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v))
        assert same_bits(np.asarray(got, dtype=np.float32).reshape(-1), np.asarray(exp, dtype=np.float32).reshape(-1)), key


@pytest.mark.parametrize("budget,slab_slots", [(None, None), (None, 2), (1, None)])
@pytest.mark.parametrize("what", ["alloc_second_arena", "h2d_second_arena", "h2d_first_arena", "side_buffer"])
def test_failed_add_leaves_nothing_behind(budget, slab_slots, what):
    rng = np.random.default_rng(11)
    e = fake_engine(max_resident_bytes=budget, slab_slots=slab_slots)
    ctx = e.ctx
    ok = [_client(rng, 0), _client(rng, 1)]
    bad = _client(rng, 2, late=True)  # also introduces a key: it must not survive the failure
    after = _client(rng, 3)
    ws = [2.0, 3.0, 5.0, 7.0]
    for c, w in zip(ok, ws):
        e.add(list(c.items()), w, True)
    state = {"armed": what, "h2d": 0, "fail_alloc": False}
    alloc, h2d_multi, h2d_ptr = ctx.alloc, ctx.h2d_tiled_multi, ctx.h2d_ptr

    def fail_alloc(nbytes):
        if state["fail_alloc"]:
            raise N.FedAvgError("injected allocation failure")
        return alloc(nbytes)

    def fail_h2d_multi(*a):
        state["h2d"] += 1
        if state["armed"] == "h2d_first_arena" or (state["armed"] == "h2d_second_arena" and state["h2d"] == 2):
            raise N.FedAvgError("injected H2D failure")
        h2d_multi(*a)
        if state["armed"] == "alloc_second_arena":
            state["fail_alloc"] = True  # from the second arena on, every allocation fails

    def fail_h2d_ptr(*a):
        if state["armed"] == "side_buffer":
            raise N.FedAvgError("injected H2D failure")
        h2d_ptr(*a)

    ctx.alloc, ctx.h2d_tiled_multi, ctx.h2d_ptr = fail_alloc, fail_h2d_multi, fail_h2d_ptr
    keys_before = set(e.keys)
    raised = False
    try:
        e.add(list(bad.items()), ws[2], True)
    except N.FedAvgError:
        raised = True
    ctx.alloc, ctx.h2d_tiled_multi, ctx.h2d_ptr = alloc, h2d_multi, h2d_ptr
    accepted, wacc = [ok[0], ok[1]], [ws[0], ws[1]]
    if raised:
        assert set(e.keys) == keys_before  # the key the failed contribution introduced is gone
    else:  # the second arena found room without allocating (an existing slab or a fold): nothing failed
        assert what == "alloc_second_arena"
        accepted.append(bad)
        wacc.append(ws[2])
    e.add(list(after.items()), ws[3], True)
    out = e.result()
    _check(out, accepted + [after], wacc + [ws[3]])
    e.reset()
    assert not e._live_slots  # the failed contribution's slots were given back


def test_undo_last_add_only():
    rng = np.random.default_rng(12)
    e = fake_engine()
    c = [_client(rng, k, late=(k == 1)) for k in range(3)]
    tx0 = e.add(list(c[0].items()), 1.0, True)
    tx1 = e.add(list(c[1].items()), 2.0, True)
    with pytest.raises(RuntimeError):
        e.undo_add(tx0)  # not the last operation any more
    e.undo_add(tx1)
    assert "late" not in e.keys
    with pytest.raises(RuntimeError):
        e.undo_add(tx1)  # already taken back
    e.add(list(c[2].items()), 3.0, True)
    _check(e.result(), [c[0], c[2]], [1.0, 3.0])


@pytest.mark.parametrize("failing_bucket", [0, 1, 2])
def test_sharded_add_rolls_back_every_bucket(failing_bucket):
    rng = np.random.default_rng(13)
    sh = ShardedFedAvg([0, 0, 0])
    for eng in sh.engines:
        eng._ctx = FakeDeviceContext()
    try:
        ok = [_client(rng, 0), _client(rng, 1)]
        bad = _client(rng, 2, late=True)
        after = _client(rng, 3)
        ws = [2.0, 3.0, 5.0, 7.0]
        for c, w in zip(ok, ws):
            sh.add(list(c.items()), w, True)
        f = _Fail(sh.engines[failing_bucket].ctx, "h2d_tiled_multi")
        f.arm(1)
        with pytest.raises(N.FedAvgError):
            sh.add(list(bad.items()), ws[2], True)
        assert "late" not in sh.keys and "late" not in sh._shapes
        sh.add(list(after.items()), ws[3], True)
        _check(sh.result(), [ok[0], ok[1], after], [ws[0], ws[1], ws[3]])
    finally:
        sh.release()


def test_sharded_add_undoes_every_bucket_when_an_undo_fails():
    """bucket 1 fails to stage, bucket 0's undo raises too -- bucket 2 is still undone, and the error
    raised is the staging error, unchanged (its own __cause__ kept), with the undo failure reported
    beside it (a note on Python 3.11+, else ``undo_failures``) and logged."""
    rng = np.random.default_rng(15)
    sh = ShardedFedAvg([0, 0, 0])
    for eng in sh.engines:
        eng._ctx = FakeDeviceContext()
    try:
        ok = _client(rng, 0)
        sh.add(list(ok.items()), 2.0, True)
        f = _Fail(sh.engines[1].ctx, "h2d_tiled_multi")
        f.arm(1)
        undone = []
        orig0, orig2 = sh.engines[0].undo_add, sh.engines[2].undo_add

        def undo0(tx):
            raise RuntimeError("injected undo failure")

        def undo2(tx):
            undone.append(tx)
            return orig2(tx)

        sh.engines[0].undo_add, sh.engines[2].undo_add = undo0, undo2
        with pytest.raises(N.FedAvgError, match="injected h2d_tiled_multi failure") as ei:
            sh.add(list(_client(rng, 1, late=True).items()), 3.0, True)
        assert len(undone) == 1, "bucket 2 must be undone although bucket 0's undo failed"
        assert ei.value.__cause__ is None  # the staging error as it was raised: nothing re-chained onto it
        notes = getattr(ei.value, "__notes__", None)
        if notes is not None:
            assert any("bucket 0" in n and "injected undo failure" in n for n in notes)
        else:
            (b, e), = ei.value.undo_failures
            assert b == 0 and "injected undo failure" in str(e)
        assert "late" not in sh._shapes
        sh.engines[0].undo_add = orig0
    finally:
        sh.release()


def test_helper_stats_skip_a_failed_contribution():
    """The drop-in helper counts a contribution (key_contribution_counts, history, counts) only once the device
    has staged it: a failed add leaves the stats and the next result as if it never arrived."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    rng = np.random.default_rng(14)
    h = WeightedAggregationHelper(exclude_vars="skip")
    h._engine = fake_engine()
    c = [{"w": rng.standard_normal(5000).astype(np.float32), "skip": np.ones(3, np.float32)} for _ in range(3)]
    c[1]["late"] = np.arange(4, dtype=np.float32)
    h.add(c[0], 1.0, "site-0", 0)
    h2d = h._engine.ctx.h2d_tiled_multi

    def boom(*a):
        raise N.FedAvgError("injected H2D failure")

    h._engine.ctx.h2d_tiled_multi = boom
    with pytest.raises(N.FedAvgError):
        h.add(c[1], 2.0, "site-1", 0)
    h._engine.ctx.h2d_tiled_multi = h2d
    assert h.key_contribution_counts == {"w": 1} and h.get_len() == 1
    h.add(c[2], 3.0, "site-2", 0)
    out = h.get_result()
    stats = h.last_aggregation_stats
    exp = FakeDeviceContext._agg([c[0]["w"], c[2]["w"]], [1.0, 3.0], N.FEDAVG_OP_NUMPY, N.FEDAVG_FIN_SCALE, 4.0, None)
    assert set(out) == {"w"} and same_bits(out["w"], exp)
    assert stats is not None
