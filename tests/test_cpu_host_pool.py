"""HostArenaPool: round results are views of one host array, reused only after every view is gone.

Memory identity is the data address (each take() hands out a fresh array object over pooled storage)."""

import sys

import numpy as np
import torch

from nvflare_amd.device import HostArenaPool


def _addr(a):
    return a.ctypes.data


def test_pool_reuses_only_released_arrays():
    pool = HostArenaPool()
    a = pool.take(100)
    a_addr = _addr(a)
    view = a[10:20]
    del a
    b = pool.take(100)
    assert _addr(b) != a_addr  # a view of the previous round is alive
    b_addr = _addr(b)
    del b, view
    c = pool.take(100)
    assert _addr(c) in (a_addr, b_addr)  # released: a pooled array again (no new pages to fault in)
    t = torch.from_numpy(c[:4].reshape(2, 2))
    c_addr = _addr(c)
    del c
    d = pool.take(100)
    assert _addr(d) != c_addr  # a torch tensor over a view keeps it alive
    assert t.shape == (2, 2)
    e = pool.take(50)
    assert e.size == 50 and e.dtype == np.float32


def test_pool_reuses_the_round_before_last():
    """Scatter-and-gather holds round r-1's result while round r is computed: r reuses r-2's array."""
    pool = HostArenaPool(depth=3)
    prev = pool.take(64)
    addrs = [_addr(prev)]
    for _ in range(4):
        cur = pool.take(64)
        addrs.append(_addr(cur))
        assert _addr(cur) != _addr(prev)
        prev = cur  # the caller drops the older result only now
    assert len(set(addrs)) == 2


def test_live_view_of_a_view_blocks_reuse(monkeypatch):
    """A live view (of a view, reshaped, 0-d) of round r's result blocks reuse of its memory, independently
    of reference-count arithmetic (HostArenaPool relied on sys.getrefcount)."""
    monkeypatch.setattr(sys, "getrefcount", lambda _o: 0)  # the pool must not consult it
    pool = HostArenaPool(depth=2)
    r = pool.take(1000)
    r[:] = 7.0
    r_addr = _addr(r)
    keys = {"w": r[0:600].reshape(20, 30), "b": r[600:1000]}
    scalar = keys["w"][3][4:5].reshape(())
    del r, keys
    for _ in range(4):
        nxt = pool.take(1000)
        assert _addr(nxt) != r_addr
        nxt[:] = -1.0  # the next rounds' D2H must never land in round r's memory
        del nxt
    assert float(scalar) == 7.0
    del scalar
    assert any(_addr(pool.take(1000)) == r_addr for _ in range(2))
