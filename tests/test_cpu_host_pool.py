"""HostArenaPool: round results are views of one host array, reused only after every view is gone."""

import numpy as np
import torch

from nvflare_amd.device import HostArenaPool


def test_pool_reuses_only_released_arrays():
    pool = HostArenaPool()
    a = pool.take(100)
    a_id = id(a)
    view = a[10:20]
    del a
    b = pool.take(100)
    assert id(b) != a_id  # a view of the previous round is alive
    b_id = id(b)
    del b, view
    c = pool.take(100)
    assert id(c) in (a_id, b_id)  # released: a pooled array again (no new pages to fault in)
    t = torch.from_numpy(c[:4].reshape(2, 2))
    c_id = id(c)
    del c
    d = pool.take(100)
    assert id(d) != c_id  # a torch tensor over a view keeps it alive
    assert t.shape == (2, 2)
    e = pool.take(50)
    assert e.size == 50 and e.dtype == np.float32


def test_pool_reuses_the_round_before_last():
    """Scatter-and-gather holds round r-1's result while round r is computed: r reuses r-2's array."""
    pool = HostArenaPool(depth=3)
    prev = pool.take(64)
    ids = [id(prev)]
    for _ in range(4):
        cur = pool.take(64)
        ids.append(id(cur))
        assert cur is not prev
        prev = cur  # the caller drops the older result only now
    assert len(set(ids)) == 2
