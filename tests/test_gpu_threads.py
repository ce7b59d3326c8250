"""Threading (row a11): ``LazyAggregator`` (nvflare/app_common/aggregators/lazy.py:42-197) runs the wrapped
aggregator's ``accept`` on a worker thread and ``aggregate`` on the controller thread once the queue has
drained; ScatterAndGather can also let late ``accept`` calls overlap ``aggregate`` (scatter_and_gather.py:
381-391).  The drop-in keeps the reference's lock discipline (weighted_aggregation_helper.py:162,228); the
HIP handle re-binds its device on every call, so any host thread may drive it.

Checked: accepts on a worker thread == sequential accepts (bitwise); accepts racing from several threads
aggregate in the order the helper recorded them (its history), bit-exact against the oracle in that order."""

import queue
import threading

import numpy as np
import pytest

from golden_util import same_bits
from nvflare_amd.app_common.aggregators import InTimeAccumulateWeightedAggregator
from nvflare_amd.compat import DXO, AppConstants, DataKind, EventType, FLContext, MetaKey, ReservedKey, from_shareable

pytestmark = pytest.mark.gpu


def _shareable(k, rows, rnd=0):
    s = DXO(DataKind.WEIGHT_DIFF, data={"w": rows[k], "b": rows[k][:333].copy()},
            meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1 + (37 * k) % 13}).to_shareable()
    s.set_peer_props({ReservedKey.IDENTITY_NAME: f"site-{k}"})
    s.add_cookie(AppConstants.CONTRIBUTION_ROUND, rnd)
    return s


def _new_agg():
    agg = InTimeAccumulateWeightedAggregator(expected_data_kind=DataKind.WEIGHT_DIFF)
    fl_ctx = FLContext()
    agg.handle_event(EventType.START_RUN, fl_ctx)
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0, private=True, sticky=True)
    return agg, fl_ctx


def test_lazy_style_worker_thread_accepts():
    rng = np.random.default_rng(0)
    rows = [rng.standard_normal(100_003).astype(np.float32) for _ in range(12)]
    agg, fl_ctx = _new_agg()
    for k in range(12):
        assert agg.accept(_shareable(k, rows), fl_ctx)
    ref = from_shareable(agg.aggregate(fl_ctx)).data

    agg, fl_ctx = _new_agg()
    q = queue.Queue()
    accepted = []

    def worker():  # LazyAggregator._process_contributions: accept sequentially off the controller thread
        while True:
            item = q.get()
            if item is None:
                return
            accepted.append(agg.accept(item, fl_ctx))
            q.task_done()

    t = threading.Thread(target=worker)
    t.start()
    for k in range(12):
        q.put(_shareable(k, rows))
    q.join()  # LazyAggregator.aggregate waits for the queue to drain (lazy.py:155-176)
    got = from_shareable(agg.aggregate(fl_ctx)).data
    q.put(None)
    t.join()
    assert all(accepted)
    for key in ref:
        assert same_bits(got[key], ref[key]), key


def test_racing_accepts_follow_recorded_arrival_order(oracle):
    rng = np.random.default_rng(1)
    K = 16
    rows = [rng.standard_normal(50_001).astype(np.float32) for _ in range(K)]
    agg, fl_ctx = _new_agg()
    barrier = threading.Barrier(4)

    def client_thread(ks):
        barrier.wait()
        for k in ks:
            assert agg.accept(_shareable(k, rows), fl_ctx)

    threads = [threading.Thread(target=client_thread, args=(list(range(i, K, 4)),)) for i in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    helper = agg.dxo_aggregators[""].aggregation_helper
    order = [int(h["contributor_name"].split("-")[1]) for h in helper.get_history()]
    weights = [h["weight"] for h in helper.get_history()]
    got = from_shareable(agg.aggregate(fl_ctx)).data["w"]
    assert sorted(order) == list(range(K))
    exp = oracle.fedavg_c([rows[k] for k in order], weights, oracle.MODE_NUMPY)
    assert same_bits(got, exp)
