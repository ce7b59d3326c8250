"""The drop-in on the GPU: the sag_np known-answer test (config 1) and ports of the reference's own
aggregator unit tests (tests/unit_test/app_common/aggregators/*), which assert with allclose; our
classes are additionally checked bit-exact against the CPU oracle where the reference tests compare
against closed forms."""

import random

import numpy as np
import pytest
import torch

from golden_util import same_bits

pytestmark = pytest.mark.gpu


def _intime(**kw):
    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator

    agg = InTimeAccumulateWeightedAggregator(**kw)
    agg._initialize(agg.aggregation_weights, agg.exclude_vars, agg.expected_data_kind)
    return agg


def _helper(**kw):
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    return WeightedAggregationHelper(**kw)


# --- config 1: job_templates/sag_np, 2 clients, 3 rounds, NPTrainer delta=1 -------------------------------
def test_sag_np_known_answer():
    """tests/integration_test/data/test_configs/standalone_job/np_job.yml:24-25, checked with assert_equal
    as src/validators/np_sag_result_validator.py:39-44 does."""
    from sag_harness import NUMPY_KEY, run_sag

    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator

    agg = InTimeAccumulateWeightedAggregator(expected_data_kind="WEIGHTS", aggregation_weights={"site-1": 1.0, "site-2": 1.0})
    model, fl_ctx = run_sag(agg, n_clients=2, num_rounds=3)
    np.testing.assert_equal(model[NUMPY_KEY], [[4, 5, 6], [7, 8, 9], [10, 11, 12]])
    assert model[NUMPY_KEY].dtype == np.float32


def test_sag_weight_diff_known_answer():
    from sag_harness import NUMPY_KEY, run_sag

    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator

    model, _ = run_sag(InTimeAccumulateWeightedAggregator(), n_clients=3, num_rounds=4, kind="WEIGHT_DIFF", delta=0.5)
    np.testing.assert_equal(model[NUMPY_KEY], np.array([[1, 2, 3], [4, 5, 6], [7, 8, 9]], np.float32) + 2.0)


# --- ports of weighted_aggregation_helper_test.py:196-443 --------------------------------------------------
def test_pytorch_float_single_contribution():
    h = _helper()
    h.add({"w1": torch.tensor([1.0, 2.0, 3.0]), "w2": torch.tensor([4.0, 5.0])}, weight=2.0, contributor_name="site-1", contribution_round=0)
    r = h.get_result()
    assert torch.allclose(r["w1"], torch.tensor([1.0, 2.0, 3.0]))
    assert torch.allclose(r["w2"], torch.tensor([4.0, 5.0]))


def test_pytorch_float_multiple_contributions():
    h = _helper()
    h.add({"w": torch.tensor([2.0, 4.0, 6.0])}, weight=1.0, contributor_name="site-1", contribution_round=0)
    h.add({"w": torch.tensor([3.0, 6.0, 9.0])}, weight=2.0, contributor_name="site-2", contribution_round=0)
    assert torch.allclose(h.get_result()["w"], torch.tensor([8.0 / 3, 16.0 / 3, 24.0 / 3]))


def test_pytorch_int_tensor_weighting():
    h = _helper()
    h.add({"count": torch.tensor([10, 20, 30], dtype=torch.long)}, weight=2.0, contributor_name="site-1", contribution_round=0)
    h.add({"count": torch.tensor([5, 10, 15], dtype=torch.long)}, weight=3.0, contributor_name="site-2", contribution_round=0)
    r = h.get_result()
    assert r["count"].dtype == torch.float32
    assert torch.allclose(r["count"], torch.tensor([7.0, 14.0, 21.0]))


def test_pytorch_mixed_float_int_tensors():
    h = _helper()
    h.add({"weights": torch.tensor([2.0, 4.0]), "counts": torch.tensor([10, 20], dtype=torch.long)}, weight=1.0, contributor_name="site-1", contribution_round=0)
    h.add({"weights": torch.tensor([3.0, 6.0]), "counts": torch.tensor([5, 10], dtype=torch.long)}, weight=2.0, contributor_name="site-2", contribution_round=0)
    r = h.get_result()
    assert torch.allclose(r["weights"], torch.tensor([8.0 / 3, 16.0 / 3]))
    assert torch.allclose(r["counts"], torch.tensor([20.0 / 3, 40.0 / 3]))


def test_numpy_single_and_multiple_contributions():
    h = _helper()
    h.add({"w": np.array([1.0, 2.0, 3.0])}, weight=2.0, contributor_name="site-1", contribution_round=0)
    np.testing.assert_allclose(h.get_result()["w"], np.array([1.0, 2.0, 3.0]))
    h.add({"w": np.array([2.0, 4.0, 6.0])}, weight=1.0, contributor_name="site-1", contribution_round=0)
    h.add({"w": np.array([3.0, 6.0, 9.0])}, weight=2.0, contributor_name="site-2", contribution_round=0)
    r = h.get_result()["w"]
    assert r.dtype == np.float64
    np.testing.assert_allclose(r, np.array([8.0 / 3, 16.0 / 3, 24.0 / 3]))


def test_exclude_vars_regex():
    h = _helper(exclude_vars="bias")
    h.add({"layer1.weight": torch.tensor([1.0, 2.0]), "layer1.bias": torch.tensor([0.1, 0.2]), "layer2.weight": torch.tensor([3.0, 4.0])},
          weight=1.0, contributor_name="site-1", contribution_round=0)
    r = h.get_result()
    assert "layer1.weight" in r and "layer2.weight" in r and "layer1.bias" not in r


def test_weigh_by_local_iter_false():
    h = _helper(weigh_by_local_iter=False)
    h.add({"w": torch.tensor([2.0, 4.0])}, weight=1.0, contributor_name="site-1", contribution_round=0)
    h.add({"w": torch.tensor([4.0, 8.0])}, weight=100.0, contributor_name="site-2", contribution_round=0)
    assert torch.allclose(h.get_result()["w"], torch.tensor([6.0 / 101, 12.0 / 101]))


def test_history_len_reset():
    h = _helper()
    assert h.get_len() == 0
    h.add({"w": torch.tensor([1.0])}, weight=2.0, contributor_name="site-1", contribution_round=0)
    h.add({"w": torch.tensor([2.0])}, weight=3.0, contributor_name="site-2", contribution_round=1)
    assert h.history[0] == {"contributor_name": "site-1", "round": 0, "weight": 2.0}
    assert h.history[1] == {"contributor_name": "site-2", "round": 1, "weight": 3.0}
    assert len(h.total) == 1 and h.get_len() == 2
    h.reset_stats()
    assert len(h.total) == 0 and len(h.counts) == 0 and len(h.history) == 0


def test_empty_data_and_sequence():
    h = _helper()
    h.add({}, weight=1.0, contributor_name="site-1", contribution_round=0)
    assert len(h.get_result()) == 0
    for i in range(10):
        h.add({"w": torch.tensor([float(i)])}, weight=1.0, contributor_name=f"site-{i}", contribution_round=0)
    assert torch.allclose(h.get_result()["w"], torch.tensor([4.5]))


def test_different_keys_per_contribution_and_stats():
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import AggregationStatsKey as K

    h = _helper()
    h.add({"w1": torch.tensor([1.0]), "w2": torch.tensor([2.0])}, weight=1.0, contributor_name="site-1", contribution_round=0)
    h.add({"w2": torch.tensor([3.0]), "w3": torch.tensor([4.0])}, weight=1.0, contributor_name="site-2", contribution_round=0)
    st = h.get_aggregation_stats()
    assert st[K.FULLY_MATCHED_KEYS] == 1 and st[K.PARTIALLY_MATCHED_KEYS] == 2 and st[K.KEYS_AGGREGATED] == 3
    r = h.get_result()
    assert torch.allclose(r["w1"], torch.tensor([1.0]))
    assert torch.allclose(r["w2"], torch.tensor([2.5]))
    assert torch.allclose(r["w3"], torch.tensor([4.0]))
    assert h.last_aggregation_stats[K.ACCEPTED_CONTRIBUTIONS] == 2
    assert h.get_aggregation_stats()[K.ACCEPTED_CONTRIBUTIONS] == 0


def test_non_callable_materialize_attribute_is_host_object():
    class V:
        def __init__(self, value):
            self.materialize = "not-callable"
            self.value = value

        def __mul__(self, other):
            return self.value * other

        def __rmul__(self, other):
            return self.__mul__(other)

        def __add__(self, other):
            return self.value + other

    h = _helper()
    h.add({"w": V(3.0)}, weight=2.0, contributor_name="site-1", contribution_round=0)
    assert h.get_result()["w"] == pytest.approx(3.0)


def test_lazy_materialize_goes_to_device():
    class Lazy:
        def __init__(self, arr):
            self.arr = arr

        def materialize(self):
            return self.arr

    h = _helper()
    h.add({"w": Lazy(np.array([1.0, 3.0], np.float32))}, weight=1.0, contributor_name="a", contribution_round=0)
    h.add({"w": Lazy(np.array([3.0, 5.0], np.float32))}, weight=1.0, contributor_name="b", contribution_round=0)
    np.testing.assert_array_equal(h.get_result()["w"], np.array([2.0, 4.0], np.float32))


# --- ports of in_time_accumulate_weighted_aggregator_test.py:157-385 ---------------------------------------
@pytest.mark.parametrize("current_round,contribution_round,expected", [(1, 1, True), (2, 1, False)])
def test_accept(current_round, contribution_round, expected):
    from nvflare_amd.compat import DXO, AppConstants, DataKind, FLContext, MetaKey, ReservedKey, Shareable

    agg = _intime(aggregation_weights={f"client_{i}": random.random() for i in range(2)})
    fl_ctx = FLContext()
    s = Shareable()
    s.set_peer_props({ReservedKey.IDENTITY_NAME: "client_0"})
    s.add_cookie(AppConstants.CONTRIBUTION_ROUND, contribution_round)
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, current_round)
    dxo = DXO(DataKind.WEIGHT_DIFF, data={"var1": np.random.random(4)}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1})
    assert agg.accept(dxo.update_shareable(s), fl_ctx) == expected


def _submit(agg, fl_ctx, name, dxo, rnd=0):
    from nvflare_amd.compat import AppConstants, ReservedKey, Shareable

    s = Shareable()
    s.set_peer_props({ReservedKey.IDENTITY_NAME: name})
    s.add_cookie(AppConstants.CONTRIBUTION_ROUND, rnd)
    return agg.accept(dxo.update_shareable(s), fl_ctx)


@pytest.mark.parametrize("shape", [4, (6, 6)])
@pytest.mark.parametrize("n_clients", [10, 50, 100])
def test_aggregate_random(shape, n_clients, oracle):
    from nvflare_amd.compat import DXO, AppConstants, DataKind, FLContext, MetaKey, from_shareable

    aw = {f"client_{i}": random.random() for i in range(n_clients)}
    agg = _intime(aggregation_weights=aw)
    weighted_sum, sum_w = np.zeros(shape), 0
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0)
    rows, ws = [], []
    for name in aw:
        it = random.randint(1, 50)
        w = np.random.random(shape)
        weighted_sum = weighted_sum + w * it * aw[name]
        sum_w = sum_w + it * aw[name]
        rows.append(w)
        ws.append(aw[name] * float(it))
        assert _submit(agg, fl_ctx, name, DXO(DataKind.WEIGHT_DIFF, data={"var1": w}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: it}))
    res = from_shareable(agg.aggregate(fl_ctx)).data["var1"]
    np.testing.assert_allclose(res, weighted_sum / sum_w)
    # and bit-exact against the pinned oracle's numpy mode (fp64 arrays)
    assert same_bits(res.reshape(-1), oracle.fedavg_c([r.reshape(-1) for r in rows], ws, oracle.MODE_NUMPY))


@pytest.mark.parametrize("defer", [False, True])
def test_intime_devices_shards_parameter_buckets(oracle, defer):
    """``devices=[...]`` on the InTime aggregator: every key split into parameter buckets over several engines
    (here three on device 0), fp32 results bit-exact with the oracle; with ``defer_result`` they are
    ``ShardedDeferredAggregate`` values (one piece per engine) that materialise to the same bits."""
    from nvflare_amd.compat import DXO, AppConstants, DataKind, FLContext, MetaKey, from_shareable
    from nvflare_amd.sharding import ShardedFedAvg

    rng = np.random.default_rng(17)
    agg = _intime(devices=[0, 0, 0], defer_result=defer)
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0)
    rows, ws = [], []
    for i in range(5):
        w = rng.standard_normal(3 * 4096 + 77).astype(np.float32)
        rows.append(w)
        ws.append(float(1 + 3 * i))
        dxo = DXO(DataKind.WEIGHT_DIFF, data={"w": w, "b": w[:10].copy()}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1 + 3 * i})
        assert _submit(agg, fl_ctx, f"site-{i}", dxo)
    assert isinstance(agg.dxo_aggregators[""].aggregation_helper.engine, ShardedFedAvg)
    out = from_shareable(agg.aggregate(fl_ctx)).data
    if defer:
        from nvflare_amd.deferred import ShardedDeferredAggregate

        assert isinstance(out["w"], ShardedDeferredAggregate) and len(out["w"].pieces) == 3
        out = {k: np.asarray(v) for k, v in out.items()}
    assert isinstance(out["w"], np.ndarray)
    assert same_bits(out["w"], oracle.fedavg_c(rows, ws, oracle.MODE_NUMPY))
    assert same_bits(out["b"], oracle.fedavg_c([r[:10].copy() for r in rows], ws, oracle.MODE_NUMPY))


@pytest.mark.parametrize("num_dxo", [1, 2, 3])
@pytest.mark.parametrize("n_clients", [10, 50])
def test_aggregate_random_dxos(num_dxo, n_clients):
    from nvflare_amd.compat import DXO, AppConstants, DataKind, FLContext, MetaKey, from_shareable

    names = [f"dxo_{i}" for i in range(num_dxo)]
    clients = [f"client_{i}" for i in range(n_clients)]
    aw = {d: {c: random.random() for c in clients} for d in names}
    agg = _intime(aggregation_weights=aw, expected_data_kind={d: DataKind.WEIGHT_DIFF for d in names})
    wsum = {d: np.zeros((6, 6)) for d in names}
    sw = {d: 0 for d in names}
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0)
    for c in clients:
        it = random.randint(1, 50)
        coll = {}
        for d in names:
            v = np.random.random((6, 6))
            coll[d] = DXO(data_kind=DataKind.WEIGHT_DIFF, data={"var1": v}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: it})
            wsum[d] = wsum[d] + v * it * aw[d][c]
            sw[d] = sw[d] + it * aw[d][c]
        assert _submit(agg, fl_ctx, c, DXO(data_kind=DataKind.COLLECTION, data=coll))
    res = from_shareable(agg.aggregate(fl_ctx))
    for d in names:
        np.testing.assert_allclose(res.data[d].data["var1"], wsum[d] / sw[d])


def test_aggregate_publishes_aggregation_stats():
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import AggregationStatsKey as K
    from nvflare_amd.compat import DXO, AppConstants, DataKind, FLContext, MetaKey

    agg = _intime(exclude_vars="bias")
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0)
    contributions = {
        "client1": {"var1": np.array([1.0]), "var2": np.array([2.0]), "bias": np.array([0.5])},
        "client2": {"var1": np.array([3.0])},
    }
    for name, data in contributions.items():
        assert _submit(agg, fl_ctx, name, DXO(DataKind.WEIGHT_DIFF, data=data, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1}))
    agg.aggregate(fl_ctx)
    st = fl_ctx.get_prop(AppConstants.AGGREGATION_STATS)
    assert st[K.ROUND] == 0 and st[K.ACCEPTED_CONTRIBUTIONS] == 2 and st[K.CONTRIBUTORS] == ["client1", "client2"]
    assert (st[K.KEYS_AGGREGATED], st[K.KEYS_SEEN], st[K.FULLY_MATCHED_KEYS], st[K.PARTIALLY_MATCHED_KEYS], st[K.SKIPPED_KEYS]) == (2, 3, 1, 1, 1)


def test_rejections_return_false():
    from nvflare_amd.compat import DXO, AppConstants, DataKind, FLContext, MetaKey, ReturnCode

    agg = _intime(expected_data_kind=DataKind.WEIGHTS)
    fl_ctx = FLContext()
    fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 3)
    good = DXO(DataKind.WEIGHTS, data={"w": np.ones(3, np.float32)}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 2})
    assert _submit(agg, fl_ctx, "a", good, rnd=3)
    assert not _submit(agg, fl_ctx, "a", good, rnd=3)  # duplicate contributor
    assert not _submit(agg, fl_ctx, "b", DXO(DataKind.WEIGHT_DIFF, data={"w": np.ones(3, np.float32)}), rnd=3)  # wrong kind
    assert not _submit(agg, fl_ctx, "c", good, rnd=2)  # stale round
    from nvflare_amd.compat import AppConstants as AC, ReservedKey, Shareable

    s = good.to_shareable()
    s.set_peer_props({ReservedKey.IDENTITY_NAME: "d"})
    s.add_cookie(AC.CONTRIBUTION_ROUND, 3)
    s.set_return_code(ReturnCode.EXECUTION_EXCEPTION)
    assert not agg.accept(s, fl_ctx)
    assert not agg.accept(Shareable(), fl_ctx)  # not a DXO
    res = agg.aggregate(fl_ctx)
    from nvflare_amd.compat import from_shareable

    np.testing.assert_array_equal(from_shareable(res).data["w"], np.ones(3, np.float32))
