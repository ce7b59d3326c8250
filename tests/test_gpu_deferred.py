"""SAG-level fusion: deferred aggregation results stepped by the device FedOpt generator in one launch.

``InTimeAccumulateWeightedAggregator(defer_result=True)`` leaves the aggregated fp32 differences in HBM
(nvflare_amd/deferred.py); ``PTFedOptModelShareableGenerator`` then runs the K-client aggregation and the
SGD / Adam / AdamW step in the same kernel launch.  The bar is bitwise equality with the eager device
flow (aggregate -> host arrays -> generator copies them back and steps with K = 0), which is itself
pinned to the reference by tests/test_gpu_fedopt_generator.py and tests/test_gpu_parity.py: same
weights every round, same optimizer state, same aggregated differences when materialised, for numpy and
torch containers, one slab, several slab geometries (first-round slab growth), more than 128 clients
(chained launches), a key missing from one client, and BatchNorm buffers (fp32 running stats through the
FedAvg branch, int64 num_batches_tracked through the host arithmetic)."""

import copy

import numpy as np
import pytest
import torch

from golden_util import fedopt_model, same_bits
from nvflare_amd.app_common.aggregators import InTimeAccumulateWeightedAggregator
from nvflare_amd.app_opt.pt import PTFedOptModelShareableGenerator
from nvflare_amd.compat import (
    DXO,
    AppConstants,
    DataKind,
    EventType,
    FLContext,
    MetaKey,
    ModelLearnableKey,
    ReservedKey,
    from_shareable,
    make_model_learnable,
)
from nvflare_amd.deferred import DeferredAggregate, DeferredValue, materialize_deferred

pytestmark = pytest.mark.gpu

OPTS = {
    "sgd_nesterov": {"path": "torch.optim.SGD", "args": {"lr": 0.5, "momentum": 0.9, "nesterov": True,
                                                          "weight_decay": 1e-3}},
    "adam": {"path": "torch.optim.Adam", "args": {"lr": 1e-2, "betas": [0.8, 0.95], "eps": 1e-6}},
    "adamw": {"path": "torch.optim.AdamW", "args": {"lr": 1e-2, "weight_decay": 0.05}},
    # optimizers with host-side per-parameter state (NAdam mu_product, ASGD eta / mu) or lazily made state (Rprop)
    "nadam": {"path": "torch.optim.NAdam", "args": {"lr": 1e-2, "momentum_decay": 5e-3}},
    "radam": {"path": "torch.optim.RAdam", "args": {"lr": 1e-2, "betas": [0.8, 0.9]}},
    "adamax": {"path": "torch.optim.Adamax", "args": {"lr": 1e-2}},
    "rprop": {"path": "torch.optim.Rprop", "args": {"lr": 1e-2}},
    "asgd": {"path": "torch.optim.ASGD", "args": {"lr": 1e-2, "t0": 1}},
}


def _np(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return np.asarray(v)


def _client_diff(rng, weights, k, rnd, container, drop_key=None):
    out = {}
    for name, w in weights.items():
        if name == drop_key:
            continue
        a = _np(w)
        if a.dtype == np.int64:
            d = np.array(1, np.int64)
        else:
            d = np.asarray(rng.standard_normal(a.shape) * 0.01, dtype=np.float32)
        out[name] = torch.from_numpy(d) if container == "torch" else d
    return out


def run_fedopt_sag(defer, container, opt, n_clients, rounds=3, drop=None, seed=0, devices=None, model_fn=None,
                   opt_args=None, sched_args=None, between_rounds=None, edit_weights=None):
    """ScatterAndGather's accept -> aggregate -> shareable_to_learnable -> reset loop (scatter_and_gather.py:
    224-349) with the drop-in aggregator and FedOpt generator; returns per-round weights, aggregated
    differences, optimizer state (one device) and the generator.  ``devices``: both sharded over them."""
    torch.manual_seed(seed)
    model = (model_fn or fedopt_model)()
    gen = PTFedOptModelShareableGenerator(optimizer_args=copy.deepcopy(opt_args or OPTS[opt]), source_model=model,
                                          device=0, devices=devices, lr_scheduler_args=copy.deepcopy(sched_args))
    fl_ctx = FLContext()
    gen.handle_event(EventType.START_RUN, fl_ctx)
    agg = InTimeAccumulateWeightedAggregator(expected_data_kind=DataKind.WEIGHT_DIFF, defer_result=defer,
                                             devices=devices)
    agg.handle_event(EventType.START_RUN, fl_ctx)
    weights = {k: v.detach().cpu().clone() if container == "torch" else v.detach().cpu().numpy().copy()
               for k, v in model.state_dict().items()}
    rng = np.random.default_rng(seed + 1)
    hist = []
    for rnd in range(rounds):
        fl_ctx.set_prop(AppConstants.CURRENT_ROUND, rnd, private=True, sticky=True)
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable(weights, {}), private=True, sticky=True)
        for k in range(n_clients):
            drop_key = drop if (k == 0 and rnd == 1) else None
            s = DXO(DataKind.WEIGHT_DIFF, data=_client_diff(rng, weights, k, rnd, container, drop_key),
                    meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1 + (37 * k) % 11}).to_shareable()
            s.set_peer_props({ReservedKey.IDENTITY_NAME: f"site-{k}"})
            s.add_cookie(AppConstants.CONTRIBUTION_ROUND, rnd)
            assert agg.accept(s, fl_ctx)
        aggr = agg.aggregate(fl_ctx)
        diff = from_shareable(aggr).data
        if defer:
            assert any(isinstance(v, DeferredValue) for v in diff.values())
        learnable = gen.shareable_to_learnable(aggr, fl_ctx)
        weights = learnable[ModelLearnableKey.WEIGHTS]
        agg.reset(fl_ctx)
        diff_host = {k: _np(materialize_deferred(v)).copy() for k, v in diff.items()}
        hist.append(({k: _np(v).copy() for k, v in weights.items()}, diff_host))
        if edit_weights is not None:  # a filter / persistor writing into the returned global model in place
            edit_weights(rnd, weights)
        if between_rounds is not None:  # may load new weights into the model; they become the global model
            new = between_rounds(rnd, model, gen)
            if new is not None:
                weights = {k: v.detach().cpu().clone() if container == "torch" else v.detach().cpu().numpy().copy()
                           for k, v in new.items()}
    dev = gen._dev_opt
    state = (dev.p.cpu().numpy().copy(), dev.m.cpu().numpy().copy(), dev.v.cpu().numpy().copy()) if devices is None else None
    return hist, state, gen


def _assert_same(a, b, what):
    assert set(a) == set(b), what
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, (what, k)
        assert same_bits(a[k], b[k]), (what, k)


@pytest.mark.parametrize("container", ["numpy", "torch"])
@pytest.mark.parametrize("opt", list(OPTS))
@pytest.mark.parametrize("n_clients", [5, 40])
def test_deferred_fedopt_matches_eager(container, opt, n_clients):
    eager, st_e, _ = run_fedopt_sag(False, container, opt, n_clients)
    fused, st_f, gen = run_fedopt_sag(True, container, opt, n_clients)
    for rnd, ((we, de), (wf, df)) in enumerate(zip(eager, fused)):
        _assert_same(we, wf, f"weights round {rnd}")
        _assert_same(de, df, f"aggregated diff round {rnd}")
    for a, b in zip(st_e, st_f):
        assert same_bits(a, b)
    # every parameter went through the fused launch: the K = 0 staging buffer was never needed
    assert gen._dev_opt.g is None


def test_deferred_fedopt_many_clients_and_partial_key():
    """>128 clients (chained launches inside the fused step) and a parameter one client left out."""
    for opt in ("adam", "sgd_nesterov"):
        eager, st_e, _ = run_fedopt_sag(False, "numpy", opt, 131, rounds=2, drop="lin2.weight")
        fused, st_f, _ = run_fedopt_sag(True, "numpy", opt, 131, rounds=2, drop="lin2.weight")
        for (we, de), (wf, df) in zip(eager, fused):
            _assert_same(we, wf, opt)
            _assert_same(de, df, opt)
        for a, b in zip(st_e, st_f):
            assert same_bits(a, b)


def _stage(agg, fl_ctx, rnd, rows):
    for k, r in enumerate(rows):
        s = DXO(DataKind.WEIGHT_DIFF, data={"w": r, "b": r[:1000].copy()},
                meta={MetaKey.NUM_STEPS_CURRENT_ROUND: k + 1}).to_shareable()
        s.set_peer_props({ReservedKey.IDENTITY_NAME: f"site-{k}"})
        s.add_cookie(AppConstants.CONTRIBUTION_ROUND, rnd)
        assert agg.accept(s, fl_ctx)


def test_deferred_values_settle_on_next_round():
    """A deferred round nobody consumed is finished on the device when the next round stages; its values
    stay readable (materialize / np.asarray / arithmetic) and equal the eager results."""
    rng = np.random.default_rng(5)
    rows0 = [rng.standard_normal(70_001).astype(np.float32) for _ in range(6)]
    rows1 = [rng.standard_normal(70_001).astype(np.float32) for _ in range(6)]
    ref = {}
    for defer in (False, True):
        agg = InTimeAccumulateWeightedAggregator(expected_data_kind=DataKind.WEIGHT_DIFF, defer_result=defer)
        fl_ctx = FLContext()
        agg.handle_event(EventType.START_RUN, fl_ctx)
        outs = []
        for rnd, rows in enumerate((rows0, rows1)):
            fl_ctx.set_prop(AppConstants.CURRENT_ROUND, rnd, private=True, sticky=True)
            _stage(agg, fl_ctx, rnd, rows)
            outs.append(from_shareable(agg.aggregate(fl_ctx)).data)
            agg.reset(fl_ctx)
        if not defer:
            ref = outs
            continue
        for (o, r) in zip(outs, ref):
            for k in ("w", "b"):
                assert isinstance(o[k], DeferredAggregate)
                assert same_bits(np.asarray(o[k]), r[k])
                assert same_bits(o[k].materialize(), r[k])
        assert same_bits(outs[0]["b"] + np.float32(1), ref[0]["b"] + np.float32(1))


@pytest.mark.parametrize("container", ["numpy", "torch"])
def test_deferred_full_model_weight_diff_apply(container):
    """FullModelShareableGenerator on a deferred WEIGHT_DIFF: aggregation and ``base + diff`` in one launch,
    bit-identical to the eager flow; the difference stays materialisable afterwards."""
    from nvflare_amd.app_common.shareablegenerators import FullModelShareableGenerator

    rng = np.random.default_rng(11)
    shapes = {"a": (33, 129), "b": (5000,), "c": (3, 3)}
    base = {k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()}
    base["n"] = np.array(7, np.int64)
    rows = [{k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()} for _ in range(19)]
    for r in rows:
        r["n"] = np.array(2, np.int64)
    conv = (lambda a: torch.from_numpy(np.array(a, copy=True))) if container == "torch" else (lambda a: np.array(a, copy=True))
    results = {}
    for defer in (False, True):
        agg = InTimeAccumulateWeightedAggregator(expected_data_kind=DataKind.WEIGHT_DIFF, defer_result=defer)
        gen = FullModelShareableGenerator(device=0)
        fl_ctx = FLContext()
        agg.handle_event(EventType.START_RUN, fl_ctx)
        fl_ctx.set_prop(AppConstants.CURRENT_ROUND, 0, private=True, sticky=True)
        fl_ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable({k: conv(v) for k, v in base.items()}, {}),
                        private=True, sticky=True)
        for k, r in enumerate(rows):
            s = DXO(DataKind.WEIGHT_DIFF, data={n: conv(v) for n, v in r.items()},
                    meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 1 + k % 4}).to_shareable()
            s.set_peer_props({ReservedKey.IDENTITY_NAME: f"site-{k}"})
            s.add_cookie(AppConstants.CONTRIBUTION_ROUND, 0)
            assert agg.accept(s, fl_ctx)
        aggr = agg.aggregate(fl_ctx)
        diff = from_shareable(aggr).data
        out = gen.shareable_to_learnable(aggr, fl_ctx)[ModelLearnableKey.WEIGHTS]
        if defer:
            assert all(diff[k].round.keys[k].done for k in shapes)
        results[defer] = ({k: _np(v).copy() for k, v in out.items()},
                          {k: _np(v.materialize() if isinstance(v, DeferredAggregate) else v).copy() for k, v in diff.items()})
    _assert_same(results[False][0], results[True][0], "weights")
    _assert_same(results[False][1], results[True][1], "diff")


@pytest.mark.parametrize("opt", ["adam", "sgd_nesterov"])
def test_deferred_fedopt_pipelined_weight_egress(monkeypatch, opt):
    """Fused step split at small EGRESS_CHUNK boundaries with readiness marks; the new weights leave through
    fedavg_d2h_marked while later pieces compute -- bit-identical to the eager flow."""
    import nvflare_amd.engine as E

    monkeypatch.setattr(E, "EGRESS_CHUNK", 16 << 10)  # 4096 fp32 params per piece: several per tensor
    eager, st_e, _ = run_fedopt_sag(False, "torch", opt, 6)
    fused, st_f, gen = run_fedopt_sag(True, "torch", opt, 6)
    for (we, de), (wf, df) in zip(eager, fused):
        _assert_same(we, wf, opt)
        _assert_same(de, df, opt)
    for a, b in zip(st_e, st_f):
        assert same_bits(a, b)
    assert gen._dev_opt.egress_pending is False
