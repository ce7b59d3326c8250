"""FedAvg-workflow drop-in on the GPU vs the reference's own outputs (tests/golden/fedavg_cases.*).

* ``aggregate_fn`` cases: ``BaseFedAvg.aggregate_fn`` (base_fedavg.py:197-230) run by make_golden.py
  --set fedavg; ours is ``nvflare_amd.app_common.workflows.aggregate_fn``.
* ``fedavg_intime`` cases: FedAvg's built-in in-time path (fedavg.py:268-366); ours is
  ``DeviceFedAvgModelAggregator`` (the ``FedAvg(aggregator=...)`` surface, model_aggregator.py:26-83).
Params bit-exact (NaN payloads excepted), metrics and meta exactly equal."""

import numpy as np
import pytest
import torch

from golden_util import fl_models_from_case, load_fedavg_golden, same_bits, same_metrics
from nvflare_amd.app_common.aggregators import DeviceFedAvgModelAggregator
from nvflare_amd.app_common.workflows import aggregate_fn, make_aggregate_fn
from nvflare_amd.compat import FLContext, FLModel

pytestmark = pytest.mark.gpu

META, ARRAYS = load_fedavg_golden()
CASES = META["cases"]


def _check(case, out):
    exp = case["expected"]
    assert set(out.params) == set(exp["params"])
    for k, name in exp["params"].items():
        got = out.params[k]
        if case["container"] == "torch":
            assert isinstance(got, torch.Tensor) and str(got.dtype).replace("torch.", "") == exp["params_dtype"][k]
            got = got.numpy()
        else:
            assert isinstance(got, np.ndarray) and str(got.dtype) == exp["params_dtype"][k]
        assert same_bits(got, ARRAYS[name]), (case["name"], k)
    assert str(out.params_type.value) == exp["params_type"]
    assert same_metrics(out.metrics, exp["metrics"]), (out.metrics, exp["metrics"])
    assert out.meta["nr_aggregated"] == exp["meta"]["nr_aggregated"]
    assert out.meta["current_round"] == exp["meta"]["current_round"]
    assert out.meta["metrics_aggregation_info"] == exp["meta"]["metrics_aggregation_info"]


@pytest.mark.parametrize("case", [c for c in CASES if c["kind"] == "aggregate_fn"], ids=lambda c: c["name"])
def test_aggregate_fn_matches_reference(case):
    models = fl_models_from_case(case, ARRAYS, FLModel, case["container"])
    _check(case, aggregate_fn(models, device=0))


@pytest.mark.parametrize("case", [c for c in CASES if c["kind"] == "aggregate_fn"][:1], ids=lambda c: c["name"])
def test_make_aggregate_fn_sharded(case):
    """The bound form, split over three buckets on one device (bit-identical by construction)."""
    models = fl_models_from_case(case, ARRAYS, FLModel, case["container"])
    _check(case, make_aggregate_fn(devices=[0, 0, 0])(models))


@pytest.mark.parametrize("case", [c for c in CASES if c["kind"] == "fedavg_intime"], ids=lambda c: c["name"])
def test_model_aggregator_matches_fedavg_intime(case):
    agg = DeviceFedAvgModelAggregator(aggregation_weights=case["aggregation_weights"], device=0)
    ctx = FLContext()
    agg.handle_event("_start_run", ctx)
    for _round in range(2):  # the aggregator resets itself: a second round gives the same bits
        models = fl_models_from_case(case, ARRAYS, FLModel, case["container"])
        accepted = [bool(agg.accept_model(m)) for m in models]
        assert accepted == case["accepted"]
        out = agg.aggregate_model()
        assert out.current_round == case["expected"]["current_round"]
        _check(case, out)
        stats = ctx.get_prop("_aggregation_stats")
        if stats is not None:
            assert stats["accepted_contributions"] == len(models)


def test_model_aggregator_via_shareable():
    """ScatterAndGather surface of ModelAggregator: accept(Shareable) -> aggregate() -> Shareable."""
    from nvflare_amd.compat import FLModelUtils

    rng = np.random.default_rng(5)
    rows = [rng.standard_normal(5000).astype(np.float32) for _ in range(3)]
    agg = DeviceFedAvgModelAggregator(device=0)
    ctx = FLContext()
    for i, r in enumerate(rows):
        s = FLModelUtils.to_shareable(FLModel(params_type="DIFF", params={"w": r}, current_round=1,
                                              meta={"NUM_STEPS_CURRENT_ROUND": i + 1, "client_name": f"c{i}"}))
        assert agg.accept(s, ctx)
    out = FLModelUtils.from_shareable(agg.aggregate(ctx))
    t = rows[0] * np.float32(1.0)
    for i in (1, 2):
        t = t + rows[i] * np.float32(i + 1)
    np.testing.assert_array_equal(out.params["w"], t * np.float32(1.0 / 6.0))
    assert out.params_type.value == "DIFF"


def test_torch_alpha_overflow_raises_like_torch():
    """torch's add_(alpha=1e300) on an fp32 total raises; the drop-in raises the same error type."""
    models = [FLModel(params={"w": torch.ones(8)}, meta={"NUM_STEPS_CURRENT_ROUND": s, "client_name": f"c{i}"})
              for i, s in enumerate([2, 1e300])]
    with pytest.raises(RuntimeError, match="without overflow"):
        aggregate_fn(models, device=0)
    # the first contribution is a mul (no range check): torch.ones(8).mul(1e300).div_(1e300) is all NaN
    out = aggregate_fn(models[1:], device=0)
    assert torch.isnan(out.params["w"]).all()
