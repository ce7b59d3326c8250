"""FedAvg-workflow drop-in, host logic only.

The weight rule (base_fedavg.py:93-104) is checked against the NUM_STEPS values and effective weights
the reference itself recorded in tests/golden/fedavg_cases.json; the ModelAggregator / FLModel stand-ins
against model_aggregator.py:26-83 and fl_model_utils.py:46-149."""

import math

import numpy as np
import pytest

from golden_util import decode_steps, load_fedavg_golden
from nvflare_amd.app_common.fedavg_rules import get_client_name, get_num_steps_weight
from nvflare_amd.compat import DataKind, FLModel, FLModelUtils, ParamsType


def _model(steps=None, name=None):
    meta = {}
    if steps is not None:
        meta["NUM_STEPS_CURRENT_ROUND"] = steps
    if name is not None:
        meta["client_name"] = name
    return FLModel(params={"w": np.zeros(1, np.float32)}, meta=meta)


@pytest.mark.parametrize(
    "steps,expected",
    [(None, 1.0), (True, 1.0), (False, 1.0), (-2, 1.0), (0, 1.0), (float("nan"), 1.0), (float("inf"), 1.0),
     ("7", 7.0), ("abc", 1.0), (2.5, 2.5), (3, 3.0), (1e300, 1e300), ([1], 1.0), (10**400, 1.0)],
)
def test_num_steps_weight_rule(steps, expected):
    assert get_num_steps_weight(_model(steps)) == expected


def test_client_name_rule():
    assert get_client_name(_model(name="site-3")) == "site-3"
    assert get_client_name(_model(name="")) == "unknown"
    assert get_client_name(_model(name=5)) == "unknown"
    assert get_client_name(_model()) == "unknown"


def test_weight_rule_matches_reference_site_weights():
    """The reference recorded its effective weights (aggregation_weight * rule) in site_weights."""
    meta, _ = load_fedavg_golden()
    n = 0
    for case in meta["cases"]:
        if case["kind"] != "fedavg_intime":
            continue
        aw = case["aggregation_weights"] or {}
        recorded = {s["name"]: s["weight"] for s in case["expected"]["meta"]["metrics_aggregation_info"]["site_weights"]}
        for c in case["clients"]:
            name = c["name"] if c["name"] else "unknown"
            steps = decode_steps(c["num_steps"])
            m = _model(steps, c["name"])
            assert aw.get(name, 1.0) * get_num_steps_weight(m) == recorded[name]
            n += 1
    assert n > 10


def test_flmodel_shareable_round_trip():
    m = FLModel(params_type="DIFF", params={"w": np.arange(3, dtype=np.float32)}, metrics={"acc": 0.5}, current_round=2,
                meta={"NUM_STEPS_CURRENT_ROUND": 4})
    s = FLModelUtils.to_shareable(m)
    back = FLModelUtils.from_shareable(s)
    assert back.params_type == ParamsType.DIFF
    assert back.current_round == 2
    assert back.metrics == {"acc": 0.5}
    assert back.meta["NUM_STEPS_CURRENT_ROUND"] == 4
    np.testing.assert_array_equal(back.params["w"], m.params["w"])
    full = FLModelUtils.from_shareable(FLModelUtils.to_shareable(FLModel(params={"w": 1})))
    assert full.params_type == ParamsType.FULL


def test_flmodel_validation():
    with pytest.raises(ValueError):
        FLModel(params_type="FULL")
    with pytest.raises(ValueError):
        FLModel(params={"w": 1}, current_round=-1)
    assert FLModel().params_type is None
    assert DataKind.WEIGHT_DIFF == "WEIGHT_DIFF"
    assert not math.isnan(get_num_steps_weight(FLModel()))
