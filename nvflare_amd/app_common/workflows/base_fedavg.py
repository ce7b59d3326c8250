"""FedAvg-workflow aggregation (``FLModel`` lists) on the MI355X.

Drop-in for the parameter path of ``BaseFedAvg.aggregate_fn``
(``nvflare/app_common/workflows/base_fedavg.py:197-230``): the same weight rule
(``_get_num_steps_weight``, ``:93-104``), client naming (``:87-90``), metric averaging
(``_aggregate_fl_model_metrics``, ``:105-126``) and result ``FLModel`` -- with the params summed by the
HIP aggregation engine through the drop-in ``WeightedAggregationHelper``, so the bits match the
reference's helper exactly.

Use::

    from nvflare_amd.app_common.workflows import make_aggregate_fn
    model = controller.aggregate(results, aggregate_fn=make_aggregate_fn(device=0))
"""

from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional

from ...compat import AppConstants, FLModel
from ..aggregators.weighted_aggregation_helper import WeightedAggregationHelper, filter_aggregatable_metrics
from ..fedavg_rules import get_client_name, get_num_steps_weight, make_fedavg_metrics_aggregation_info  # noqa: F401


def aggregate_fl_model_metrics(results: List[FLModel]) -> Optional[Dict[str, Any]]:
    """``_aggregate_fl_model_metrics`` (base_fedavg.py:105-126): host-side weighted average of scalar
    metrics (a handful of Python numbers -- never worth a device round trip)."""
    helper = WeightedAggregationHelper()
    for r in results:
        if r.metrics is None:
            return None
        aggregatable = filter_aggregatable_metrics(r.metrics)
        if aggregatable:
            helper.add(data=aggregatable, weight=get_num_steps_weight(r), contributor_name=get_client_name(r),
                       contribution_round=r.current_round)
    return helper.get_result() or None


def aggregate_fn(results: List[FLModel], device: Optional[int] = None, devices: Optional[list] = None,
                 max_resident_bytes: Optional[int] = None) -> FLModel:
    """``BaseFedAvg.aggregate_fn`` (base_fedavg.py:197-230) with the params aggregated on the GPU."""
    if not results:
        raise ValueError("received empty results for aggregation.")
    helper = WeightedAggregationHelper(device=device, devices=devices, max_resident_bytes=max_resident_bytes)
    for r in results:
        helper.add(data=r.params, weight=get_num_steps_weight(r), contributor_name=get_client_name(r),
                   contribution_round=r.current_round)
    params = helper.get_result()
    return FLModel(
        params=params,
        params_type=results[0].params_type,
        metrics=aggregate_fl_model_metrics(results),
        meta={
            "nr_aggregated": len(results),
            "current_round": results[0].current_round,
            AppConstants.METRICS_AGGREGATION_INFO: make_fedavg_metrics_aggregation_info(),
        },
    )


def make_aggregate_fn(device: Optional[int] = None, devices: Optional[list] = None,
                      max_resident_bytes: Optional[int] = None) -> Callable[[List[FLModel]], FLModel]:
    """Bind the device arguments, giving the ``aggregate_fn(results)`` that ``BaseFedAvg.aggregate``
    (base_fedavg.py:232-262) accepts."""

    def _fn(results: List[FLModel]) -> FLModel:
        return aggregate_fn(results, device=device, devices=devices, max_resident_bytes=max_resident_bytes)

    return _fn
