"""FedAvg-workflow weight and naming rules (leaf module: no aggregator imports).

``base_fedavg.py:37-104`` of the reference: ``_get_client_name``, ``_get_num_steps_weight`` and
``make_fedavg_metrics_aggregation_info``.
"""

from __future__ import annotations

import math
from typing import Any, Dict, List, Optional

from ..compat import AppConstants, FLMetaKey, FLModel


def get_client_name(result: FLModel) -> str:
    """``_get_client_name`` (base_fedavg.py:87-90)."""
    meta = result.meta or {}
    value = meta.get("client_name", AppConstants.CLIENT_UNKNOWN)
    return value if isinstance(value, str) and value else AppConstants.CLIENT_UNKNOWN


def get_num_steps_weight(result: FLModel) -> float:
    """``_get_num_steps_weight`` (base_fedavg.py:93-104): NUM_STEPS_CURRENT_ROUND as a float; None, bools,
    non-numbers, non-finite and non-positive values all weigh 1.0."""
    value = (result.meta or {}).get(FLMetaKey.NUM_STEPS_CURRENT_ROUND)
    if value is None or isinstance(value, bool):
        return 1.0
    try:
        weight = float(value)
    except (TypeError, ValueError, OverflowError):
        return 1.0
    if not math.isfinite(weight) or weight <= 0:
        return 1.0
    return weight


def make_fedavg_metrics_aggregation_info(weight_key: str = FLMetaKey.NUM_STEPS_CURRENT_ROUND,
                                         weight_formula: Optional[str] = None,
                                         site_weights: Optional[List[Dict[str, Any]]] = None) -> Dict[str, Any]:
    """The ``metrics_aggregation_info`` meta entry (base_fedavg.py:37-66, without key-metric fields)."""
    aggregation = {
        "method": "weighted_average",
        "weight_key": weight_key,
        "metric_policy": "finite_numeric_metrics_only_per_key_denominator",
    }
    if weight_formula:
        aggregation["weight_formula"] = weight_formula
    info = {"metric_source": "client_reported_flmodel_metrics", "aggregation": aggregation}
    if site_weights:
        info["site_weights"] = site_weights
    return info
