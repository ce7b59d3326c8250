"""``ModelAggregator`` for ``FedAvg(aggregator=...)`` that sums on the MI355X.

Reproduces the FedAvg workflow's built-in in-time aggregation
(``nvflare/app_common/workflows/fedavg.py:268-366``, ``_aggregate_one_result`` /
``_get_aggregated_result``) behind the secondary drop-in surface
``ModelAggregator.accept_model / aggregate_model / reset_stats``
(``nvflare/app_common/aggregators/model_aggregator.py:26-83``):

* weight = ``aggregation_weights.get(client, 1.0) * _get_num_steps_weight(result)``  (fedavg.py:297-303,
  base_fedavg.py:93-104), arrival order = ``accept_model`` order;
* params through the drop-in ``WeightedAggregationHelper`` (HIP kernel), bit-identical to the reference
  helper in numpy or torch mode according to the container type;
* metrics: host-side weighted average of the aggregatable entries, disabled for the round as soon as
  one client omits metrics (fedavg.py:317-334).
"""

from __future__ import annotations

import threading
from typing import Dict, Optional

from ...compat import AppConstants, FLModel, ModelAggregator
from ..fedavg_rules import get_client_name, get_num_steps_weight, make_fedavg_metrics_aggregation_info
from .weighted_aggregation_helper import AggregationStatsKey, WeightedAggregationHelper, filter_aggregatable_metrics


class DeviceFedAvgModelAggregator(ModelAggregator):
    def __init__(self, aggregation_weights: Optional[Dict[str, float]] = None, device: Optional[int] = None,
                 devices: Optional[list] = None, max_resident_bytes: Optional[int] = None, defer_result: bool = False):
        """Args:
            aggregation_weights: per-client multipliers (FedAvg's ``aggregation_weights``), default 1.0.
            device / devices / max_resident_bytes: passed to the drop-in ``WeightedAggregationHelper``.
            defer_result: fp32 params of the aggregate stay in HBM as ``DeferredAggregate`` values; the FedOpt
                controller drop-in (app_opt/pt/fedopt_ctl.py) then aggregates and steps them in one launch.
        """
        super().__init__()
        self.aggregation_weights = dict(aggregation_weights or {})
        self._helper = WeightedAggregationHelper(device=device, devices=devices, max_resident_bytes=max_resident_bytes,
                                                 defer_result=defer_result)
        self._lock = threading.Lock()
        self.reset_stats()

    def reset_stats(self):
        with self._lock:
            self._helper.reset_stats()
            self._metrics_helper = WeightedAggregationHelper()
            self._all_metrics = True
            self._warned_metric_keys = set()
            self._site_weights = {}
            self._params_type = None
            self._current_round = None
            self._received = 0

    def accept_model(self, model: FLModel):
        client = get_client_name(model)
        if not model.params:
            self.warning(f"Empty result from client {client}, skipping.")
            return False
        with self._lock:
            if self._params_type is None:
                self._params_type = model.params_type
            if self._current_round is None:
                self._current_round = model.current_round
            weight = self.aggregation_weights.get(client, 1.0) * get_num_steps_weight(model)
            self._site_weights[client] = {"name": client, "weight": weight, "weight_key": "effective_fedavg_metric_weight"}
            self._helper.add(data=model.params, weight=weight, contributor_name=client,
                             contribution_round=model.current_round)
            if model.metrics is None:
                self._all_metrics = False
            if self._all_metrics and model.metrics:
                aggregatable = filter_aggregatable_metrics(
                    model.metrics, warn_skipped=lambda k, tn: self.warning(f"Metric '{k}' ({tn}) skipped for aggregation."),
                    warned_metric_keys=self._warned_metric_keys)
                if aggregatable:
                    self._metrics_helper.add(data=aggregatable, weight=weight, contributor_name=client,
                                             contribution_round=model.current_round)
            self._received += 1
            return True

    def aggregate_model(self) -> FLModel:
        with self._lock:
            if self._received == 0:
                raise RuntimeError("nvflare_amd: aggregate_model() called before any model was accepted")
            if self.fl_ctx is not None:
                stats = self._helper.get_aggregation_stats()
                stats[AggregationStatsKey.ROUND] = self._current_round
                self.fl_ctx.set_prop(AppConstants.AGGREGATION_STATS, stats, private=True, sticky=False)
            params = self._helper.get_result()
            metrics = (self._metrics_helper.get_result() or None) if self._all_metrics else None
            site_weights = list(self._site_weights.values()) or None  # fedavg.py:367-380
            info = make_fedavg_metrics_aggregation_info(
                weight_key="effective_fedavg_metric_weight" if site_weights else "NUM_STEPS_CURRENT_ROUND",
                weight_formula="aggregation_weight * NUM_STEPS_CURRENT_ROUND" if site_weights else None,
                site_weights=site_weights)
            result = FLModel(
                params=params,
                params_type=self._params_type,
                metrics=metrics,
                current_round=self._current_round,
                meta={
                    "nr_aggregated": self._received,
                    "current_round": self._current_round,
                    AppConstants.METRICS_AGGREGATION_INFO: info,
                },
            )
        self.reset_stats()
        return result
