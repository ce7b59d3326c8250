"""GPU drop-in for ``InTimeAccumulateWeightedAggregator``.

A scatter-and-gather job switches to the MI355X path by changing only the component ``path``
(job_templates/sag_np/config_fed_server.conf:78-82):

    path = "nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator.InTimeAccumulateWeightedAggregator"

Constructor kwargs, START_RUN initialisation, config validation (same ValueError messages),
``accept`` / ``aggregate`` / ``reset`` and the AGGREGATION_STATS publication follow
intime_accumulate_model_aggregator.py:47-288.  Each expected DXO gets a HIP-backed ``DXOAggregator``.
"""

from __future__ import annotations

from typing import Any, Dict, Optional, Union

from ...compat import (
    DXO,
    Aggregator,
    AppConstants,
    DataKind,
    EventType,
    FLContext,
    ReservedKey,
    ReturnCode,
    Shareable,
    from_shareable,
)
from .dxo_aggregator import DXOAggregator
from .weighted_aggregation_helper import AggregationStatsKey

_KINDS = [DataKind.WEIGHT_DIFF, DataKind.WEIGHTS, DataKind.METRICS]
_SUMMED_STATS = (
    AggregationStatsKey.KEYS_AGGREGATED,
    AggregationStatsKey.KEYS_SEEN,
    AggregationStatsKey.FULLY_MATCHED_KEYS,
    AggregationStatsKey.PARTIALLY_MATCHED_KEYS,
    AggregationStatsKey.SKIPPED_KEYS,
)


def _is_nested_aggregation_weights(aggregation_weights) -> bool:
    if not aggregation_weights or not isinstance(aggregation_weights, dict):
        return False
    return isinstance(next(iter(aggregation_weights.values())), dict)


def _get_missing_keys(ref_dict: dict, dict_to_check: dict):
    return [k for k in ref_dict if k not in dict_to_check]


class InTimeAccumulateWeightedAggregator(Aggregator):
    def __init__(
        self,
        exclude_vars: Union[str, Dict[str, str], None] = None,
        aggregation_weights: Union[Dict[str, Any], Dict[str, Dict[str, Any]], None] = None,
        expected_data_kind: Union[DataKind, Dict[str, DataKind]] = DataKind.WEIGHT_DIFF,
        weigh_by_local_iter: bool = True,
        device: Optional[int] = None,
        defer_result: bool = False,
        devices: Optional[list] = None,
    ):
        """Accumulated weighted (FedAvg) aggregation on the MI355X.

        Args: as the reference (intime_accumulate_model_aggregator.py:48-90), plus ``device``, the HIP
        device index of the aggregation engine (default $NVFLARE_AMD_DEVICE or 0), ``defer_result``:
        the aggregated fp32 values stay in HBM as ``DeferredAggregate`` objects until read, so the device
        FedOpt generator steps the model in the same launch as the aggregation (nvflare_amd/deferred.py),
        and ``devices``: several HIP devices, every key split into per-device parameter buckets
        (nvflare_amd/sharding.py; with ``defer_result`` the values are ``ShardedDeferredAggregate`` objects whose
        bucket pieces stay on their devices).
        """
        super().__init__()
        self._single_dxo_key = ""
        self._weigh_by_local_iter = weigh_by_local_iter
        self._device = device
        self._devices = devices
        self._defer_result = defer_result
        self.aggregation_weights = aggregation_weights
        self.exclude_vars = exclude_vars
        self.expected_data_kind = expected_data_kind

    def handle_event(self, event_type: str, fl_ctx: FLContext):
        # initialised on START_RUN, not in the constructor (intime_accumulate_model_aggregator.py:92-97)
        if event_type == EventType.START_RUN:
            self._initialize(self.aggregation_weights, self.exclude_vars, self.expected_data_kind)

    def _initialize(self, aggregation_weights, exclude_vars, expected_data_kind):
        if isinstance(expected_data_kind, dict):
            for k, v in expected_data_kind.items():
                if v not in _KINDS:
                    raise ValueError(
                        f"expected_data_kind[{k}] = {v} is not {DataKind.WEIGHT_DIFF} or {DataKind.WEIGHTS} or {DataKind.METRICS}"
                    )
            self.expected_data_kind = expected_data_kind
        else:
            if expected_data_kind not in _KINDS:
                raise ValueError(
                    f"expected_data_kind = {expected_data_kind} is not {DataKind.WEIGHT_DIFF} or {DataKind.WEIGHTS} or {DataKind.METRICS}"
                )
            self.expected_data_kind = {self._single_dxo_key: expected_data_kind}

        if exclude_vars:
            if not isinstance(exclude_vars, (dict, str)):
                raise ValueError(f"exclude_vars = {exclude_vars} should be a regex string but got {type(exclude_vars)}.")
            if isinstance(exclude_vars, dict):
                missing = _get_missing_keys(expected_data_kind, exclude_vars)
                if missing:
                    raise ValueError(
                        "A dict exclude_vars should specify exclude_vars for every key in expected_data_kind. "
                        f"But missed these keys: {missing}"
                    )
        exclude_by_key = {}
        for k in self.expected_data_kind:
            if isinstance(exclude_vars, dict):
                if k in exclude_vars:
                    if not isinstance(exclude_vars[k], str):
                        raise ValueError(
                            f"exclude_vars[{k}] = {exclude_vars[k]} should be a regex string but got {type(exclude_vars[k])}."
                        )
                    exclude_by_key[k] = exclude_vars[k]
            else:
                exclude_by_key[k] = exclude_vars  # same regex for every DXO of a collection
        if self._single_dxo_key in self.expected_data_kind:
            exclude_by_key[self._single_dxo_key] = exclude_vars
        self.exclude_vars = exclude_by_key

        if _is_nested_aggregation_weights(aggregation_weights):
            missing = _get_missing_keys(expected_data_kind, aggregation_weights)
            if missing:
                raise ValueError(
                    "A dict of dict aggregation_weights should specify aggregation_weights "
                    f"for every key in expected_data_kind. But missed these keys: {missing}"
                )
        aggregation_weights = aggregation_weights or {}
        self.aggregation_weights = {
            k: aggregation_weights[k] if k in aggregation_weights else aggregation_weights for k in self.expected_data_kind
        }

        self.dxo_aggregators = {
            k: DXOAggregator(
                exclude_vars=self.exclude_vars[k],
                aggregation_weights=self.aggregation_weights[k],
                expected_data_kind=self.expected_data_kind[k],
                name_postfix=k,
                weigh_by_local_iter=self._weigh_by_local_iter,
                device=self._device,
                defer_result=self._defer_result,
                devices=self._devices,
            )
            for k in self.expected_data_kind
        }

    def accept(self, shareable: Shareable, fl_ctx: FLContext) -> bool:
        """Stage one client's result; False on any rejection (intime_accumulate_model_aggregator.py:174-230)."""
        try:
            dxo = from_shareable(shareable)
        except Exception:
            self.log_exception(fl_ctx, "shareable data is not a valid DXO")
            return False

        if dxo.data_kind not in (DataKind.WEIGHT_DIFF, DataKind.WEIGHTS, DataKind.METRICS, DataKind.COLLECTION):
            self.log_error(
                fl_ctx,
                f"cannot handle data kind {dxo.data_kind}, "
                f"expecting DataKind.WEIGHT_DIFF, DataKind.WEIGHTS, or DataKind.COLLECTION.",
            )
            return False

        contributor_name = shareable.get_peer_prop(key=ReservedKey.IDENTITY_NAME, default="?")
        contribution_round = shareable.get_cookie(AppConstants.CONTRIBUTION_ROUND)

        rc = shareable.get_return_code()
        if rc and rc != ReturnCode.OK:
            self.log_warning(fl_ctx, f"Contributor {contributor_name} returned rc: {rc}. Disregarding contribution.")
            return False

        n_accepted = 0
        for key in self.expected_data_kind:
            sub_dxo = dxo if key == self._single_dxo_key else dxo.data.get(key)
            if not isinstance(sub_dxo, DXO):
                self.log_warning(fl_ctx, f"Collection does not contain DXO for key {key} but {type(sub_dxo)}.")
                continue
            if not self.dxo_aggregators[key].accept(
                dxo=sub_dxo, contributor_name=contributor_name, contribution_round=contribution_round, fl_ctx=fl_ctx
            ):
                return False
            n_accepted += 1

        if n_accepted > 0:
            return True
        self.log_warning(fl_ctx, f"Did not accept any DXOs from {contributor_name} in round {contribution_round}!")
        return False

    def aggregate(self, fl_ctx: FLContext) -> Shareable:
        """Weighted mean of the accepted results (intime_accumulate_model_aggregator.py:232-255)."""
        results = {}
        for key in self.expected_data_kind:
            aggregated_dxo = self.dxo_aggregators[key].aggregate(fl_ctx)
            if key == self._single_dxo_key:
                self._publish_aggregation_stats(fl_ctx)
                return aggregated_dxo.to_shareable()
            self.log_info(fl_ctx, f"Aggregated contributions matching key '{key}'.")
            results[key] = aggregated_dxo
        self._publish_aggregation_stats(fl_ctx)
        return DXO(data_kind=DataKind.COLLECTION, data=results).to_shareable()

    # reset(): inherited no-op, as in the reference (abstract/aggregator.py:23-32); get_result() already
    # resets each helper, and a late accept between aggregate() and reset() carries over exactly as there.

    def _publish_aggregation_stats(self, fl_ctx: FLContext):
        """Merge per-DXO stats and post them (intime_accumulate_model_aggregator.py:257-288)."""
        combined = None
        for agg in self.dxo_aggregators.values():
            stats = agg.last_aggregation_stats
            if not stats:
                continue
            if combined is None:
                combined = dict(stats)
                continue
            for key in _SUMMED_STATS:
                combined[key] += stats[key]
            contributors = set(combined[AggregationStatsKey.CONTRIBUTORS]) | set(stats[AggregationStatsKey.CONTRIBUTORS])
            combined[AggregationStatsKey.CONTRIBUTORS] = sorted(contributors)
            combined[AggregationStatsKey.ACCEPTED_CONTRIBUTIONS] = len(contributors)
        if combined:
            fl_ctx.set_prop(AppConstants.AGGREGATION_STATS, combined, private=True, sticky=False)
