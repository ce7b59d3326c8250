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


def _kind_error(label: str, kind) -> ValueError:
    allowed = " or ".join(f"{k}" for k in _KINDS)
    return ValueError(f"{label} = {kind} is not {allowed}")


def _absent(required, given: dict) -> list:
    """Keys of ``required`` that ``given`` lacks, in ``required``'s order."""
    return [name for name in required if name not in given]


def _kinds_by_dxo(expected_data_kind, single_key: str) -> dict:
    """{dxo name: DataKind}; one bare DataKind means the single unnamed DXO (reference :101-113)."""
    table = expected_data_kind if isinstance(expected_data_kind, dict) else {single_key: expected_data_kind}
    for name, kind in table.items():
        if kind not in _KINDS:
            raise _kind_error(f"expected_data_kind[{name}]" if table is expected_data_kind else "expected_data_kind", kind)
    return table


def _excludes_by_dxo(exclude_vars, raw_kinds, kinds: dict, single_key: str) -> dict:
    """{dxo name: regex or None} (reference :114-141): a dict must name every DXO, a string applies to all."""
    per_dxo = isinstance(exclude_vars, dict)
    if exclude_vars and not (per_dxo or isinstance(exclude_vars, str)):
        raise ValueError(f"exclude_vars = {exclude_vars} should be a regex string but got {type(exclude_vars)}.")
    if exclude_vars and per_dxo:
        gaps = _absent(raw_kinds, exclude_vars)
        if gaps:
            raise ValueError(
                "A dict exclude_vars should specify exclude_vars for every key in expected_data_kind. "
                f"But missed these keys: {gaps}"
            )
    table = {}
    for name in kinds:
        if not per_dxo:
            table[name] = exclude_vars
        elif name in exclude_vars:
            regex = exclude_vars[name]
            if not isinstance(regex, str):
                raise ValueError(f"exclude_vars[{name}] = {regex} should be a regex string but got {type(regex)}.")
            table[name] = regex
    if single_key in kinds:
        table[single_key] = exclude_vars
    return table


def _weights_by_dxo(aggregation_weights, raw_kinds, kinds: dict) -> dict:
    """{dxo name: {contributor: weight}} (reference :142-158); a dict of dicts must name every DXO."""
    nested = bool(aggregation_weights) and isinstance(aggregation_weights, dict) and isinstance(
        next(iter(aggregation_weights.values())), dict
    )
    if nested:
        gaps = _absent(raw_kinds, aggregation_weights)
        if gaps:
            raise ValueError(
                "A dict of dict aggregation_weights should specify aggregation_weights "
                f"for every key in expected_data_kind. But missed these keys: {gaps}"
            )
    shared = aggregation_weights or {}
    return {name: shared[name] if name in shared else shared for name in kinds}


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
        # validation order and messages as intime_accumulate_model_aggregator.py:99-172
        kinds = _kinds_by_dxo(expected_data_kind, self._single_dxo_key)
        self.expected_data_kind = kinds
        self.exclude_vars = _excludes_by_dxo(exclude_vars, expected_data_kind, kinds, self._single_dxo_key)
        self.aggregation_weights = _weights_by_dxo(aggregation_weights, expected_data_kind, kinds)
        engine_kwargs = dict(device=self._device, defer_result=self._defer_result, devices=self._devices,
                             weigh_by_local_iter=self._weigh_by_local_iter)
        self.dxo_aggregators = {}
        for name, kind in kinds.items():
            self.dxo_aggregators[name] = DXOAggregator(
                exclude_vars=self.exclude_vars[name], aggregation_weights=self.aggregation_weights[name],
                expected_data_kind=kind, name_postfix=name, **engine_kwargs)

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

        taken = 0
        for name, agg in self.dxo_aggregators.items():
            part = dxo if name == self._single_dxo_key else dxo.data.get(name)
            if not isinstance(part, DXO):
                self.log_warning(fl_ctx, f"Collection does not contain DXO for key {name} but {type(part)}.")
                continue
            ok = agg.accept(dxo=part, contributor_name=contributor_name, contribution_round=contribution_round,
                            fl_ctx=fl_ctx)
            if not ok:
                return False  # one rejected DXO rejects the whole contribution
            taken += 1
        if not taken:
            self.log_warning(fl_ctx, f"Did not accept any DXOs from {contributor_name} in round {contribution_round}!")
        return taken > 0

    def aggregate(self, fl_ctx: FLContext) -> Shareable:
        """Weighted mean of the accepted results (intime_accumulate_model_aggregator.py:232-255)."""
        parts = {}
        for name, agg in self.dxo_aggregators.items():
            out = agg.aggregate(fl_ctx)
            if name == self._single_dxo_key:  # the unnamed DXO is returned as it is, stats published first
                self._publish_aggregation_stats(fl_ctx)
                return out.to_shareable()
            self.log_info(fl_ctx, f"Aggregated contributions matching key '{name}'.")
            parts[name] = out
        self._publish_aggregation_stats(fl_ctx)
        return DXO(data_kind=DataKind.COLLECTION, data=parts).to_shareable()

    # reset(): inherited no-op, as in the reference (abstract/aggregator.py:23-32); get_result() already
    # resets each helper, and a late accept between aggregate() and reset() carries over exactly as there.

    def _publish_aggregation_stats(self, fl_ctx: FLContext):
        """Merge per-DXO stats and post them (intime_accumulate_model_aggregator.py:257-288)."""
        merged: Optional[dict] = None
        for stats in (agg.last_aggregation_stats for agg in self.dxo_aggregators.values()):
            if not stats:
                continue
            if merged is None:
                merged = dict(stats)
                continue
            merged.update({key: merged[key] + stats[key] for key in _SUMMED_STATS})
            everyone = sorted(set(merged[AggregationStatsKey.CONTRIBUTORS]).union(stats[AggregationStatsKey.CONTRIBUTORS]))
            merged[AggregationStatsKey.CONTRIBUTORS] = everyone
            merged[AggregationStatsKey.ACCEPTED_CONTRIBUTIONS] = len(everyone)
        if merged:
            fl_ctx.set_prop(AppConstants.AGGREGATION_STATS, merged, private=True, sticky=False)
