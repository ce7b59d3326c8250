"""GPU drop-in for ``nvflare.app_common.aggregators.dxo_aggregator.DXOAggregator``.

Per-DXO validation and weight derivation exactly as the reference (dxo_aggregator.py:71-163); the
weighted accumulation is delegated to the HIP-backed ``WeightedAggregationHelper`` of this package.
"""

from __future__ import annotations

from typing import Any, Dict, Optional

from ...compat import DXO, AppConstants, DataKind, FLComponent, FLContext, MetaKey, get_module_logger
from .weighted_aggregation_helper import AggregationStatsKey, WeightedAggregationHelper

_AGGREGATABLE_KINDS = (DataKind.WEIGHT_DIFF, DataKind.WEIGHTS, DataKind.METRICS)


class DXOAggregator(FLComponent):
    def __init__(
        self,
        exclude_vars: Optional[str] = None,
        aggregation_weights: Optional[Dict[str, Any]] = None,
        expected_data_kind: DataKind = DataKind.WEIGHT_DIFF,
        name_postfix: str = "",
        weigh_by_local_iter: bool = True,
        device: Optional[int] = None,
        defer_result: bool = False,
    ):
        """Accumulated weighted aggregation of one kind of DXO (dxo_aggregator.py:26-66).

        Args: as the reference, plus ``device`` (HIP device index of the aggregation engine) and
        ``defer_result`` (fp32 results stay in HBM as ``DeferredAggregate`` values, nvflare_amd/deferred.py).
        """
        super().__init__()
        self.expected_data_kind = expected_data_kind
        self.aggregation_weights = aggregation_weights or {}
        self.aggregation_helper = WeightedAggregationHelper(
            exclude_vars=exclude_vars, weigh_by_local_iter=weigh_by_local_iter, device=device,
            defer_result=defer_result,
        )
        self.warning_count = {}
        self.warning_limit = 10
        self.processed_algorithm = None
        self.last_aggregation_stats = None
        if name_postfix:
            self._name += name_postfix
            self.logger = get_module_logger(self.__module__, f"{self.__class__.__qualname__}{name_postfix}")

    def reset_aggregation_helper(self):
        if self.aggregation_helper:
            self.aggregation_helper.reset_stats()

    def _warn_limited(self, fl_ctx, contributor_name, msg):
        # at most warning_limit+1 warnings per contributor (dxo_aggregator.py:133-156)
        if self.warning_count.get(contributor_name, 0) <= self.warning_limit:
            self.log_warning(fl_ctx, msg)
            self.warning_count[contributor_name] = (
                self.warning_count[contributor_name] + 1 if contributor_name in self.warning_count else 0
            )

    def accept(self, dxo: DXO, contributor_name, contribution_round, fl_ctx: FLContext) -> bool:
        """Validate one contribution and stage it on the device; False (never raise) on rejection."""
        if not isinstance(dxo, DXO):
            self.log_error(fl_ctx, f"Expected DXO but got {type(dxo)}")
            return False
        if dxo.data_kind not in _AGGREGATABLE_KINDS:
            self.log_error(fl_ctx, "cannot handle data kind {}".format(dxo.data_kind))
            return False
        if dxo.data_kind != self.expected_data_kind:
            self.log_error(fl_ctx, "expected {} but got {}".format(self.expected_data_kind, dxo.data_kind))
            return False

        algo = dxo.get_meta_prop(MetaKey.PROCESSED_ALGORITHM)
        if algo is not None:
            if self.processed_algorithm is None:
                self.processed_algorithm = algo
            elif self.processed_algorithm != algo:
                self.log_error(
                    fl_ctx,
                    f"Only supports aggregation of data processed with the same algorithm ({self.processed_algorithm}) "
                    f"but got algorithm: {algo}",
                )
                return False

        current_round = fl_ctx.get_prop(AppConstants.CURRENT_ROUND)
        if contribution_round != current_round:
            self.log_warning(
                fl_ctx,
                f"discarding DXO from {contributor_name} at round: {contribution_round}. Current round is: {current_round}",
            )
            return False

        data = dxo.data
        if data is None:
            self.log_error(fl_ctx, "no data to aggregate")
            return False

        for item in self.aggregation_helper.get_history():
            if contributor_name == item["contributor_name"]:
                self.log_warning(
                    fl_ctx,
                    f"discarding DXO from {contributor_name} at round: {contribution_round} as {item['round']} accepted already",
                )
                return False

        n_iter = dxo.get_meta_prop(MetaKey.NUM_STEPS_CURRENT_ROUND)
        if n_iter is None:
            self._warn_limited(
                fl_ctx,
                contributor_name,
                f"NUM_STEPS_CURRENT_ROUND missing in meta of DXO from {contributor_name} and set to default value, 1.0. "
                f" This kind of message will show {self.warning_limit} times at most.",
            )
            n_iter = 1.0
        float_n_iter = float(n_iter)
        aggregation_weight = self.aggregation_weights.get(contributor_name)
        if aggregation_weight is None:
            self._warn_limited(
                fl_ctx,
                contributor_name,
                f"Aggregation_weight missing for {contributor_name} and set to default value, 1.0"
                f" This kind of message will show {self.warning_limit} times at most.",
            )
            aggregation_weight = 1.0

        # the weight is the reference's fp64 product (dxo_aggregator.py:161)
        self.aggregation_helper.add(data, aggregation_weight * float_n_iter, contributor_name, contribution_round)
        return True

    def aggregate(self, fl_ctx: FLContext) -> DXO:
        """Weighted mean of the accepted DXOs (dxo_aggregator.py:165-191)."""
        current_round = fl_ctx.get_prop(AppConstants.CURRENT_ROUND)
        self.log_info(fl_ctx, f"aggregating {self.aggregation_helper.get_len()} update(s) at round {current_round}")
        aggregated = self.aggregation_helper.get_result()
        # stats snapshotted atomically with the reset inside get_result (late accepts cannot slip in)
        stats = dict(self.aggregation_helper.last_aggregation_stats or {})
        stats[AggregationStatsKey.ROUND] = current_round
        self.last_aggregation_stats = stats
        dxo = DXO(data_kind=self.expected_data_kind, data=aggregated)
        if self.processed_algorithm is not None:
            dxo.set_meta_prop(MetaKey.PROCESSED_ALGORITHM, self.processed_algorithm)
            self.processed_algorithm = None
        return dxo
