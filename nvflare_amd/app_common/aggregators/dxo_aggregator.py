"""GPU drop-in for ``nvflare.app_common.aggregators.dxo_aggregator.DXOAggregator``.

Contract (dxo_aggregator.py:71-191): a contribution is rejected -- logged, ``False`` returned, nothing
staged -- when it is not a DXO, has a kind other than WEIGHT_DIFF / WEIGHTS / METRICS or the expected one,
was processed by a different algorithm than earlier contributions, belongs to another round, carries no
data, or comes from a contributor already accepted this round.  Otherwise its weight is
``aggregation_weight (default 1.0) * float(NUM_STEPS_CURRENT_ROUND (default 1.0))`` in fp64, and the data
go to the HIP-backed ``WeightedAggregationHelper`` of this package (staged in HBM at once).  The log
messages and the per-contributor warning limit are the reference's, so job logs read the same.
"""

from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

from ...compat import DXO, AppConstants, DataKind, FLComponent, FLContext, MetaKey, get_module_logger
from .weighted_aggregation_helper import AggregationStatsKey, WeightedAggregationHelper

_AGGREGATABLE_KINDS = (DataKind.WEIGHT_DIFF, DataKind.WEIGHTS, DataKind.METRICS)
_ERROR, _WARNING = "error", "warning"


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
        devices: Optional[list] = None,
    ):
        """Accumulated weighted aggregation of one kind of DXO (dxo_aggregator.py:26-66).

        Args: as the reference, plus ``device`` (HIP device index of the aggregation engine),
        ``defer_result`` (fp32 results stay in HBM as ``DeferredAggregate`` values, nvflare_amd/deferred.py)
        and ``devices`` (parameter buckets over several HIP devices, nvflare_amd/sharding.py).
        """
        super().__init__()
        self.expected_data_kind = expected_data_kind
        self.aggregation_weights = aggregation_weights or {}
        self.aggregation_helper = WeightedAggregationHelper(
            exclude_vars=exclude_vars, weigh_by_local_iter=weigh_by_local_iter, device=device,
            defer_result=defer_result, devices=devices,
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

    # ------------------------------------------------------------------ validation
    def _rejection(self, dxo, contributor_name, contribution_round, fl_ctx) -> Optional[Tuple[str, str]]:
        """(level, message) of the first failed check, in the reference's order; None if acceptable.
        Records the contribution's PROCESSED_ALGORITHM when it is the first one seen."""
        if not isinstance(dxo, DXO):
            return _ERROR, f"Expected DXO but got {type(dxo)}"
        kind = dxo.data_kind
        if kind not in _AGGREGATABLE_KINDS:
            return _ERROR, "cannot handle data kind {}".format(kind)
        if kind != self.expected_data_kind:
            return _ERROR, "expected {} but got {}".format(self.expected_data_kind, kind)
        algo = dxo.get_meta_prop(MetaKey.PROCESSED_ALGORITHM)
        if algo is not None:
            if self.processed_algorithm is None:
                self.processed_algorithm = algo
            elif algo != self.processed_algorithm:
                return _ERROR, (f"Only supports aggregation of data processed with the same algorithm "
                                f"({self.processed_algorithm}) but got algorithm: {algo}")
        current_round = fl_ctx.get_prop(AppConstants.CURRENT_ROUND)
        if contribution_round != current_round:
            return _WARNING, (f"discarding DXO from {contributor_name} at round: {contribution_round}. "
                              f"Current round is: {current_round}")
        if dxo.data is None:
            return _ERROR, "no data to aggregate"
        earlier = [h for h in self.aggregation_helper.get_history() if h["contributor_name"] == contributor_name]
        if earlier:
            return _WARNING, (f"discarding DXO from {contributor_name} at round: {contribution_round} as "
                              f"{earlier[0]['round']} accepted already")
        return None

    def _limited_warning(self, fl_ctx, contributor_name, msg) -> None:
        """At most warning_limit + 1 defaulting warnings per contributor (dxo_aggregator.py:133-156)."""
        seen = self.warning_count.get(contributor_name)
        if (seen or 0) > self.warning_limit:
            return
        self.log_warning(fl_ctx, msg)
        self.warning_count[contributor_name] = 0 if seen is None else seen + 1

    def _contribution_weight(self, dxo, contributor_name, fl_ctx) -> float:
        """aggregation_weight * NUM_STEPS_CURRENT_ROUND, both defaulting to 1.0, as a python (fp64) float."""
        limit = self.warning_limit
        n_iter = dxo.get_meta_prop(MetaKey.NUM_STEPS_CURRENT_ROUND)
        if n_iter is None:
            self._limited_warning(
                fl_ctx, contributor_name,
                f"NUM_STEPS_CURRENT_ROUND missing in meta of DXO from {contributor_name} and set to default value, "
                f"1.0.  This kind of message will show {limit} times at most.")
            n_iter = 1.0
        steps = float(n_iter)
        aggregation_weight = self.aggregation_weights.get(contributor_name)
        if aggregation_weight is None:
            self._limited_warning(
                fl_ctx, contributor_name,
                f"Aggregation_weight missing for {contributor_name} and set to default value, 1.0 "
                f"This kind of message will show {limit} times at most.")
            aggregation_weight = 1.0
        return aggregation_weight * steps

    # ------------------------------------------------------------------ Aggregator surface
    def accept(self, dxo: DXO, contributor_name, contribution_round, fl_ctx: FLContext) -> bool:
        """Validate one contribution and stage it on the device; False (never raise) on rejection."""
        rejected = self._rejection(dxo, contributor_name, contribution_round, fl_ctx)
        if rejected is not None:
            level, msg = rejected
            (self.log_error if level == _ERROR else self.log_warning)(fl_ctx, msg)
            return False
        weight = self._contribution_weight(dxo, contributor_name, fl_ctx)
        self.aggregation_helper.add(dxo.data, weight, contributor_name, contribution_round)
        return True

    def aggregate(self, fl_ctx: FLContext) -> DXO:
        """Weighted mean of the accepted DXOs (dxo_aggregator.py:165-191)."""
        rnd = fl_ctx.get_prop(AppConstants.CURRENT_ROUND)
        self.log_info(fl_ctx, f"aggregating {self.aggregation_helper.get_len()} update(s) at round {rnd}")
        result = self.aggregation_helper.get_result()
        # the stats snapshot is taken with the reset inside get_result, so a late accept cannot slip in
        self.last_aggregation_stats = {**(self.aggregation_helper.last_aggregation_stats or {}),
                                       AggregationStatsKey.ROUND: rnd}
        out = DXO(data_kind=self.expected_data_kind, data=result)
        if self.processed_algorithm is not None:
            out.set_meta_prop(MetaKey.PROCESSED_ALGORITHM, self.processed_algorithm)
            self.processed_algorithm = None
        return out
