"""Drop-in for the deprecated ``nvflare.app_common.aggregators.accumulate_model_aggregator`` path
(accumulate_model_aggregator.py:20-22): the same class as ``InTimeAccumulateWeightedAggregator``, so old job
configs that name this module switch by changing the package prefix only."""

import warnings

from .intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator


class AccumulateWeightedAggregator(InTimeAccumulateWeightedAggregator):
    def __init__(self, *args, **kwargs):
        warnings.warn("AccumulateWeightedAggregator is deprecated. Please use 'InTimeAccumulateWeightedAggregator'",
                      DeprecationWarning, stacklevel=2)
        super().__init__(*args, **kwargs)
