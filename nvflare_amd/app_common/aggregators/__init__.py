from .dxo_aggregator import DXOAggregator
from .fedavg_model_aggregator import DeviceFedAvgModelAggregator
from .intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator
from .weighted_aggregation_helper import AggregationStatsKey, WeightedAggregationHelper

AccumulateWeightedAggregator = InTimeAccumulateWeightedAggregator  # deprecated alias (accumulate_model_aggregator.py:20-22)

__all__ = [
    "AccumulateWeightedAggregator",
    "AggregationStatsKey",
    "DXOAggregator",
    "DeviceFedAvgModelAggregator",
    "InTimeAccumulateWeightedAggregator",
    "WeightedAggregationHelper",
]
