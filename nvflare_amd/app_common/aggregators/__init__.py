from .accumulate_model_aggregator import AccumulateWeightedAggregator
from .dxo_aggregator import DXOAggregator
from .fedavg_model_aggregator import DeviceFedAvgModelAggregator
from .intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator
from .weighted_aggregation_helper import AggregationStatsKey, WeightedAggregationHelper

__all__ = [
    "AccumulateWeightedAggregator",
    "AggregationStatsKey",
    "DXOAggregator",
    "DeviceFedAvgModelAggregator",
    "InTimeAccumulateWeightedAggregator",
    "WeightedAggregationHelper",
]
