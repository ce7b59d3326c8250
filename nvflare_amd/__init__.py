"""nvflare_amd -- MI355X-native (gfx950) FedAvg weighted aggregation behind NVFlare's Aggregator API.

Drop-in classes (same constructor kwargs and behaviour as the NVFlare originals):
  nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator.InTimeAccumulateWeightedAggregator
  nvflare_amd.app_common.aggregators.dxo_aggregator.DXOAggregator
  nvflare_amd.app_common.aggregators.weighted_aggregation_helper.WeightedAggregationHelper

The arithmetic runs in hand-written HIP kernels (nvflare_amd/csrc) behind a C-ABI
(include/nvflare_amd_fedavg.h) loaded with ctypes; there is no CPU fallback.
"""

__version__ = "0.1.0"
