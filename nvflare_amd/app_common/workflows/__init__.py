"""FedAvg-workflow aggregation entry points on the MI355X."""

from .base_fedavg import aggregate_fn, get_client_name, get_num_steps_weight, make_aggregate_fn  # noqa: F401
from .scaffold import make_scaffold_aggregate_fn, scaffold_aggregate_fn  # noqa: F401
