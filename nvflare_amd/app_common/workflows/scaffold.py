"""SCAFFOLD aggregation on the MI355X: the second FedAvg-workflow caller of the hot path.

Reference: ``scaffold_aggregate_fn`` (nvflare/app_common/workflows/scaffold.py:149-189) averages the clients'
params and their control-variate differences (``FLModel.meta[AlgorithmConstants.SCAFFOLD_CTRL_DIFF]``) with
two ``WeightedAggregationHelper`` instances and the FedAvg weight rule (``_get_num_steps_weight``,
base_fedavg.py:93-104).  Both sums use the same per-client weight and the helper keeps a weight sum per key,
so here they share ONE drop-in helper: the control keys are staged under a reserved prefix beside the params,
the engine sums params and controls in the same launches (one slab, one D2H), and the result is split back.
Per-key arithmetic, key order and values are those of the reference's two helpers.

``Scaffold`` is the reference controller (scaffold.py:54-146) with ``aggregate`` routed to this function when
``nvflare``'s workflow runtime is importable; the control-variate update stays the reference's host code.

Use::

    from nvflare_amd.app_common.workflows.scaffold import make_scaffold_aggregate_fn
    model = controller.aggregate(results, aggregate_fn=make_scaffold_aggregate_fn(device=0))
"""

from __future__ import annotations

from typing import Callable, List, Optional

from ...compat import HAVE_NVFLARE, AlgorithmConstants, AppConstants, FLModel
from ..aggregators.weighted_aggregation_helper import WeightedAggregationHelper
from ..fedavg_rules import get_client_name, get_num_steps_weight, make_fedavg_metrics_aggregation_info
from .base_fedavg import aggregate_fl_model_metrics, make_aggregate_fn

# control-variate keys ride in the params helper under this prefix (NUL bytes: never a parameter name)
CTRL_PREFIX = "\x00scaffold_ctrl\x00"


def scaffold_aggregate_fn(results: List[FLModel], device: Optional[int] = None, devices: Optional[list] = None,
                          max_resident_bytes: Optional[int] = None) -> FLModel:
    """``scaffold_aggregate_fn`` (scaffold.py:149-189) with params and control differences summed together
    on the GPU.  Raises the reference's ValueError for a client without ``SCAFFOLD_CTRL_DIFF``."""
    helper = WeightedAggregationHelper(device=device, devices=devices, max_resident_bytes=max_resident_bytes)
    ctrl_key = AlgorithmConstants.SCAFFOLD_CTRL_DIFF
    for r in results:
        weight = get_num_steps_weight(r)
        name = get_client_name(r)
        staged = {k: v for k, v in r.params.items()}  # the reference adds the params first (scaffold.py:157)
        if ctrl_key not in r.meta:
            raise ValueError(
                f"Client '{name}' did not return required "
                f"FLModel.meta['{ctrl_key}'] for Scaffold aggregation."
            )
        for k, v in r.meta[ctrl_key].items():
            staged[CTRL_PREFIX + k] = v
        helper.add(data=staged, weight=weight, contributor_name=name, contribution_round=r.current_round)

    params, ctrl = {}, {}
    n = len(CTRL_PREFIX)
    for k, v in helper.get_result().items():
        if k.startswith(CTRL_PREFIX):
            ctrl[k[n:]] = v
        else:
            params[k] = v

    return FLModel(
        params=params,
        params_type=results[0].params_type,
        metrics=aggregate_fl_model_metrics(results),
        meta={
            ctrl_key: ctrl,
            "nr_aggregated": len(results),
            "current_round": results[0].current_round,
            AppConstants.METRICS_AGGREGATION_INFO: make_fedavg_metrics_aggregation_info(),
        },
    )


def make_scaffold_aggregate_fn(device: Optional[int] = None, devices: Optional[list] = None,
                               max_resident_bytes: Optional[int] = None) -> Callable[[List[FLModel]], FLModel]:
    """Bind the device arguments, giving the ``aggregate_fn(results)`` that ``BaseFedAvg.aggregate``
    (base_fedavg.py:232-262) accepts."""

    def _fn(results: List[FLModel]) -> FLModel:
        return scaffold_aggregate_fn(results, device=device, devices=devices, max_resident_bytes=max_resident_bytes)

    return _fn


_ReferenceScaffold = None
_reference_scaffold_fn = None
_ReferenceBaseFedAvg = None
if HAVE_NVFLARE:
    try:
        from nvflare.app_common.workflows.scaffold import Scaffold as _ReferenceScaffold
        from nvflare.app_common.workflows.scaffold import scaffold_aggregate_fn as _reference_scaffold_fn
    except Exception:  # the workflow package needs more of nvflare than the API types
        _ReferenceScaffold = None
    try:
        from nvflare.app_common.workflows.base_fedavg import BaseFedAvg as _ReferenceBaseFedAvg
    except Exception:
        _ReferenceBaseFedAvg = None

if _ReferenceScaffold is not None:

    class Scaffold(_ReferenceScaffold):
        """``nvflare.app_common.workflows.scaffold.Scaffold`` with its aggregation on the MI355X.

        Same arguments plus ``aggregation_device`` / ``aggregation_devices`` / ``max_resident_bytes`` (the
        drop-in helper's ``device`` / ``devices`` / ``max_resident_bytes``)."""

        def __init__(self, *args, aggregation_device: Optional[int] = None, aggregation_devices: Optional[list] = None,
                     max_resident_bytes: Optional[int] = None, **kwargs):
            super().__init__(*args, **kwargs)
            dev = dict(device=aggregation_device, devices=aggregation_devices, max_resident_bytes=max_resident_bytes)
            self._device_scaffold_fn = make_scaffold_aggregate_fn(**dev)
            self._device_fedavg_fn = make_aggregate_fn(**dev)

        def aggregate(self, results: List[FLModel], aggregate_fn=None) -> FLModel:
            """BaseFedAvg.aggregate (base_fedavg.py:232-262) with the reference's two aggregation functions
            (``scaffold_aggregate_fn``, and ``BaseFedAvg.aggregate_fn`` when none is given) on the device;
            any other caller-supplied function runs as given."""
            if aggregate_fn is _reference_scaffold_fn:
                aggregate_fn = self._device_scaffold_fn
            elif not aggregate_fn:
                # the reference falls back to self.aggregate_fn (base_fedavg.py:251-252): an instance attribute
                # (self.aggregate_fn = fn, set in __init__ or by the caller) or a subclass's own override runs as
                # given; only the reference's BaseFedAvg.aggregate_fn moves to the device
                if "aggregate_fn" in self.__dict__:
                    aggregate_fn = self.__dict__["aggregate_fn"]
                else:
                    own = getattr(type(self), "aggregate_fn", None)
                    ref = getattr(_ReferenceBaseFedAvg, "aggregate_fn", None) if _ReferenceBaseFedAvg is not None else None
                    aggregate_fn = self._device_fedavg_fn if own is ref else self.aggregate_fn
            return super().aggregate(results, aggregate_fn=aggregate_fn)

else:

    class Scaffold:  # pragma: no cover - needs the NVFlare workflow runtime
        def __init__(self, *args, **kwargs):
            raise ImportError("nvflare_amd Scaffold controller: the workflow needs the nvflare package; "
                              "scaffold_aggregate_fn holds the device aggregation on its own")
