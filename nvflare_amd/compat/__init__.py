"""NVFlare API types for the drop-in: the real ``nvflare`` classes when importable, so the GPU
aggregator plugs into a live NVFlare server unchanged; otherwise the minimal stand-ins in
``_standins.py``.  ``NVFLARE_AMD_FORCE_STANDINS=1`` forces the stand-ins."""

from __future__ import annotations

import os

HAVE_NVFLARE = False
if os.environ.get("NVFLARE_AMD_FORCE_STANDINS", "0") != "1":
    try:
        from nvflare.apis.dxo import DXO, DataKind, MetaKey, from_shareable  # noqa: F401
        from nvflare.apis.event_type import EventType  # noqa: F401
        from nvflare.apis.fl_component import FLComponent  # noqa: F401
        from nvflare.apis.fl_constant import ReservedKey, ReturnCode  # noqa: F401
        from nvflare.apis.fl_context import FLContext  # noqa: F401
        from nvflare.apis.shareable import Shareable  # noqa: F401
        from nvflare.app_common.abstract.aggregator import Aggregator  # noqa: F401
        from nvflare.app_common.app_constant import AlgorithmConstants, AppConstants  # noqa: F401
        from nvflare.fuel.utils.log_utils import get_module_logger  # noqa: F401
        from nvflare.apis.fl_constant import FLMetaKey  # noqa: F401
        from nvflare.app_common.abstract.fl_model import FLModel, ParamsType  # noqa: F401
        from nvflare.app_common.aggregators.model_aggregator import ModelAggregator  # noqa: F401
        from nvflare.app_common.utils.fl_model_utils import FLModelUtils  # noqa: F401
        from nvflare.app_common.abstract.learnable import Learnable  # noqa: F401
        from nvflare.app_common.abstract.model import (  # noqa: F401
            ModelLearnable,
            ModelLearnableKey,
            make_model_learnable,
            model_learnable_to_dxo,
        )
        from nvflare.app_common.abstract.shareable_generator import ShareableGenerator  # noqa: F401
        from nvflare.apis.dxo_filter import DXOFilter  # noqa: F401

        HAVE_NVFLARE = True
    except Exception:
        HAVE_NVFLARE = False

if not HAVE_NVFLARE:
    from ._standins import (  # noqa: F401
        DXO,
        Aggregator,
        AlgorithmConstants,
        DXOFilter,
        AppConstants,
        DataKind,
        EventType,
        FLComponent,
        FLContext,
        FLMetaKey,
        FLModel,
        FLModelUtils,
        Learnable,
        ModelAggregator,
        ModelLearnable,
        ModelLearnableKey,
        ParamsType,
        MetaKey,
        ReservedKey,
        ReturnCode,
        Shareable,
        ShareableGenerator,
        from_shareable,
        get_module_logger,
        make_model_learnable,
        model_learnable_to_dxo,
    )

__all__ = [
    "HAVE_NVFLARE",
    "DXO",
    "DXOFilter",
    "Aggregator",
    "AlgorithmConstants",
    "AppConstants",
    "DataKind",
    "EventType",
    "FLComponent",
    "FLContext",
    "FLMetaKey",
    "FLModel",
    "FLModelUtils",
    "Learnable",
    "ModelAggregator",
    "ModelLearnable",
    "ModelLearnableKey",
    "ParamsType",
    "MetaKey",
    "ReservedKey",
    "ReturnCode",
    "Shareable",
    "ShareableGenerator",
    "from_shareable",
    "get_module_logger",
    "make_model_learnable",
    "model_learnable_to_dxo",
]
