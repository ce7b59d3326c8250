"""Minimal stand-ins for the NVFlare API types the aggregator touches.

Used only when the real ``nvflare`` package is not importable (e.g. on a bare GPU box or in this
repository's tests).  They reproduce the behaviour the aggregation path relies on -- nothing more:

* ``DXO`` / ``from_shareable`` / ``DataKind`` / ``MetaKey``      nvflare/apis/dxo.py:23-177
* ``Shareable`` (headers, cookies, peer props, return code)      nvflare/apis/shareable.py:41-127
* ``FLContext.get_prop/set_prop``                                 nvflare/apis/fl_context.py:134-175
* ``FLComponent`` logging helpers and ``handle_event``            nvflare/apis/fl_component.py:28-231
* ``Aggregator`` ABC                                               nvflare/app_common/abstract/aggregator.py:22-58
* ``FLModel`` / ``ParamsType``                                     nvflare/app_common/abstract/fl_model.py:22-110
* ``ModelAggregator`` ABC and the ``FLModelUtils`` conversions it uses
                                                  nvflare/app_common/aggregators/model_aggregator.py:26-83,
                                                  nvflare/app_common/utils/fl_model_utils.py:46-149
* ``DXOFilter`` (process / process_dxo / filter history)          nvflare/apis/dxo_filter.py:26-140
* ``ShareableGenerator``, ``Learnable``, ``ModelLearnable`` helpers  app_common/abstract/shareable_generator.py,
                                                  learnable.py, model.py:25-71
* constants: ``ReservedKey`` (fl_constant.py:69-80), ``ReturnCode`` (:26-36),
  ``AppConstants`` (app_common/app_constant.py:33-79), ``AlgorithmConstants`` (:156-160),
  ``EventType.START_RUN`` (apis/event_type.py:22)
"""

from __future__ import annotations

import logging
from abc import ABC, abstractmethod
from enum import Enum
from typing import Any, Dict, Optional


class DataKind(str, Enum):
    FL_MODEL = "FL_MODEL"
    WEIGHTS = "WEIGHTS"
    WEIGHT_DIFF = "WEIGHT_DIFF"
    METRICS = "METRICS"
    ANALYTIC = "ANALYTIC"
    COLLECTION = "COLLECTION"
    STATISTICS = "STATISTICS"
    PSI = "PSI"
    APP_DEFINED = "APP_DEFINED"


class MetaKey:
    NUM_STEPS_CURRENT_ROUND = "NUM_STEPS_CURRENT_ROUND"
    PROCESSED_ALGORITHM = "PROCESSED_ALGORITHM"
    INITIAL_METRICS = "initial_metrics"
    FILTER_HISTORY = "filter_history"


class ReservedKey:
    ENGINE = "__engine__"
    IDENTITY_NAME = "__identity_name__"
    RC = "__rc__"
    COOKIE_JAR = "__cookie_jar__"


class ReturnCode:
    OK = "OK"
    BAD_TASK_DATA = "BAD_TASK_DATA"
    EXECUTION_EXCEPTION = "EXECUTION_EXCEPTION"
    EXECUTION_RESULT_ERROR = "EXECUTION_RESULT_ERROR"
    TASK_ABORTED = "TASK_ABORTED"


class ReservedHeaderKey:
    HEADERS = "__headers__"
    RC = ReservedKey.RC
    COOKIE_JAR = ReservedKey.COOKIE_JAR
    PEER_PROPS = "__peer_props__"
    CONTENT_TYPE = "__content_type__"


class FLMetaKey:
    NUM_STEPS_CURRENT_ROUND = "NUM_STEPS_CURRENT_ROUND"
    INITIAL_METRICS = "initial_metrics"


class AppConstants:
    GLOBAL_MODEL = "global_model"
    CURRENT_ROUND = "current_round"
    START_ROUND = "start_round"
    CLIENT_UNKNOWN = "unknown"
    METRICS_AGGREGATION_INFO = "metrics_aggregation_info"
    NUM_ROUNDS = "num_rounds"
    CONTRIBUTION_ROUND = "contribution_round"
    AGGREGATION_STATS = "_aggregation_stats"


class AlgorithmConstants:
    SCAFFOLD_CTRL_DIFF = "scaffold_c_diff"
    SCAFFOLD_CTRL_GLOBAL = "scaffold_c_global"


class EventType:
    START_RUN = "_start_run"
    END_RUN = "_end_run"
    BEFORE_AGGREGATION = "_before_aggregation"
    AFTER_AGGREGATION = "_after_aggregation"


class Shareable(dict):
    """A dict with a header sub-dict (rc, cookies, peer props, content type)."""

    def __init__(self, data: Optional[dict] = None):
        super().__init__()
        if data:
            self.update(data)
        self[ReservedHeaderKey.HEADERS] = {}

    def _headers(self, create: bool):
        h = self.get(ReservedHeaderKey.HEADERS)
        if not h and create:
            h = {}
            self[ReservedHeaderKey.HEADERS] = h
        return h

    def set_header(self, key: str, value):
        self._headers(True)[key] = value

    def get_header(self, key: str, default=None):
        h = self._headers(False)
        if not h:
            return default
        if not isinstance(h, dict):
            raise ValueError(f"header object must be a dict, but got {type(h)}")
        return h.get(key, default)

    def get_return_code(self, default=ReturnCode.OK):
        return self.get_header(ReservedHeaderKey.RC, default)

    def set_return_code(self, rc):
        self.set_header(ReservedHeaderKey.RC, rc)

    def add_cookie(self, name: str, data):
        jar = self.get_cookie_jar()
        if not jar:
            jar = {}
            self.set_header(ReservedHeaderKey.COOKIE_JAR, jar)
        jar[name] = data

    def get_cookie_jar(self):
        return self.get_header(ReservedHeaderKey.COOKIE_JAR, None)

    def set_cookie_jar(self, jar):
        self.set_header(ReservedHeaderKey.COOKIE_JAR, jar)

    def get_cookie(self, name: str, default=None):
        jar = self.get_cookie_jar()
        return jar.get(name, default) if jar else default

    def set_peer_props(self, props: dict):
        self.set_header(ReservedHeaderKey.PEER_PROPS, props)

    def get_peer_props(self):
        return self.get_header(ReservedHeaderKey.PEER_PROPS, None)

    def get_peer_prop(self, key: str, default):
        props = self.get_peer_props()
        return props.get(key, default) if isinstance(props, dict) else default


_DXO_KEY = "DXO"


class DXO:
    def __init__(self, data_kind: str, data: dict, meta: Optional[dict] = None):
        self.data_kind = data_kind
        self.data = {} if data is None else data
        self.meta = {} if meta is None else meta
        if self.data_kind != DataKind.APP_DEFINED and not isinstance(self.data, dict):
            raise ValueError(f"invalid DXO: invalid data: expect dict but got {type(self.data)}")
        if not isinstance(self.meta, dict):
            raise ValueError(f"invalid DXO: invalid props: expect dict but got {type(self.meta)}")

    def get_meta_prop(self, key: str, default=None):
        return self.meta.get(key, default) if isinstance(self.meta, dict) else default

    def set_meta_prop(self, key: str, value):
        if self.meta is None:
            self.meta = {}
        self.meta[key] = value

    def get_meta_props(self):
        return self.meta

    def remove_meta_props(self, keys):
        if self.meta and keys:
            for k in keys:
                self.meta.pop(k, None)

    def add_filter_history(self, filter_name):
        if not filter_name:
            return
        hist = self.get_meta_prop(MetaKey.FILTER_HISTORY)
        if not hist:
            hist = []
            self.set_meta_prop(MetaKey.FILTER_HISTORY, hist)
        if isinstance(filter_name, str):
            hist.append(filter_name)
        else:
            hist.extend(filter_name)

    def get_filter_history(self):
        return self.get_meta_prop(MetaKey.FILTER_HISTORY)

    def to_dict(self) -> dict:
        return {"kind": self.data_kind, "data": self.data, "meta": self.meta}

    def update_shareable(self, s: Shareable) -> Shareable:
        s.set_header(ReservedHeaderKey.CONTENT_TYPE, "DXO")
        s[_DXO_KEY] = self.to_dict()
        return s

    def to_shareable(self) -> Shareable:
        return self.update_shareable(Shareable())


def from_dict(encoded: dict) -> DXO:
    if not isinstance(encoded, dict):
        raise ValueError(f"encoded value must be dict but got {type(encoded)}")
    return DXO(data_kind=encoded.get("kind"), data=encoded.get("data"), meta=encoded.get("meta"))


def from_shareable(s: Shareable) -> DXO:
    ct = s.get_header(ReservedHeaderKey.CONTENT_TYPE)
    if ct != "DXO":
        raise ValueError(f"the shareable is not a valid DXO - expect content_type DXO but got {ct}")
    enc = s.get(_DXO_KEY, None)
    if not enc:
        raise ValueError("the shareable is not a valid DXO - missing content")
    if not isinstance(enc, dict):
        raise ValueError(f"the shareable is not a valid DXO - should be encoded as dict but got {type(enc)}")
    return from_dict(enc)


class FLContext:
    """Property bag; private/sticky flags are recorded but have no effect without an engine."""

    def __init__(self):
        self._props: Dict[str, Dict[str, Any]] = {}

    def set_prop(self, key: str, value, private=True, sticky=True):
        self._props[key] = {"value": value, "private": private, "sticky": sticky}
        return True

    def get_prop(self, key, default=None):
        p = self._props.get(key)
        return default if p is None else p["value"]

    def get_prop_detail(self, key):
        return self._props.get(key)

    def remove_prop(self, key: str, force_removal=False):
        self._props.pop(key, None)

    def get_identity_name(self, default=""):
        return self.get_prop(ReservedKey.IDENTITY_NAME, default)

    def get_engine(self):
        return self.get_prop(ReservedKey.ENGINE)


def get_module_logger(module: str = None, name: str = None):
    return logging.getLogger(f"{module}.{name}" if module and name else (module or name or "nvflare_amd"))


class FLComponent:
    def __init__(self):
        self._name = self.__class__.__name__
        self.logger = get_module_logger(self.__module__, self.__class__.__qualname__)

    @property
    def name(self):
        return self._name

    def handle_event(self, event_type: str, fl_ctx: FLContext):
        pass

    def _log(self, level, msg):
        self.logger.log(level, msg)

    def log_info(self, fl_ctx, msg: str, fire_event=False):
        self._log(logging.INFO, msg)

    def log_warning(self, fl_ctx, msg: str, fire_event=True):
        self._log(logging.WARNING, msg)

    def log_error(self, fl_ctx, msg: str, fire_event=True):
        self._log(logging.ERROR, msg)

    def log_debug(self, fl_ctx, msg: str, fire_event=False):
        self._log(logging.DEBUG, msg)

    def log_critical(self, fl_ctx, msg: str, fire_event=True):
        self._log(logging.CRITICAL, msg)

    def log_exception(self, fl_ctx, msg: str, fire_event=False):
        self.logger.exception(msg)

    def system_panic(self, reason: str, fl_ctx):
        self.log_critical(fl_ctx, f"system panic: {reason}")


class Aggregator(FLComponent, ABC):
    def reset(self, fl_ctx: FLContext):
        pass

    @abstractmethod
    def accept(self, shareable: Shareable, fl_ctx: FLContext) -> bool:
        pass

    @abstractmethod
    def aggregate(self, fl_ctx: FLContext) -> Shareable:
        pass


class ParamsType(str, Enum):
    FULL = "FULL"
    DIFF = "DIFF"


class FLModel:
    """The FLModel fields the FedAvg path reads and writes (fl_model.py:38-110; no validation helpers)."""

    def __init__(self, params_type=None, params=None, optimizer_params=None, metrics=None, start_round=0,
                 current_round=None, total_rounds=None, meta=None):
        if params_type is None:
            if params is not None:
                params_type = ParamsType.FULL
        else:
            params_type = ParamsType(params_type)
        if params_type in (ParamsType.FULL, ParamsType.DIFF) and params is None:
            raise ValueError(f"params must be provided when params_type is {params_type}")
        if metrics is not None and not isinstance(metrics, dict):
            raise TypeError(f"metrics must be dict, but got {type(metrics)}")
        for name, val in (("start_round", start_round), ("current_round", current_round), ("total_rounds", total_rounds)):
            if val is not None and (not isinstance(val, int) or val < 0):
                raise ValueError(f"{name} must be a non-negative int, but got {val!r}")
        if meta is not None and not isinstance(meta, dict):
            raise TypeError(f"meta must be dict, but got {type(meta)}")
        self.params_type = params_type
        self.params = params
        self.optimizer_params = optimizer_params
        self.metrics = metrics
        self.start_round = start_round
        self.current_round = current_round
        self.total_rounds = total_rounds
        self.meta = {} if meta is None else meta


_PARAMS_TYPE_TO_KIND = {ParamsType.FULL.value: DataKind.WEIGHTS, ParamsType.DIFF.value: DataKind.WEIGHT_DIFF}
_KIND_TO_PARAMS_TYPE = {DataKind.WEIGHTS: ParamsType.FULL, DataKind.WEIGHT_DIFF: ParamsType.DIFF}


class FLModelUtils:
    @staticmethod
    def to_shareable(fl_model: FLModel) -> Shareable:
        if fl_model.params is None and fl_model.metrics is None:
            raise ValueError("FLModel without params and metrics is NOT supported.")
        if fl_model.params is not None:
            if fl_model.params_type is None:
                fl_model.params_type = ParamsType.FULL
            kind = _PARAMS_TYPE_TO_KIND.get(ParamsType(fl_model.params_type).value)
            meta = {} if fl_model.metrics is None else {FLMetaKey.INITIAL_METRICS: fl_model.metrics}
            dxo = DXO(kind, data=fl_model.params, meta=meta)
        else:
            dxo = DXO(DataKind.METRICS, data=fl_model.metrics, meta={})
        dxo.meta.update(fl_model.meta or {})
        s = dxo.to_shareable()
        for key, val in ((AppConstants.START_ROUND, fl_model.start_round), (AppConstants.CURRENT_ROUND, fl_model.current_round),
                         (AppConstants.NUM_ROUNDS, fl_model.total_rounds)):
            if val is not None:
                s.set_header(key, val)
        return s

    @staticmethod
    def from_shareable(shareable: Shareable, fl_ctx: Optional[FLContext] = None) -> FLModel:
        dxo = from_shareable(shareable)
        meta = dict(dxo.meta)
        metrics = params = params_type = None
        if dxo.data_kind == DataKind.METRICS:
            metrics = dxo.data
        else:
            params = dxo.data
            params_type = _KIND_TO_PARAMS_TYPE.get(dxo.data_kind, ParamsType.FULL)
            metrics = meta.get(FLMetaKey.INITIAL_METRICS)
        return FLModel(params_type=params_type, params=params, metrics=metrics,
                       start_round=shareable.get_header(AppConstants.START_ROUND, None),
                       current_round=shareable.get_header(AppConstants.CURRENT_ROUND, None),
                       total_rounds=shareable.get_header(AppConstants.NUM_ROUNDS, None), meta=meta)


class ModelAggregator(Aggregator):
    """FLModel-level aggregator ABC (model_aggregator.py:26-83)."""

    def __init__(self):
        super().__init__()
        self.fl_ctx = None

    def handle_event(self, event_type: str, fl_ctx: FLContext):
        if event_type == EventType.START_RUN:
            self.fl_ctx = fl_ctx

    @abstractmethod
    def accept_model(self, model: FLModel):
        raise NotImplementedError

    @abstractmethod
    def aggregate_model(self) -> FLModel:
        raise NotImplementedError

    @abstractmethod
    def reset_stats(self):
        raise NotImplementedError

    def accept(self, shareable: Shareable, fl_ctx: FLContext) -> bool:
        self.fl_ctx = fl_ctx
        self.accept_model(FLModelUtils.from_shareable(shareable, fl_ctx))
        return True

    def aggregate(self, fl_ctx: FLContext) -> Shareable:
        self.fl_ctx = fl_ctx
        return FLModelUtils.to_shareable(self.aggregate_model())

    def reset(self, fl_ctx: FLContext):
        self.fl_ctx = fl_ctx
        self.reset_stats()

    def info(self, message: str):
        self.log_info(self.fl_ctx, message)

    def warning(self, message: str):
        self.log_warning(self.fl_ctx, message)

    def error(self, message: str):
        self.log_error(self.fl_ctx, message)

    def exception(self, message: str):
        self.log_exception(self.fl_ctx, message)


class Learnable(dict):
    def is_empty(self):
        return False


class ModelLearnableKey:
    WEIGHTS = "weights"
    META = "meta"


class ModelLearnable(Learnable):
    def is_empty(self):
        return not self.get(ModelLearnableKey.WEIGHTS)


def make_model_learnable(weights, meta_props) -> ModelLearnable:
    ml = ModelLearnable()
    ml[ModelLearnableKey.WEIGHTS] = weights
    ml[ModelLearnableKey.META] = meta_props
    return ml


def model_learnable_to_dxo(ml: ModelLearnable) -> DXO:
    if not isinstance(ml, ModelLearnable):
        raise ValueError(f"invalid model learnable: expect Model type but got {type(ml)}")
    for key in (ModelLearnableKey.WEIGHTS, ModelLearnableKey.META):
        if key not in ml:
            raise ValueError(f"invalid model learnable: missing {key}")
    return DXO(data_kind=DataKind.WEIGHTS, data=ml[ModelLearnableKey.WEIGHTS], meta=ml[ModelLearnableKey.META])


class ShareableGenerator(FLComponent, ABC):
    @abstractmethod
    def learnable_to_shareable(self, model: Learnable, fl_ctx: FLContext) -> Shareable:
        pass

    @abstractmethod
    def shareable_to_learnable(self, shareable: Shareable, fl_ctx: FLContext) -> Learnable:
        pass


class DXOFilter(FLComponent, ABC):
    """DXO-level filter (dxo_filter.py:26-140, without the job-audit event)."""

    def __init__(self, supported_data_kinds=None, data_kinds_to_filter=None):
        super().__init__()
        if supported_data_kinds and not isinstance(supported_data_kinds, list):
            raise ValueError(f"supported_data_kinds must be a list of str but got {type(supported_data_kinds)}")
        if data_kinds_to_filter and not isinstance(data_kinds_to_filter, list):
            raise ValueError(f"data_kinds_to_filter must be a list of str but got {type(data_kinds_to_filter)}")
        if supported_data_kinds and data_kinds_to_filter:
            if not all(dk in supported_data_kinds for dk in data_kinds_to_filter):
                raise ValueError(f"invalid data kinds: {data_kinds_to_filter}. Only support {supported_data_kinds}")
        self.data_kinds = data_kinds_to_filter or supported_data_kinds

    def process(self, shareable: Shareable, fl_ctx: FLContext):
        if shareable.get_return_code() != ReturnCode.OK:
            return shareable
        try:
            dxo = from_shareable(shareable)
        except Exception:
            return shareable
        if dxo.data is None:
            return shareable
        start = [dxo]
        self._filter_dxos(start, shareable, fl_ctx)
        return start[0].update_shareable(shareable)

    @abstractmethod
    def process_dxo(self, dxo: DXO, shareable: Shareable, fl_ctx: FLContext):
        pass

    def _apply_filter(self, dxo: DXO, shareable, fl_ctx) -> DXO:
        if not dxo.data:
            return dxo
        result = self.process_dxo(dxo, shareable, fl_ctx)
        if not result:
            return dxo
        if not isinstance(result, DXO):
            raise RuntimeError(f"Result from {self.__class__.__name__} is {type(result)} - must be DXO")
        if result is not dxo:
            result.add_filter_history(dxo.get_filter_history())
        result.add_filter_history(self.__class__.__name__)
        return result

    def _filter_dxos(self, coll, shareable, fl_ctx):
        items = list(enumerate(coll)) if isinstance(coll, list) else list(coll.items())
        for k, v in items:
            if not isinstance(v, DXO):
                continue
            if v.data_kind == DataKind.COLLECTION:
                self._filter_dxos(v.data, shareable, fl_ctx)
            elif not self.data_kinds or v.data_kind in self.data_kinds:
                coll[k] = self._apply_filter(v, shareable, fl_ctx)
