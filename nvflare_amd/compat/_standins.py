"""Minimal stand-ins for the NVFlare API types the aggregator touches.

Used only when the real ``nvflare`` package is not importable (e.g. on a bare GPU box or in this
repository's tests).  They reproduce the behaviour the aggregation path relies on -- nothing more:

* ``DXO`` / ``from_shareable`` / ``DataKind`` / ``MetaKey``      nvflare/apis/dxo.py:23-177
* ``Shareable`` (headers, cookies, peer props, return code)      nvflare/apis/shareable.py:41-127
* ``FLContext.get_prop/set_prop``                                 nvflare/apis/fl_context.py:134-175
* ``FLComponent`` logging helpers and ``handle_event``            nvflare/apis/fl_component.py:28-231
* ``Aggregator`` ABC                                               nvflare/app_common/abstract/aggregator.py:22-58
* constants: ``ReservedKey`` (fl_constant.py:69-80), ``ReturnCode`` (:26-36),
  ``AppConstants`` (app_common/app_constant.py:33-79), ``EventType.START_RUN`` (apis/event_type.py:22)
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


class AppConstants:
    CURRENT_ROUND = "current_round"
    NUM_ROUNDS = "num_rounds"
    CONTRIBUTION_ROUND = "contribution_round"
    GLOBAL_MODEL = "global_model"
    AGGREGATION_STATS = "_aggregation_stats"


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
