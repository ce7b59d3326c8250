"""GPU drop-in for ``nvflare.app_common.aggregators.weighted_aggregation_helper``.

Same public surface as the reference module (weighted_aggregation_helper.py:20-271):
``WeightedAggregationHelper(exclude_vars, weigh_by_local_iter)`` with ``add`` / ``get_result`` /
``reset_stats`` / ``get_aggregation_stats`` / ``get_history`` / ``get_len`` and the
``last_aggregation_stats`` snapshot; ``AggregationStatsKey``, ``compute_key_match_stats`` and
``filter_aggregatable_metrics`` are provided with the reference's behaviour.

Where the arithmetic runs:
* every numpy array / torch tensor value goes to the HIP kernels through ``DeviceFedAvg`` (no CPU
  fallback: a missing HIP library raises);
* values that are not arrays (python numbers, opaque objects such as HE ciphertexts, lazily
  materialised refs after ``materialize()``) follow the reference's object protocol on the host
  (``v * w``, ``total + v * w``, ``total * (1.0 / count)``): they are bookkeeping, not tensors.

Results are bitwise equal to the reference on identical inputs and arrival order (tests/).
"""

from __future__ import annotations

import re
import threading
from typing import Any, Callable, Dict, Optional, Set

import numpy as np

from ...engine import DeviceFedAvg, is_device_array
from ...ingest import as_mapped
from ...quantized import QuantizedPayload
from ...sharding import ShardedFedAvg


def _is_aggregatable_metric_value(v: Any) -> bool:
    """True if ``v`` supports ``v * w`` and ``v + v`` (weighted_aggregation_helper.py:20-38).

    Containers and strings never aggregate; bools count as 0/1 rates.  TypeError / ValueError /
    AttributeError from the probe mean "not aggregatable"; any other exception propagates."""
    if v is None or isinstance(v, (dict, list, set, tuple, str)):
        return False
    if isinstance(v, (int, float, bool)):
        return True
    try:
        v * 1.0
        v + v
    except (TypeError, ValueError, AttributeError):
        return False
    return True


def filter_aggregatable_metrics(
    metrics: Optional[Dict[str, Any]],
    warn_skipped: Optional[Callable[[str, str], None]] = None,
    warned_metric_keys: Optional[Set[str]] = None,
) -> Dict[str, Any]:
    """Keep only aggregatable metric entries (weighted_aggregation_helper.py:41-71)."""
    out: Dict[str, Any] = {}
    for key, value in (metrics or {}).items():
        if _is_aggregatable_metric_value(value):
            out[key] = value
        elif warn_skipped is not None and (warned_metric_keys is None or key not in warned_metric_keys):
            warn_skipped(key, type(value).__name__)
            if warned_metric_keys is not None:
                warned_metric_keys.add(key)
    return out


class AggregationStatsKey:
    """Keys of the per-round aggregation stats dict (weighted_aggregation_helper.py:74-84)."""

    ROUND = "round"
    ACCEPTED_CONTRIBUTIONS = "accepted_contributions"
    CONTRIBUTORS = "contributors"
    KEYS_AGGREGATED = "keys_aggregated"
    KEYS_SEEN = "keys_seen"
    FULLY_MATCHED_KEYS = "fully_matched_keys"
    PARTIALLY_MATCHED_KEYS = "partially_matched_keys"
    SKIPPED_KEYS = "skipped_keys"


def _stats(n_contrib: int, contributors, key_counts: Dict[str, int], n_aggregated: int, n_skipped: int) -> dict:
    full = sum(1 for c in key_counts.values() if c == n_contrib) if n_contrib > 0 else 0
    return {
        AggregationStatsKey.ACCEPTED_CONTRIBUTIONS: n_contrib,
        AggregationStatsKey.CONTRIBUTORS: sorted(set(contributors)),
        AggregationStatsKey.KEYS_AGGREGATED: n_aggregated,
        AggregationStatsKey.KEYS_SEEN: n_aggregated + n_skipped,
        AggregationStatsKey.FULLY_MATCHED_KEYS: full,
        AggregationStatsKey.PARTIALLY_MATCHED_KEYS: n_aggregated - full,
        AggregationStatsKey.SKIPPED_KEYS: n_skipped,
    }


def compute_key_match_stats(contributions: Dict[str, Any]) -> dict:
    """Key-match stats from {contributor: iterable of keys} (weighted_aggregation_helper.py:87-114)."""
    counts: Dict[str, int] = {}
    for keys in contributions.values():
        for k in keys:
            counts[k] = counts.get(k, 0) + 1
    return _stats(len(contributions), contributions.keys(), counts, len(counts), 0)


_ON_DEVICE = "device"  # marker in self.total: the key's running sum lives in the engine


class _HostValue:
    """Running sum of one non-array key, with the reference's object arithmetic."""

    __slots__ = ("total",)

    def __init__(self, total):
        self.total = total


class WeightedAggregationHelper(object):
    def __init__(
        self,
        exclude_vars: Optional[str] = None,
        weigh_by_local_iter: bool = True,
        device: Optional[int] = None,
        max_resident_bytes: Optional[int] = None,
        devices: Optional[list] = None,
        defer_result: bool = False,
    ):
        """Weighted aggregation on the MI355X (drop-in for weighted_aggregation_helper.py:117-131).

        Args:
            exclude_vars: regex of keys to skip.
            weigh_by_local_iter: multiply each contribution by its weight (False: plain sum, still
                divided by the sum of weights).
            device: HIP device index (default: $NVFLARE_AMD_DEVICE or 0).
            max_resident_bytes: HBM budget for staged contributions before they are folded.
            devices: several HIP devices: every key is split into per-device parameter buckets
                (sharding.ShardedFedAvg; host arrays only), bit-identical to one device.
            defer_result: ``get_result`` returns the fp32 keys as ``DeferredAggregate`` values
                (``ShardedDeferredAggregate`` with ``devices``) that stay in HBM until read
                (``materialize()`` / ``np.asarray``) or consumed by the device FedOpt generator in the same
                launch as its optimizer step (nvflare_amd/deferred.py).
        """
        super().__init__()
        self.lock = threading.Lock()
        self.exclude_vars = re.compile(exclude_vars) if exclude_vars else None
        self.weigh_by_local_iter = weigh_by_local_iter
        self.defer_result = bool(defer_result)
        if devices and len(devices) > 1:
            self._engine = ShardedFedAvg(devices, max_resident_bytes=max_resident_bytes)
        else:
            dev = devices[0] if devices else device
            self._engine = DeviceFedAvg(device=dev, max_resident_bytes=max_resident_bytes)
        self.last_aggregation_stats = None
        self.reset_stats()

    @property
    def engine(self) -> DeviceFedAvg:
        return self._engine

    def reset_stats(self):
        self.total = dict()  # key -> device key state or _HostValue (len() = keys aggregated)
        self.counts = dict()
        self.history = list()
        self.key_contribution_counts = dict()
        self.skipped_keys = set()
        self._engine.reset()

    @staticmethod
    def _is_pytorch_tensor(tensor):
        return hasattr(tensor, "add_") and hasattr(tensor, "mul_") and hasattr(tensor, "clone")

    def add(self, data, weight, contributor_name, contribution_round):
        """Stage one contribution (arrival order is the accumulation order, as in the reference)."""
        with self.lock:
            device_items = []
            host_items = []
            sharded = isinstance(self._engine, ShardedFedAvg)
            total = self.total
            skipped, counted = [], []  # committed once the device has staged the contribution
            for k, v in data.items():
                if self.exclude_vars is not None and self.exclude_vars.search(k):
                    skipped.append(k)
                    continue
                counted.append(k)
                if type(v) is np.ndarray:  # plain array: no lazy ref, no quantized payload -> device unless host key
                    (host_items if isinstance(total.get(k), _HostValue) else device_items).append((k, v))
                    continue
                materialize = getattr(v, "materialize", None)
                device_quantized = isinstance(v, QuantizedPayload) and not sharded
                mapped = None
                if callable(materialize) and not device_quantized and not sharded \
                        and not isinstance(total.get(k), _HostValue):
                    mapped = as_mapped(v)  # disk-offloaded safetensors ref: staged from the mmap, no tensor built
                if mapped is not None:
                    v = mapped
                elif callable(materialize) and not device_quantized:
                    # lazy disk-offloaded refs (weighted_aggregation_helper.py:170-175); quantized payloads
                    # stay compressed until the engine dequantizes them into their slot
                    v = materialize()
                if isinstance(v, QuantizedPayload) and isinstance(self.total.get(k), _HostValue):
                    v = v.materialize()
                if is_device_array(v) and not isinstance(self.total.get(k), _HostValue):
                    device_items.append((k, v))
                else:
                    host_items.append((k, v))
            if device_items:
                # all or nothing (engine.DeviceFedAvg.add): a failed staging leaves no trace of this contribution
                self._engine.add(device_items, weight, self.weigh_by_local_iter)
                for k, _ in device_items:
                    self.total[k] = _ON_DEVICE
            self.skipped_keys.update(skipped)
            kcc = self.key_contribution_counts
            for k in counted:
                kcc[k] = kcc.get(k, 0) + 1
            for k, v in host_items:
                self._add_host(k, v, weight)
            for k, _ in device_items:
                self.counts[k] = weight if k not in self.counts else self.counts[k] + weight
            self.history.append({"contributor_name": contributor_name, "round": contribution_round, "weight": weight})

    def _add_host(self, k, v, weight):
        cur = self.total.get(k)
        if cur is None:
            if self.weigh_by_local_iter:
                t = v.mul(weight) if self._is_pytorch_tensor(v) else v * weight
            elif self._is_pytorch_tensor(v):
                t = v.clone()
            else:
                try:
                    t = v.copy() if hasattr(v, "copy") else v
                except (ValueError, RuntimeError):
                    t = v  # e.g. an encrypted value that cannot be copied: immutable, safe to reference
            self.total[k] = _HostValue(t)
            self.counts[k] = weight
        else:
            if not isinstance(cur, _HostValue):
                raise TypeError(f"nvflare_amd: key {k!r} mixes device arrays and host objects")
            if self._is_pytorch_tensor(v) and self._is_pytorch_tensor(cur.total):
                if self.weigh_by_local_iter:
                    cur.total.add_(v, alpha=weight)
                else:
                    cur.total.add_(v)
            else:
                cur.total = cur.total + v * weight if self.weigh_by_local_iter else cur.total + v
            self.counts[k] = self.counts[k] + weight

    def get_result(self):
        """Divide the weighted sums by the sums of weights (weighted_aggregation_helper.py:226-240)."""
        with self.lock:
            if not self._engine.keys:
                device_results = {}
            elif self.defer_result:
                device_results = self._engine.result_deferred()
            else:
                device_results = self._engine.result()
            aggregated = {}
            total = self.total
            # key_contribution_counts holds the keys in first-arrival order (the reference's ``total`` order);
            # ``total`` itself lists a contribution's device keys before its host keys
            for k in self.key_contribution_counts:
                v = total.get(k)
                if v is None:
                    continue
                if isinstance(v, _HostValue):
                    t = v.total
                    aggregated[k] = t.div_(self.counts[k]) if self._is_pytorch_tensor(t) else t * (1.0 / self.counts[k])
                else:
                    aggregated[k] = device_results[k]
            self.last_aggregation_stats = self._compute_aggregation_stats()
            self.reset_stats()
            return aggregated

    def _compute_aggregation_stats(self) -> dict:
        return _stats(
            len(self.history),
            [h["contributor_name"] for h in self.history],
            self.key_contribution_counts,
            len(self.total),
            len(self.skipped_keys),
        )

    def get_aggregation_stats(self) -> dict:
        with self.lock:
            return self._compute_aggregation_stats()

    def get_history(self):
        return self.history

    def get_len(self):
        return len(self.get_history())
