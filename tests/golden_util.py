"""Loader for the golden vectors produced by tests/golden/make_golden.py (reference outputs)."""

from __future__ import annotations

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_cache = {}


def load_golden():
    if "g" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "helper_cases.json")) as f:
            meta = json.load(f)
        arrays = dict(np.load(os.path.join(GOLDEN_DIR, "helper_cases.npz"), allow_pickle=False))
        _cache["g"] = (meta, arrays)
    return _cache["g"]


def helper_cases():
    meta, arrays = load_golden()
    return [c for c in meta["cases"] if c["kind"] == "helper"], arrays


def intime_cases():
    meta, arrays = load_golden()
    return [c for c in meta["cases"] if c["kind"] == "intime"], arrays


def per_key_sequences(case, arrays):
    """Yield (key, [rows in arrival order], [weights]) for every aggregated key of a helper case,
    applying exclude_vars exactly as weighted_aggregation_helper.py:164-166 does."""
    import re

    excl = re.compile(case["exclude_vars"]) if case["exclude_vars"] else None
    seq = {}
    for c in case["contributions"]:
        for k, name in c["data"].items():
            if excl is not None and excl.search(k):
                continue
            seq.setdefault(k, ([], []))
            seq[k][0].append(arrays[name])
            seq[k][1].append(c["weight"])
    return seq


def same_bits(a: np.ndarray, b: np.ndarray) -> bool:
    """Bitwise equality, except that any NaN matches any NaN (payloads are not part of the contract)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    an = np.isnan(a) if a.dtype.kind == "f" else np.zeros(a.shape, bool)
    bn = np.isnan(b) if b.dtype.kind == "f" else np.zeros(b.shape, bool)
    if not np.array_equal(an, bn):
        return False
    ua = a[~an].view(np.uint8)
    ub = b[~bn].view(np.uint8)
    return np.array_equal(ua, ub)
