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


def load_fedavg_golden():
    """FedAvg-workflow cases (make_golden.py --set fedavg): BaseFedAvg.aggregate_fn and FedAvg's in-time path."""
    if "f" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "fedavg_cases.json")) as f:
            meta = json.load(f)
        arrays = dict(np.load(os.path.join(GOLDEN_DIR, "fedavg_cases.npz"), allow_pickle=False))
        _cache["f"] = (meta, arrays)
    return _cache["f"]


def decode_steps(rec):
    t = rec["t"]
    if t == "none":
        return None
    if t == "float":
        return float(rec["v"])
    return rec["v"]


def fl_models_from_case(case, arrays, FLModel, container):
    import torch

    models = []
    for c in case["clients"]:
        meta = {"client_name": c["name"]}
        steps = c["num_steps"]
        if steps["t"] != "none":
            meta["NUM_STEPS_CURRENT_ROUND"] = decode_steps(steps)
        params = {}
        for k, name in c["data"].items():
            a = np.array(arrays[name], copy=True)
            params[k] = torch.from_numpy(a) if container == "torch" else a
        models.append(FLModel(params=params, metrics=c["metrics"], current_round=3, meta=meta))
    return models


def load_scaffold_golden():
    """SCAFFOLD cases (make_golden.py --set scaffold): the reference's scaffold_aggregate_fn."""
    if "s" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "scaffold_cases.json")) as f:
            meta = json.load(f)
        arrays = dict(np.load(os.path.join(GOLDEN_DIR, "scaffold_cases.npz"), allow_pickle=False))
        _cache["s"] = (meta, arrays)
    return _cache["s"]


def scaffold_models_from_case(case, arrays, FLModel):
    """The case's clients as FLModels: params and SCAFFOLD_CTRL_DIFF in their recorded containers."""
    import torch

    def box(name, container):
        a = np.array(arrays[name], copy=True)
        return torch.from_numpy(a) if container == "torch" else a

    models = []
    for c in case["clients"]:
        meta = {"client_name": c["name"]}
        if c["num_steps"]["t"] != "none":
            meta["NUM_STEPS_CURRENT_ROUND"] = decode_steps(c["num_steps"])
        if c["ctrl"] is not None:
            meta["scaffold_c_diff"] = {k: box(n, c["ctrl_container"]) for k, n in c["ctrl"].items()}
        models.append(FLModel(params={k: box(n, c["params_container"]) for k, n in c["params"].items()},
                              metrics=c["metrics"], current_round=3, meta=meta))
    return models


def check_scaffold_result(case, arrays, out):
    """Params, controls (values, dtypes, containers, key order), metrics and meta as the reference made them."""
    import torch

    exp = case["expected"]

    def same(got, name, kind, dtype, what):
        assert isinstance(got, torch.Tensor if kind == "torch" else np.ndarray), (case["name"], what)
        if isinstance(got, torch.Tensor):
            assert str(got.dtype).replace("torch.", "") == dtype, (case["name"], what)
            got = got.numpy()
        assert str(got.dtype) == dtype and same_bits(got, arrays[name]), (case["name"], what)

    assert list(out.params) == exp["params_order"]
    for k, name in exp["params"].items():
        same(out.params[k], name, exp["params_kind"][k], exp["params_dtype"][k], k)
    ctrl = out.meta["scaffold_c_diff"]
    assert list(ctrl) == exp["ctrl_order"]
    for k, name in exp["ctrl"].items():
        same(ctrl[k], name, exp["ctrl_kind"][k], exp["ctrl_dtype"][k], "ctrl " + k)
    assert str(out.params_type.value if out.params_type is not None else None) == exp["params_type"]
    assert same_metrics(out.metrics, exp["metrics"]), (out.metrics, exp["metrics"])
    assert {k: v for k, v in out.meta.items() if k != "scaffold_c_diff"} == exp["meta"]


def same_metrics(a, b) -> bool:
    """Exact equality of metric dicts (python floats; NaN == NaN)."""
    import math

    if a is None or b is None:
        return a is None and b is None
    if set(a) != set(b):
        return False
    for k in a:
        x, y = float(a[k]), float(b[k])
        if not (x == y or (math.isnan(x) and math.isnan(y))):
            return False
    return True


def load_fedopt_golden():
    """PTFedOptModelShareableGenerator cases (make_golden.py --set fedopt), reference run on CPU."""
    if "o" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "fedopt_cases.json")) as f:
            meta = json.load(f)
        arrays = dict(np.load(os.path.join(GOLDEN_DIR, "fedopt_cases.npz"), allow_pickle=False))
        _cache["o"] = (meta, arrays)
    return _cache["o"]


def fedopt_model():
    """Same architecture as make_golden.py's fedopt_model (state is loaded from the fixture)."""
    import torch

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin1 = torch.nn.Linear(7, 64)
            self.bn = torch.nn.BatchNorm1d(64)
            self.lin2 = torch.nn.Linear(64, 90, bias=False)
            self.register_buffer("offset", torch.zeros(5))

    return Net()


def fedopt_params_exact(reference_sqrt: str) -> bool:
    """Whether a FedOpt step with a sqrt must reproduce the reference's parameters bit for bit: the device
    epilogue runs torch CPU's restated sqrt (nvflare_amd.torch_sqrt.mode()) and the reference computed that same
    sqrt -- ``reference_sqrt`` is "torch_cpu" for the golden fixtures (generated where torch's vsSqrt is the
    restated one, tests/test_torch_sqrt.py), or "live" for torch running on this host (torch_sqrt.detect())."""
    from nvflare_amd import torch_sqrt

    ref = torch_sqrt.detect() if reference_sqrt == "live" else reference_sqrt
    return ref in torch_sqrt.MODES and torch_sqrt.mode() == ref


def assert_fedopt_param(got, ref, p0, lr, steps, reference_sqrt, msg=""):
    """Bit-exact when fedopt_params_exact(reference_sqrt), else within adam_param_tolerance (a device sqrt that is
    not the reference's: e.g. NVFLARE_AMD_TORCH_SQRT=ieee, or a host whose torch sqrt matches neither)."""
    if fedopt_params_exact(reference_sqrt):
        assert same_bits(got, ref), (msg, int(np.count_nonzero(np.asarray(got).view(np.uint32) != np.asarray(ref).view(np.uint32))))
        return
    tol = adam_param_tolerance(p0, ref, lr, max(steps, 1))
    d = np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64))
    assert np.all(d <= tol), (msg, float((d / tol).max()))


def adam_param_tolerance(p0, p_ref, lr, steps):
    """|p - p_torch| bound for Adam params: torch CPU's MKL sqrt is not correctly rounded (see
    tests/test_fedopt_oracle.py); its error passes through the two divisions into the update and the
    final rounding of p + update can land one binade up: 2 * steps * spacing(max(|p0|, |p_torch|, lr))
    (measured maximum: 2 spacings after one step, golden case numpy_adam_wd)."""
    return 2 * steps * np.spacing(np.maximum(np.maximum(np.abs(p0), np.abs(p_ref)), np.float32(lr))).astype(np.float64)


def load_quant_golden():
    """AdaQuantizer round trips of the reference (make_golden.py --set quant)."""
    if "q" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "quant_cases.json")) as f:
            meta = json.load(f)
        arrays = dict(np.load(os.path.join(GOLDEN_DIR, "quant_cases.npz"), allow_pickle=False))
        _cache["q"] = (meta, arrays)
    return _cache["q"]


def adaquant_state(case, arrays):
    """The case's quant_state with its arrays restored."""
    return {k: (arrays[v["array"]] if isinstance(v, dict) else v) for k, v in case["quant_state"].items()}


# --- reduced-precision / integer client arrays (make_golden.py --set dtypes) -------------------------------
def load_dtype_golden():
    if "d" not in _cache:
        with open(os.path.join(GOLDEN_DIR, "dtype_cases.json")) as f:
            meta = json.load(f)
        arrays = dict(np.load(os.path.join(GOLDEN_DIR, "dtype_cases.npz"), allow_pickle=False))
        _cache["d"] = (meta, arrays)
    return _cache["d"]


def dtype_case_weights(case):
    """Weights as the reference received them (python floats, or numpy scalars of the recorded type)."""
    out = []
    for w, t in zip(case["weights"], case["weight_types"]):
        if t in ("float32", "float64", "float16"):
            out.append(getattr(np, t)(float(w[w.index("(") + 1:-1])))
        else:
            out.append(w)
    return out


def dtype_case_inputs(case, arrays):
    """Client values as the reference received them (numpy arrays or CPU tensors; bfloat16 from bits)."""
    import torch

    rows = []
    for name in case["rows"]:
        a = np.array(arrays[name], copy=True)
        if case["dtype"] == "bfloat16":
            rows.append(torch.from_numpy(a.view(np.int16)).view(torch.bfloat16))
        elif case["container"] == "torch":
            rows.append(torch.from_numpy(a))
        else:
            rows.append(a)
    return rows


def as_f32_values(v, dtype: str) -> np.ndarray:
    """fp32 values of a 16-bit result (numpy array, tensor or stored bits)."""
    import torch

    if isinstance(v, torch.Tensor):
        v = v.view(torch.int16).numpy().view(np.uint16) if v.dtype == torch.bfloat16 else v.numpy()
    v = np.asarray(v)
    if dtype == "bfloat16":
        return (v.astype(np.uint32) << 16).view(np.float32)
    return v.astype(np.float32)


def torch16_tail_tolerance(rows_f32, weights, expected_f32, dtype: str) -> np.ndarray:
    """Bound for torch's scalar-tail elements (the last n % 32 of a thread's chunk), where torch rounds the
    add_ product and the sum separately instead of one fp32 fma: at most one 16-bit rounding per step of
    the running sum, whose magnitude is bounded by sum_k |w_k v_k|, scaled by the final division."""
    mag = np.zeros_like(expected_f32, dtype=np.float64)
    for r, w in zip(rows_f32, weights):
        mag += np.abs(r.astype(np.float64) * float(w))
    count = float(sum(float(w) for w in weights))
    ulp_bits = 10 if dtype == "float16" else 7
    ulp = lambda x: np.exp2(np.floor(np.log2(np.maximum(np.abs(x), 1e-30))) - ulp_bits)
    return (len(rows_f32) + 1) * ulp(mag) / abs(count) + ulp(expected_f32)
