"""CPU-only checks: the C-ABI library loads and exports every symbol of include/nvflare_amd_fedavg.h
(no compute calls), host-side config validation of the drop-in (ported from the reference's
in_time_accumulate_weighted_aggregator_test.py:32-155), the dtype-promotion table the engine uses,
the compat stand-ins and the SAG harness."""

import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nvflare_amd_fedavg.h")


def _declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(fedavg_\w+)\s*\(", text, re.M)))


def test_library_builds_and_exports_header_symbols():
    from nvflare_amd import _build, _native

    _build.build_library()
    lib = ctypes.CDLL(_build.LIB_PATH)
    declared = _declared_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_native.EXPORTED)
    assert _native.load().fedavg_abi_version() == _native.ABI_VERSION
    # struct layouts: the library's sizeof matches the ctypes mirrors (load() refuses a mismatch)
    assert _native.load().fedavg_struct_size(0) == ctypes.sizeof(_native.Epilogue)
    assert _native.load().fedavg_struct_size(1) == ctypes.sizeof(_native.Quant)
    assert _native.load().fedavg_struct_size(7) == 0


def test_library_is_gfx950_code_object():
    from nvflare_amd import _build

    data = open(_build.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU error path")
def test_no_device_fails_loudly():
    from nvflare_amd import _native

    with pytest.raises(_native.FedAvgError, match="hipGetDeviceCount|no ROCm|device"):
        _native.device_count()


def test_missing_library_fails_loudly(monkeypatch):
    from nvflare_amd import _native

    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setenv("NVFLARE_AMD_FEDAVG_LIB", "/nonexistent/lib.so")
    with pytest.raises(_native.FedAvgError, match="no CPU fallback"):
        _native.load()


# --- config validation (no GPU: the engine opens its device lazily) -----------------------------------------
from nvflare_amd.compat import DataKind  # noqa: E402


@pytest.mark.parametrize(
    "exclude_vars,aggregation_weights,expected_data_kind,error_msg,is_regex",
    [
        (2.0, None, DataKind.WEIGHT_DIFF, f"exclude_vars = 2.0 should be a regex string but got {type(2.0)}.", False),
        ({"dxo1": 3.0, "dxo2": ""}, None, {"dxo1": DataKind.WEIGHT_DIFF, "dxo2": DataKind.WEIGHT_DIFF},
         f"exclude_vars[dxo1] = 3.0 should be a regex string but got {type(3.0)}.", False),
        (None, None, DataKind.ANALYTIC, r"expected_data_kind.*ANALYTIC.*is not.*WEIGHT_DIFF.*WEIGHTS.*METRICS", True),
        (None, None, {"dxo1": DataKind.WEIGHT_DIFF, "dxo2": DataKind.ANALYTIC},
         r"expected_data_kind\[dxo2\].*ANALYTIC.*is not.*WEIGHT_DIFF.*WEIGHTS.*METRICS", True),
        (None, {"dxo1": {"client_0": 1.0, "client_1": 2.0}}, {"dxo1": DataKind.WEIGHT_DIFF, "dxo2": DataKind.WEIGHT_DIFF},
         "A dict of dict aggregation_weights should specify aggregation_weights "
         "for every key in expected_data_kind. But missed these keys: ['dxo2']", False),
        ({"dxo2": ""}, None, {"dxo1": DataKind.WEIGHT_DIFF, "dxo2": DataKind.WEIGHT_DIFF},
         "A dict exclude_vars should specify exclude_vars for every key in expected_data_kind. "
         "But missed these keys: ['dxo1']", False),
    ],
)
def test_invalid_create(exclude_vars, aggregation_weights, expected_data_kind, error_msg, is_regex):
    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator

    with pytest.raises(ValueError) as exc_info:
        a = InTimeAccumulateWeightedAggregator(exclude_vars=exclude_vars, aggregation_weights=aggregation_weights,
                                               expected_data_kind=expected_data_kind)
        a._initialize(a.aggregation_weights, a.exclude_vars, a.expected_data_kind)
    msg = str(exc_info.value)
    assert re.search(error_msg, msg) if is_regex else error_msg in msg


@pytest.mark.parametrize(
    "args,expected_args",
    [
        (dict(exclude_vars=None, aggregation_weights=None, expected_data_kind=DataKind.WEIGHTS),
         dict(exclude_vars=None, aggregation_weights=None, expected_data_kind=DataKind.WEIGHTS)),
        (dict(exclude_vars="hello", aggregation_weights=None, expected_data_kind={"dxo1": DataKind.WEIGHTS, "dxo2": DataKind.WEIGHT_DIFF}),
         dict(exclude_vars={"dxo1": "hello", "dxo2": "hello"}, aggregation_weights=None,
              expected_data_kind={"dxo1": DataKind.WEIGHTS, "dxo2": DataKind.WEIGHT_DIFF})),
        (dict(exclude_vars=None, aggregation_weights={"client_0": 1.0, "client_1": 2.0},
              expected_data_kind={"dxo1": DataKind.WEIGHTS, "dxo2": DataKind.WEIGHT_DIFF}),
         dict(exclude_vars=None,
              aggregation_weights={"dxo1": {"client_0": 1.0, "client_1": 2.0}, "dxo2": {"client_0": 1.0, "client_1": 2.0}},
              expected_data_kind={"dxo1": DataKind.WEIGHTS, "dxo2": DataKind.WEIGHT_DIFF})),
    ],
)
def test_create(args, expected_args):
    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator

    e = InTimeAccumulateWeightedAggregator(**expected_args)
    e._initialize(e.aggregation_weights, e.exclude_vars, e.expected_data_kind)
    r = InTimeAccumulateWeightedAggregator(**args)
    r._initialize(r.aggregation_weights, r.exclude_vars, r.expected_data_kind)
    assert r.exclude_vars == e.exclude_vars
    assert r.aggregation_weights == e.aggregation_weights
    assert r.expected_data_kind == e.expected_data_kind


def test_string_data_kind_from_job_config():
    """job configs pass expected_data_kind = "WEIGHTS" (job_templates/sag_np/config_fed_server.conf:81)."""
    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator

    a = InTimeAccumulateWeightedAggregator(expected_data_kind="WEIGHTS")
    a._initialize(a.aggregation_weights, a.exclude_vars, a.expected_data_kind)
    assert a.expected_data_kind == {"": "WEIGHTS"}


# --- dtype promotion table used by the engine: checked against numpy / torch themselves --------------------
@pytest.mark.parametrize("dt", [np.float32, np.float64, np.int32, np.int64, np.float16, np.uint8, np.int8, np.int16,
                                np.bool_, np.uint16, np.uint32, np.uint64])
@pytest.mark.parametrize("weight", [0.75, np.float64(0.75), np.float32(0.75), np.float16(0.75)])
def test_numpy_promotion_table(dt, weight):
    from nvflare_amd.engine import _resolve_types

    v = np.ones(3, dtype=dt)
    ref = (v * weight + v * weight) * (1.0 / (weight + weight))
    unsupported = (ref.dtype == np.float32 and np.dtype(dt) in (np.dtype(np.uint16), np.dtype(np.uint32), np.dtype(np.uint64))) or \
        (ref.dtype == np.float16 and np.dtype(dt) != np.float16)
    if unsupported:  # no (input, accumulator) kernel: refused, never computed on the host
        with pytest.raises(TypeError):
            _resolve_types(v, weight, True)
        return
    _, in_np, acc_np, op, fin = _resolve_types(v, weight, True)
    assert acc_np == ref.dtype


@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.int32, torch.int64, torch.float16, torch.bfloat16,
                                torch.uint8, torch.int8, torch.int16, torch.bool])
def test_torch_promotion_table(dt):
    from nvflare_amd.engine import _NP_TO_TORCH, _resolve_types

    v = torch.ones(3, dtype=dt)
    _, in_np, acc_np, op, fin = _resolve_types(v, 0.75, True)
    t = v.mul(0.75)
    t.add_(v, alpha=0.75)
    assert _NP_TO_TORCH[acc_np] == t.div_(1.5).dtype


def test_unsupported_dtypes_raise():
    from nvflare_amd.engine import _resolve_types

    with pytest.raises(TypeError):
        _resolve_types(np.ones(3, np.complex64), 1.0, True)
    with pytest.raises(TypeError):
        _resolve_types(torch.ones(3, dtype=torch.complex64), 1.0, True)
    # weigh_by_local_iter=False integer values: numpy sums in the array dtype then scales to float64; torch keeps
    # an integer total whose div_ raises at get_result (the engine raises the same RuntimeError there)
    from nvflare_amd import _native as N

    assert _resolve_types(np.ones(3, np.int32), 1.0, False)[2:4] == (np.dtype(np.float64), N.FEDAVG_OP_UNWEIGHTED)
    assert _resolve_types(torch.ones(3, dtype=torch.int64), 1.0, False)[2] == np.dtype(np.int64)


def test_unweighted_integers_on_the_fake_device():
    """numpy integer / bool sums wrap (bool: OR) and scale to float64 as numpy does; a torch integer key makes
    result() raise torch's div_ RuntimeError, as the reference's get_result does."""
    from fake_device import fake_engine

    e = fake_engine(max_resident_bytes=1)  # folds after every contribution: the sum continues through acc_in
    vals = {"i8": [np.array([100, -100, 7], np.int8), np.array([100, -100, 9], np.int8), np.array([1, 2, 3], np.int8)],
            "b": [np.array([True, False, False]), np.array([True, True, False]), np.array([False, False, False])],
            "u64": [np.array([2**63, 5], np.uint64)] * 3}
    ws = [1.0, 2.5, 0.25]
    for k in range(3):
        e.add([(n, v[k]) for n, v in vals.items()], ws[k], False)
    out = e.result()
    c = ws[0] + ws[1] + ws[2]
    for n, v in vals.items():
        t = v[0].copy()
        for x in v[1:]:
            t = t + x
        exp = t * (1.0 / c)
        assert out[n].dtype == np.float64 and np.array_equal(out[n], exp), n
    e2 = fake_engine()
    e2.add([("f", torch.ones(3)), ("n", torch.ones(2, dtype=torch.int32))], 1.0, False)
    with pytest.raises(RuntimeError, match="desired output type Int"):
        e2.result()


# --- compat stand-ins ----------------------------------------------------------------------------------------
def test_compat_shareable_dxo_roundtrip():
    from nvflare_amd.compat import DXO, AppConstants, DataKind, MetaKey, ReservedKey, ReturnCode, Shareable, from_shareable

    s = DXO(DataKind.WEIGHTS, data={"a": 1}, meta={MetaKey.NUM_STEPS_CURRENT_ROUND: 3}).to_shareable()
    s.set_peer_props({ReservedKey.IDENTITY_NAME: "site-9"})
    s.add_cookie(AppConstants.CONTRIBUTION_ROUND, 4)
    assert s.get_peer_prop(ReservedKey.IDENTITY_NAME, "?") == "site-9"
    assert s.get_cookie(AppConstants.CONTRIBUTION_ROUND) == 4
    assert s.get_return_code() == ReturnCode.OK
    d = from_shareable(s)
    assert d.data_kind == DataKind.WEIGHTS and d.data == {"a": 1} and d.get_meta_prop(MetaKey.NUM_STEPS_CURRENT_ROUND) == 3
    with pytest.raises(ValueError):
        from_shareable(Shareable())


# --- SAG harness validated with a host-side oracle aggregator (test infra only) -----------------------------
class _OracleAggregator:
    """Host restatement used only to validate tests/sag_harness.py on CPU."""

    def __init__(self):
        self.rows, self.ws = [], []

    def handle_event(self, *a):
        pass

    def accept(self, s, fl_ctx):
        from nvflare_amd.compat import MetaKey, from_shareable

        d = from_shareable(s)
        self.kind = d.data_kind
        self.rows.append(d.data)
        self.ws.append(1.0 * float(d.get_meta_prop(MetaKey.NUM_STEPS_CURRENT_ROUND)))
        return True

    def aggregate(self, fl_ctx):
        from oracle.fedavg_oracle import numpy_mode_reference

        from nvflare_amd.compat import DXO

        keys = self.rows[0].keys()
        out = {k: numpy_mode_reference([r[k] for r in self.rows], self.ws) for k in keys}
        self.rows, self.ws = [], []
        return DXO(self.kind, data=out).to_shareable()

    def reset(self, fl_ctx):
        pass


def test_sag_harness_known_answer_with_oracle():
    from sag_harness import NUMPY_KEY, run_sag

    model, _ = run_sag(_OracleAggregator(), n_clients=2, num_rounds=3)
    np.testing.assert_equal(model[NUMPY_KEY], [[4, 5, 6], [7, 8, 9], [10, 11, 12]])


def test_deprecated_accumulate_aggregator_path():
    """accumulate_model_aggregator.py:20-22: the deprecated class path exists and is the InTime aggregator."""
    import warnings

    from nvflare_amd.app_common.aggregators.accumulate_model_aggregator import AccumulateWeightedAggregator
    from nvflare_amd.app_common.aggregators.intime_accumulate_model_aggregator import InTimeAccumulateWeightedAggregator

    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        agg = AccumulateWeightedAggregator(expected_data_kind="WEIGHTS")
    assert isinstance(agg, InTimeAccumulateWeightedAggregator)
    assert any(issubclass(x.category, DeprecationWarning) for x in w)
