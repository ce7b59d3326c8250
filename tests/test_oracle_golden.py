"""Pin the CPU oracle against the reference's own outputs (tests/golden/, made by make_golden.py).

Every restatement in oracle/fedavg_oracle.py must reproduce the reference helper bit-for-bit
(weighted_aggregation_helper.py:153-240), NaN payloads excepted."""

import numpy as np
import pytest
import torch

from golden_util import helper_cases, per_key_sequences, same_bits

CASES, ARRAYS = helper_cases()


def _conv(rows, container):
    kind = rows[0].dtype.kind
    if kind in "iub":
        # numpy: int * python float -> float64; torch: long.mul(float) -> default dtype float32
        return [r.astype(np.float64 if container == "numpy" else np.float32) for r in rows]
    return rows


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_c_oracle_matches_reference(case, oracle):
    mode = oracle.MODE_TORCH if case["container"] == "torch" else oracle.MODE_NUMPY
    for key, (rows, ws) in per_key_sequences(case, ARRAYS).items():
        exp = ARRAYS[case["expected"][key]]
        rows = _conv(rows, case["container"])
        got = oracle.fedavg_c(rows, ws, mode, weighted=case["weigh_by_local_iter"]).reshape(exp.shape)
        assert got.dtype == exp.dtype, (key, got.dtype, exp.dtype)
        assert same_bits(got, exp), f"{case['name']}:{key}"


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_python_restatements_match_reference(case, oracle):
    for key, (rows, ws) in per_key_sequences(case, ARRAYS).items():
        exp = ARRAYS[case["expected"][key]]
        if case["container"] == "numpy":
            got = np.asarray(oracle.numpy_mode_reference([r.copy() for r in rows], ws, weighted=case["weigh_by_local_iter"]))
        else:
            got = oracle.torch_mode_reference([torch.from_numpy(r.copy()) for r in rows], ws, weighted=case["weigh_by_local_iter"]).numpy()
        assert same_bits(got.reshape(exp.shape), exp), f"{case['name']}:{key}"


def test_oracle_threads_do_not_change_bits(oracle):
    rng = np.random.default_rng(1)
    rows = [rng.standard_normal(100_003).astype(np.float32) for _ in range(9)]
    ws = [float(1 + (37 * k) % 100) for k in range(9)]
    for mode in (oracle.MODE_NUMPY, oracle.MODE_TORCH):
        a = oracle.fedavg_c(rows, ws, mode, nthreads=1)
        b = oracle.fedavg_c(rows, ws, mode, nthreads=4)
        assert same_bits(a, b)


def test_oracle_chunked_accumulate_is_bitwise(oracle):
    """Folding the arrival sequence in chunks through acc_in gives the same bits (the device engine relies on it)."""
    rng = np.random.default_rng(2)
    rows = [rng.standard_normal(4096).astype(np.float32) for _ in range(10)]
    ws = [0.3 + k for k in range(10)]
    for mode in (oracle.MODE_NUMPY, oracle.MODE_TORCH):
        full = oracle.fedavg_c(rows, ws, mode)
        part = oracle.fedavg_c(rows[:4], ws[:4], mode, fin=oracle.FIN_NONE)
        rest = oracle.fedavg_c(rows[4:], ws[4:], mode, acc_in=part, count=sum_in_order(ws))
        assert same_bits(full, rest)


def sum_in_order(ws):
    c = None
    for w in ws:
        c = w if c is None else c + w
    return c


def test_synth_generator_is_deterministic(oracle):
    cols = np.arange(0, 1_000_000, 997, dtype=np.uint64)
    a = oracle.synth_values(7, 3, cols)
    b = oracle.synth_values(7, 3, cols)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    full = oracle.synth_values(7, 3, np.arange(200_000, dtype=np.uint64))
    assert abs(float(full.mean())) < 0.02 and abs(float(full.std()) - 1.0) < 0.02
