"""Oracle vs the reference on float16 / bfloat16 / integer / bool client arrays (tests/golden/dtype_cases.*,
produced by running weighted_aggregation_helper.py:153-240 itself, make_golden.py --set dtypes).

* numpy containers (float16 and every integer / bool dtype; python-float and numpy-scalar weights): the
  numpy-op restatement is bit-exact everywhere.
* torch integer / bool tensors: the torch-op restatement is bit-exact.
* torch float16 / bfloat16: ``torch16_reference`` (fp32 ops with a 16-bit rounding after each library
  operation on the vectorised elements; on torch's scalar tail -- ``vector_end`` .. n at the one torch thread
  the fixtures were made with -- the add_ product and sum rounded separately) is bit-exact on every element.
  The vector-only restatement stays within ``torch16_tail_tolerance`` on that tail."""

import numpy as np
import pytest
import torch

from golden_util import (
    as_f32_values,
    dtype_case_inputs,
    dtype_case_weights,
    load_dtype_golden,
    same_bits,
    torch16_tail_tolerance,
)
from oracle import fedavg_oracle as orc

META, ARRAYS = load_dtype_golden()
CASES = sorted(META["cases"].items())


@pytest.mark.parametrize("name,case", CASES, ids=[n for n, _ in CASES])
def test_oracle_matches_reference_dtypes(name, case):
    rows = dtype_case_inputs(case, ARRAYS)
    ws = dtype_case_weights(case)
    dt = case["dtype"]
    exp_bits = ARRAYS[case["expected"]]
    if case["container"] == "numpy":
        got = orc.numpy_mode_reference(rows, ws, weighted=case["weighted"])
        assert str(np.asarray(got).dtype) == case["expected_dtype"]
        assert same_bits(np.asarray(got), exp_bits)
        return
    if dt not in ("float16", "bfloat16"):
        got = orc.torch_mode_reference([r.clone() for r in rows], ws, weighted=case["weighted"])
        assert str(got.dtype).replace("torch.", "") == case["expected_dtype"]
        assert same_bits(got.numpy(), exp_bits)
        return
    rows_f32 = [as_f32_values(r, dt) for r in rows]
    exp = as_f32_values(exp_bits, dt)
    ve = case["vector_end"]
    if case["weighted"]:
        assert ve == orc.torch16_scalar_mask(exp.size).argmax() or not orc.torch16_scalar_mask(exp.size).any(), name
    assert same_bits(orc.torch16_reference(rows_f32, ws, dt, weighted=case["weighted"]), exp), name
    got = orc.torch16_vector_reference(rows_f32, ws, dt, weighted=case["weighted"])
    assert same_bits(got[:ve], exp[:ve]), name
    tol = torch16_tail_tolerance([r[ve:] for r in rows_f32], ws, exp[ve:], dt)
    d = np.abs(got[ve:].astype(np.float64) - exp[ve:].astype(np.float64))
    both_nan = np.isnan(got[ve:]) & np.isnan(exp[ve:])
    assert np.all((d <= tol) | both_nan | (got[ve:] == exp[ve:])), name


def test_round16_matches_torch_casts():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.standard_normal(10000).astype(np.float32) * 1000,
                        np.array([0.0, -0.0, np.inf, -np.inf, 65504.0, 65520.0, 65519.0, 1e-8, 6e-8, 3.4e38], np.float32)])
    for fmt, tdt in (("float16", torch.float16), ("bfloat16", torch.bfloat16)):
        exp = torch.from_numpy(x).to(tdt).to(torch.float32).numpy()
        assert same_bits(orc.round16(x, fmt), exp), fmt
