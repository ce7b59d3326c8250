"""Dequantisation: oracle pinning and the filter's host logic.

* adaquant: the C restatement (oracle_dequantize) is pinned bit-for-bit to AdaQuantizer round trips run by
  the reference itself (tests/golden/quant_cases.*, ada_quant.py:39-87, dequantizer.py:146-160);
* float16: pinned to numpy's own fp16 -> fp32 widening over all 65536 bit patterns (dequantizer.py:98-100,
  :168-170 is exactly ``astype(np.float32)``);
* blockwise8 / float4 / normfloat4: bitsandbytes (setup.cfg:74, unpinned) is not installed -- "parity
  unpinned"; the restatement is cross-checked against an independent numpy formulation of bitsandbytes'
  published kernels (General8bit lookup x absmax, dDequantizeFP4Tree, dDequantizeNF4)."""

import bz2

import numpy as np
import pytest

from golden_util import adaquant_state, load_quant_golden, same_bits
from nvflare_amd import _native as N
from nvflare_amd.app_opt.pt.quantization import ModelDequantizer
from nvflare_amd.compat import DXO, DataKind, FLContext, MetaKey
from nvflare_amd.quantized import QuantizedPayload

QM, QA = load_quant_golden()


@pytest.mark.parametrize("case", QM["cases"], ids=lambda c: c["name"])
def test_oracle_adaquant_matches_reference(oracle, case):
    st = adaquant_state(case, QA)
    n = int(np.prod(st["tensor_shape"]))
    if "norm" not in st:
        out = oracle.dequantize(oracle.Q_ADA_U8, np.zeros(1, np.uint8), n, offset=st["offset"], has_norm=False)
    else:
        if "compressed_tensor" in st:
            q = np.frombuffer(bz2.decompress(st["compressed_tensor"].tobytes()), dtype=np.dtype(st["new_dtype"]))
        else:
            q = QA[case["quantized"]]
        qt = oracle.Q_ADA_U8 if q.dtype.itemsize == 1 else oracle.Q_ADA_U16
        out = oracle.dequantize(qt, q, n, norm=st["norm"], level=st["quantization_level"], offset=st["offset"])
    assert same_bits(out.reshape(st["tensor_shape"]), QA[case["expected"]])


def test_oracle_fp16_all_patterns(oracle):
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    assert same_bits(oracle.dequantize(oracle.Q_F16, h, h.size), h.view(np.float16).astype(np.float32))


def test_oracle_bf16(oracle):
    h = np.arange(0, 65536, 7, dtype=np.uint32).astype(np.uint16)
    ref = (h.astype(np.uint32) << 16).view(np.float32)
    assert same_bits(oracle.dequantize(oracle.Q_BF16, h, h.size), ref)


NF4 = np.array([-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453, -0.28444138169288635,
                -0.18477343022823334, -0.09105003625154495, 0.0, 0.07958029955625534, 0.16093020141124725,
                0.24611230194568634, 0.33791524171829224, 0.44070982933044434, 0.5626170039176941,
                0.7229568362236023, 1.0], np.float32)
FP4 = np.array([0.0, 5.208333333e-03, 0.66666667, 1.0, 0.33333333, 0.5, 0.16666667, 0.25], np.float32)


def _nibbles(packed, n):
    hi, lo = packed >> 4, packed & 15
    return np.stack([hi, lo], axis=1).reshape(-1)[:n]


@pytest.mark.parametrize("n,bs", [(4099, 64), (8192, 128), (1, 64), (130, 4)])
def test_oracle_4bit_and_blockwise8_vs_numpy_formula(oracle, n, bs):
    rng = np.random.default_rng(n)
    nb = (n + bs - 1) // bs
    absmax = (rng.random(nb) * 3).astype(np.float32)
    absmax[0] = 0.0
    packed = rng.integers(0, 256, (n + 1) // 2).astype(np.uint8)
    nib = _nibbles(packed, n)
    am = absmax[np.arange(n) // bs]
    nf4 = NF4[nib] * am
    sign = np.where(nib & 8, np.float32(-1), np.float32(1))
    fp4 = (FP4[nib & 7] * am) * sign
    assert same_bits(oracle.dequantize(oracle.Q_NF4, packed, n, absmax=absmax, blocksize=bs), nf4)
    assert same_bits(oracle.dequantize(oracle.Q_FP4, packed, n, absmax=absmax, blocksize=bs), fp4)
    code = np.sort(rng.standard_normal(256)).astype(np.float32)
    q8 = rng.integers(0, 256, n).astype(np.uint8)
    b8 = code[q8] * am
    assert same_bits(oracle.dequantize(oracle.Q_BLOCKWISE8, q8, n, absmax=absmax, code=code, blocksize=bs), b8)


def _dxo(qtype, params, qstate, srcdt):
    return DXO(DataKind.WEIGHT_DIFF, data=params,
               meta={MetaKey.PROCESSED_ALGORITHM: qtype, "quant_state": qstate, "source_datatype": srcdt,
                     "quantized_flag": True})


def test_lazy_filter_builds_payloads_and_strips_meta():
    import torch

    f = ModelDequantizer(lazy=True)
    rng = np.random.default_rng(0)
    w16 = rng.standard_normal(100).astype(np.float16)
    params = {"a": w16.copy(), "b": torch.from_numpy(w16.copy()), "flag": np.array([True]), "h": w16.copy()}
    dxo = _dxo("float16", params, {"a": {}, "b": {}, "flag": {}, "h": {}},
               {"a": "float32", "b": "float32", "flag": "bool", "h": "float16"})
    out = f.process_dxo(dxo, dxo.to_shareable(), FLContext())
    assert isinstance(out.data["a"], QuantizedPayload) and out.data["a"].container == "numpy"
    assert isinstance(out.data["b"], QuantizedPayload) and out.data["b"].container == "torch"
    assert out.data["a"].qtype == N.FEDAVG_Q_F16 and out.data["a"].shape == (100,)
    assert out.data["flag"] is params["flag"]          # bool: skipped (dequantizer.py:58-59)
    assert out.data["h"].dtype == np.float16           # 16-bit quantization of a 16-bit source: skipped
    for k in (MetaKey.PROCESSED_ALGORITHM, "quant_state", "source_datatype", "quantized_flag"):
        assert k not in out.meta


def test_lazy_filter_formats():
    f = ModelDequantizer(lazy=True)
    rng = np.random.default_rng(1)
    n = 1000
    q4 = rng.integers(0, 256, (n // 2, 1)).astype(np.uint8)
    st4 = {"absmax": rng.random(16).astype(np.float32), "blocksize": 64, "quant_map": NF4, "dtype": "float32",
           "shape": [10, 100], "quant_type": "nf4"}
    dxo = _dxo("normfloat4", {"w": q4}, {"w": st4}, {"w": "float32"})
    p = f.process_dxo(dxo, dxo.to_shareable(), FLContext()).data["w"]
    assert p.qtype == N.FEDAVG_Q_NF4 and p.shape == (10, 100) and p.blocksize == 64 and p.nbytes == n // 2
    q8 = rng.integers(0, 256, (10, 100)).astype(np.uint8)
    dxo = _dxo("blockwise8", {"w": q8}, {"w": {"absmax": rng.random(1).astype(np.float32),
                                               "code": np.linspace(-1, 1, 256, dtype=np.float32)}}, {"w": "float32"})
    p = f.process_dxo(dxo, dxo.to_shareable(), FLContext()).data["w"]
    assert p.qtype == N.FEDAVG_Q_BLOCKWISE8 and p.blocksize == 4096 and p.shape == (10, 100)
    with pytest.raises(ValueError):
        f.process_dxo(_dxo("int3", {"w": q8}, {"w": {}}, {"w": "float32"}), None, FLContext())


def test_payload_validation():
    with pytest.raises(ValueError):
        QuantizedPayload(N.FEDAVG_Q_BLOCKWISE8, np.zeros(10, np.uint8), (10,), "numpy", absmax=np.ones(1, np.float32),
                         blocksize=4096)  # no code
    with pytest.raises(ValueError):
        QuantizedPayload(N.FEDAVG_Q_NF4, np.zeros(2, np.uint8), (10,), "numpy", absmax=np.ones(1, np.float32),
                         blocksize=64)  # payload too short
    with pytest.raises(ValueError):
        QuantizedPayload(N.FEDAVG_Q_FP4, np.zeros(5, np.uint8), (10,), "numpy", absmax=np.ones(1, np.float32),
                         blocksize=6)  # blocksize not a multiple of 4
