"""Zero-copy ingest (row f2): decoded views equal the reference decoders' copies; lazy refs map in place."""

import io

import numpy as np
import pytest
import torch

from golden_util import same_bits
from nvflare_amd.ingest import MappedTensor, as_mapped, parse_safetensors_header, recompose_npy, recompose_safetensors


def _npy(a):
    s = io.BytesIO()
    np.save(s, a, allow_pickle=False)
    return s.getvalue()


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.float16, np.int64, np.int8, np.uint8, np.bool_])
@pytest.mark.parametrize("shape", [(), (0,), (7,), (3, 5), (2, 3, 4)])
def test_recompose_npy_matches_np_load(dtype, shape):
    rng = np.random.default_rng(0)
    a = (rng.standard_normal(shape) * 10).astype(dtype)
    data = _npy(a)
    got = recompose_npy(data)
    ref = np.load(io.BytesIO(data), allow_pickle=False)
    assert got.dtype == ref.dtype and got.shape == ref.shape
    assert same_bits(got, ref)
    if a.size:
        assert not got.flags.writeable  # a view over the received bytes, not a copy


def test_recompose_npy_fortran_order_and_big_endian():
    a = np.asfortranarray(np.arange(12, dtype=np.float32).reshape(3, 4))
    got = recompose_npy(_npy(a))
    assert np.array_equal(got, a) and got.shape == (3, 4)
    b = np.arange(5, dtype=">f8")
    got = recompose_npy(_npy(b))
    assert got.dtype == np.dtype(">f8") and np.array_equal(got, b)


def test_recompose_safetensors_matches_load():
    from safetensors.torch import load, save

    rng = np.random.default_rng(1)
    ts = {"f32": torch.from_numpy(rng.standard_normal((4, 5)).astype(np.float32)),
          "bf16": torch.from_numpy(rng.standard_normal(33).astype(np.float32)).to(torch.bfloat16),
          "f16": torch.from_numpy(rng.standard_normal(7).astype(np.float16)),
          "i64": torch.arange(9, dtype=torch.int64), "empty": torch.empty(0, 3), "scalar": torch.tensor(2.5)}
    data = save(ts)
    got = recompose_safetensors(data)
    ref = load(data)
    assert set(got) == set(ref)
    for k in ref:
        assert got[k].dtype == ref[k].dtype and got[k].shape == ref[k].shape, k
        assert torch.equal(got[k].view(-1).view(torch.uint8) if got[k].numel() else got[k],
                           ref[k].view(-1).view(torch.uint8) if ref[k].numel() else ref[k]), k


def test_decomposer_dropins_round_trip():
    from nvflare_amd.app_common.decomposers.numpy_decomposers import NumpyArrayDecomposer
    from nvflare_amd.app_opt.pt.decomposers import TensorDecomposer

    a = np.random.default_rng(2).standard_normal((6, 7)).astype(np.float32)
    d = NumpyArrayDecomposer()
    assert same_bits(d.native_recompose(d.native_decompose(a)), a)
    t = torch.from_numpy(a).to(torch.bfloat16)
    td = TensorDecomposer()
    back = td.native_recompose(td.native_decompose(t))
    assert back.dtype == torch.bfloat16 and torch.equal(back, t)


class _LazyRefLike:
    """Same attributes as lazy_tensor_dict.py:60-77's _LazyRef (file_path, key, materialize)."""

    def __init__(self, file_path, key):
        self.file_path = file_path
        self.key = key

    def materialize(self):
        from safetensors import safe_open

        with safe_open(self.file_path, framework="pt") as f:
            return f.get_tensor(self.key)


def test_mapped_tensor_reads_file_bytes(tmp_path):
    from safetensors.torch import save_file

    rng = np.random.default_rng(3)
    ts = {"w": torch.from_numpy(rng.standard_normal((10, 3)).astype(np.float32)),
          "b": torch.from_numpy(rng.standard_normal(5).astype(np.float32)).to(torch.bfloat16)}
    path = str(tmp_path / "c.safetensors")
    save_file(ts, path)
    for k, t in ts.items():
        m = as_mapped(_LazyRefLike(path, k))
        assert isinstance(m, MappedTensor) and m.shape == tuple(t.shape) and m.dtype == t.dtype
        keep, ptr, nbytes = m.host_view()
        raw = keep[1].tobytes()
        assert nbytes == t.numel() * t.element_size()
        assert raw == t.contiguous().view(torch.uint8).numpy().tobytes()
        assert torch.equal(m.materialize(), t)
    assert as_mapped(_LazyRefLike(str(tmp_path / "missing.safetensors"), "w")) is None
    assert as_mapped(object()) is None
    with open(path, "rb") as f:
        start, header = parse_safetensors_header(f.read())
    assert set(header) == {"w", "b"} and start > 8
