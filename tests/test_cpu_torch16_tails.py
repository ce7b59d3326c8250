"""nvflare_amd/torch16.py (which elements of a 16-bit torch add_ run through torch's scalar loop) against torch
CPU itself: the oracle's two-loop restatement with the product's element list must equal torch's own
``T.add_(v, alpha=w)`` bit for bit, for sizes below and above the 32768-element grain and 1-8 threads; the
oracle's own partition (oracle/fedavg_oracle.py torch16_scalar_mask) must agree with the product's."""

import numpy as np
import pytest
import torch

from nvflare_amd import torch16
from oracle import fedavg_oracle as orc

SIZES = [1, 5, 31, 32, 33, 1031, 32767, 32768, 32769, 40000, 65536 + 17, 100003, 2359296 + 7]


@pytest.mark.parametrize("dt,fmt", [(torch.float16, "float16"), (torch.bfloat16, "bfloat16")])
@pytest.mark.parametrize("threads", [1, 2, 3, 8])
def test_scalar_elements_match_torch(dt, fmt, threads):
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rng = np.random.default_rng(threads)
        for n in SIZES:
            T = torch.from_numpy((rng.standard_normal(n) * 50).astype(np.float32)).to(dt)
            V = torch.from_numpy((rng.standard_normal(n) * 50).astype(np.float32)).to(dt)
            w = float(rng.random() * 9 + 0.1)
            got = T.clone().add_(V, alpha=w).float().numpy()
            idx = torch16.scalar_tail_indices([(0, n)], torch16.torch_threads(), torch16.vector_block())
            mask = np.zeros(n, bool)
            mask[idx] = True
            assert np.array_equal(mask, orc.torch16_scalar_mask(n, threads)), (n, threads)
            a = orc.round16(np.float32(w), fmt)
            t, v = T.float().numpy(), V.float().numpy()
            vec = orc.round16((v.astype(np.float64) * np.float64(a) + t.astype(np.float64)).astype(np.float32), fmt)
            sc = orc.round16(t + orc.round16(v * np.float32(a), fmt), fmt)
            assert np.array_equal(np.where(mask, sc, vec), got), (fmt, n, threads)
    finally:
        torch.set_num_threads(old)


def test_keys_at_offsets_and_build_without_vectors(monkeypatch):
    idx = torch16.scalar_tail_indices([(0, 40), (48, 64), (112, 70001)], 1, 32)
    assert idx.tolist()[:8] == [32, 33, 34, 35, 36, 37, 38, 39]
    assert (112 + 70001 - 70001 % 32) in idx and 48 + 63 not in idx
    monkeypatch.setenv("NVFLARE_AMD_TORCH16_VEC_BLOCK", "0")
    assert torch16.vector_block() == 0
    assert torch16.scalar_tail_indices([(8, 5)], 1, 0).tolist() == [8, 9, 10, 11, 12]


def test_rocm_f16_unrolled_elements():
    """torch-ROCm's float16 add_: the last partial 2048-element block (all of a smaller tensor) is unrolled."""
    assert torch16.rocm_f16_unrolled_indices([(0, 1500)]).tolist() == list(range(1500))
    assert torch16.rocm_f16_unrolled_indices([(0, 2048)]).size == 0
    assert torch16.rocm_f16_unrolled_indices([(16, 3072)]).tolist() == list(range(16 + 2048, 16 + 3072))
    # a bucket [4096, 6149) of a 6149-element tensor: only the whole tensor's tail 6144.. is unrolled
    assert torch16.rocm_f16_unrolled_indices([(0, 2053, 4096, 6149)]).tolist() == list(range(2048, 2053))
