"""Which elements of a float16 / bfloat16 torch total take torch CPU's scalar step.

The reference adds a client's 16-bit tensor with ``T.add_(v, alpha=w)`` (weighted_aggregation_helper.py:207).
torch runs that on the CPU through TensorIterator (third-party, torch 2.x):

* ``TensorIteratorBase::for_each``: a tensor of fewer than ``at::internal::GRAIN_SIZE`` (32768) elements, or a
  single-thread process, is one range ``[0, n)``; otherwise ``at::parallel_for`` (``ATen/ParallelOpenMP.h``)
  splits it over ``min(threads, ceil(n / 32768))`` threads into ranges of ``ceil(n / threads')`` elements;
* every range goes through ``cpu_kernel_vec``'s ``vectorized_loop`` (``ATen/native/cpu/Loops.h``): blocks of
  two vectors (32 half-precision elements on the AVX2 and AVX512 builds) with one fp32 fma each, then the
  remaining ``len % 32`` elements through the scalar loop, whose ``c10::Half`` / ``c10::BFloat16`` operators
  round the product and the sum separately.  A build without vector kernels (``DEFAULT`` capability) runs
  every element through the scalar loop.

The engine hands the resulting element lists to ``fedavg_accumulate_tiled16_tails`` so that the device
reproduces both steps where torch uses them (checked against torch itself for sizes up to 2.4 M elements and
1-16 threads: tests/test_cpu_torch16_tails.py)."""

from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np

GRAIN_SIZE = 32768  # at::internal::GRAIN_SIZE
_VEC_BLOCK = 32  # 2 * Vectorized<c10::Half>::size() on the AVX2 / AVX512 builds (measured, see module doc)


def vector_block() -> int:
    """Elements per vectorised block of the running torch build (0: no vector loop, every element scalar).
    ``NVFLARE_AMD_TORCH16_VEC_BLOCK`` overrides it."""
    env = os.environ.get("NVFLARE_AMD_TORCH16_VEC_BLOCK")
    if env:
        return int(env)
    import torch

    return 0 if torch.backends.cpu.get_cpu_capability() == "DEFAULT" else _VEC_BLOCK


def torch_threads() -> int:
    import torch

    return max(1, int(torch.get_num_threads()))


def thread_ranges(n: int, threads: int) -> List[Tuple[int, int]]:
    """The element ranges at::parallel_for gives the threads of one contiguous n-element add_."""
    if n < GRAIN_SIZE or threads <= 1:
        return [(0, n)] if n > 0 else []
    nt = min(threads, -(-n // GRAIN_SIZE))
    chunk = -(-n // nt)
    return [(b, min(b + chunk, n)) for b in range(0, n, chunk)]


def scalar_ranges(n: int, threads: int, block: int) -> List[Tuple[int, int]]:
    """[start, end) element ranges of an n-element tensor that torch adds with its scalar loop."""
    out = []
    for b, e in thread_ranges(n, threads):
        s = b if block <= 0 else b + (e - b) // block * block
        if s < e:
            out.append((s, e))
    return out


def scalar_tail_indices(keys: Sequence[Tuple[int, ...]], threads: int, block: int) -> np.ndarray:
    """Sorted flat indices of the elements torch's scalar loop adds, over keys given as (flat offset, n) -- a
    whole tensor -- or (flat offset, n, lo, n_whole): elements [lo, lo + n) of an n_whole-element tensor (a
    parameter bucket; the loops run over the whole tensor)."""
    parts = []
    for key in keys:
        off, n = int(key[0]), int(key[1])
        lo, whole = (int(key[2]), int(key[3])) if len(key) > 2 else (0, n)
        for s, e in scalar_ranges(whole, threads, block):
            s, e = max(s, lo), min(e, lo + n)
            if s < e:
                parts.append(np.arange(off + s - lo, off + e - lo, dtype=np.int64))
    if not parts:
        return np.empty(0, dtype=np.int64)
    idx = np.concatenate(parts)
    idx.sort()
    return idx


# torch-ROCm (device-resident float16 tensors): its vectorized elementwise kernel gives every block of 256
# threads x 8 halves (16-byte vectors) = 2048 elements; blocks run the vector path (fp32 fma, then fp16: two
# roundings, like the CPU vector loop), the last partial block runs the unrolled path, where the compiler fuses
# the fma and the fp16 conversion (v_fma_mixlo_f16: one rounding).  Measured on MI355X with torch 2.10+rocm7.0
# (tools/debug_fp16_device.py): 1500 / 2047 elements all single-rounded, 2048 / 4096 / 10240 all double,
# 3072: elements 2048.. single.  Assumes 16-byte aligned tensors (torch's fresh allocations; a misaligned
# client tensor would take narrower vectors).  bfloat16 has no fused path: both round twice.
ROCM_F16_BLOCK = int(os.environ.get("NVFLARE_AMD_ROCM_F16_BLOCK", "2048"))


def rocm_f16_unrolled_indices(keys: Sequence[Tuple[int, ...]], block: int = 0) -> np.ndarray:
    """Sorted flat indices of the float16 elements torch-ROCm's add_ runs through its unrolled path, over keys
    given as (flat offset, n[, lo, n_whole]) like scalar_tail_indices."""
    block = block or ROCM_F16_BLOCK
    parts = []
    for key in keys:
        off, n = int(key[0]), int(key[1])
        lo, whole = (int(key[2]), int(key[3])) if len(key) > 2 else (0, n)
        s, e = max(whole - whole % block, lo), min(whole, lo + n)
        if s < e:
            parts.append(np.arange(off + s - lo, off + e - lo, dtype=np.int64))
    if not parts:
        return np.empty(0, dtype=np.int64)
    idx = np.concatenate(parts)
    idx.sort()
    return idx
