"""Which fp32 sqrt the reference's server optimizer computes -- torch CPU's on this host.

The FedOpt server step (nvflare/app_opt/pt/fedopt.py:157-182) calls torch's single-tensor optimizers, whose
``exp_avg_sq.sqrt()`` (torch/optim/adam.py:545; NAdam, RAdam, RMSprop, Adagrad alike) is torch CPU's unary sqrt
kernel.  torch 2.10 with MKL computes it with MKL VML vsSqrt (ATen vml.h, IMPLEMENT_VML_MKL(sqrt, Sqrt)), which is
NOT the correctly rounded sqrt, and MKL picks its code path by CPU.  The device epilogue reproduces:

* ``"torch_cpu"`` -- the AVX-512 path (Intel hosts; where the golden FedOpt fixtures were generated): one Newton step
  from the VRSQRT14PS estimate (tools/sqrt_probe.c; ~0.5 % of results 1 ulp low), restated in fedavg_arith.h
  ``sqrt_torch_cpu`` with the captured estimate table (``data/rsqrt14_avx512.bin``, 2 x 2^15 estimates) evaluated as
  64 exact line segments (fedavg_rsqrt14.h, tools/make_rsqrt14_segments.py);
* ``"torch_cpu_amd"`` -- the SSE4.2 / AVX path MKL runs on the GPU pool's AMD EPYC hosts: a coupled Newton step in
  plain fp32 from that CPU's RSQRTPS estimate (~16 % of results +-1 ulp), restated in fedavg_arith.h
  ``sqrt_mkl_rsqrtps`` with the estimate table captured on the box (``data/rsqrtps_amd.bin``, 2 x 4096 estimates,
  tools/rsqrtps_dump.c); the sequence equals MKL's own kernel on all 2^32 inputs with this container's RSQRTPS and
  the box's torch.sqrt on every fp32 in [1, 4) with the AMD table (tools/sqrt_mkl_sse_check.py);
* ``"ieee"`` -- the correctly rounded sqrt (torch builds / CPUs whose vsSqrt rounds correctly).

``mode()`` follows ``$NVFLARE_AMD_TORCH_SQRT`` (``torch_cpu`` | ``torch_cpu_amd`` | ``ieee`` | ``auto``, the default):
``auto`` asks this host's torch for the sqrt of ``data/sqrt_vectors.npz``'s probe values (6400 inputs where the AVX-512
path and the correctly rounded sqrt differ, 3072 where the AMD path differs from both, and inputs where they agree)
and picks the one it matches bit for bit, ``ieee`` when it matches none (then the FedOpt parameters carry the
documented sqrt bound)."""

from __future__ import annotations

import logging
import os
import threading
from typing import Optional

import numpy as np

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
TABLE_FILE = os.path.join(DATA, "rsqrt14_avx512.bin")
VECTORS_FILE = os.path.join(DATA, "sqrt_vectors.npz")
MODES = ("torch_cpu", "torch_cpu_amd", "ieee")

_lock = threading.RLock()
_detected: Optional[str] = None
_warned = False
_table: Optional[np.ndarray] = None


def table() -> np.ndarray:
    """The estimate table as the kernel indexes it: 65536 uint16, mantissa bits 22..7 of VRSQRT14PS for x in
    [1, 2) then [2, 4) at the top-15-bit mantissas (every raw entry has exponent 126 and 7 clear low bits)."""
    global _table
    with _lock:
        if _table is None:
            raw = np.fromfile(TABLE_FILE, dtype=np.uint32)
            if raw.size != 65536 or np.any((raw >> 23) != 126) or np.any(raw & 0x7F):
                raise ValueError(f"{TABLE_FILE}: not a VRSQRT14 estimate table")
            _table = np.ascontiguousarray(((raw >> 7) & 0xFFFF).astype(np.uint16))
        return _table


def detect() -> str:
    """The mode (``MODES``) whose results this host's torch.sqrt gives on every probe value, else ``"unmatched"``."""
    global _detected
    with _lock:
        if _detected is None:
            import torch

            v = np.load(VECTORS_FILE, allow_pickle=False)
            got = torch.from_numpy(np.ascontiguousarray(v["x"])).sqrt().numpy().view(np.uint32)
            _detected = next((m for m in MODES if np.array_equal(got, v[m].view(np.uint32))), "unmatched")
        return _detected


def mode() -> str:
    """The sqrt the device server optimizer reproduces (module docstring)."""
    env = os.environ.get("NVFLARE_AMD_TORCH_SQRT", "auto").strip().lower()
    if env in MODES:
        return env
    if env != "auto":
        raise ValueError(f"NVFLARE_AMD_TORCH_SQRT={env!r}: expected torch_cpu, torch_cpu_amd, ieee or auto")
    d = detect()
    if d in MODES:
        return d
    global _warned
    with _lock:
        if not _warned:
            _warned = True
            logging.getLogger(__name__).warning(
                "torch CPU's sqrt on this host matches none of the restated paths (%s); the device server optimizer "
                "uses the correctly rounded sqrt, so Adam-family parameters can differ from torch's by a few ulp "
                "(capture this CPU's RSQRTPS with tools/rsqrtps_dump.c to add its path)", ", ".join(MODES[:-1]))
    return "ieee"


def epilogue_flag(sqrt_mode: Optional[str] = None) -> int:
    """``fedavg_epilogue.torch_sqrt`` (FEDAVG_SQRT_*) for a step in the given (default: this host's) mode."""
    from nvflare_amd import _native as N

    m = sqrt_mode or mode()
    if m not in MODES:
        raise ValueError(f"sqrt mode {m!r}: expected one of {MODES}")
    return {"torch_cpu": N.FEDAVG_SQRT_TORCH_AVX512, "torch_cpu_amd": N.FEDAVG_SQRT_TORCH_AMD,
            "ieee": N.FEDAVG_SQRT_IEEE}[m]
