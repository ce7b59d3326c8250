"""Which fp32 sqrt the reference's server optimizer computes -- torch CPU's on this host.

The FedOpt server step (nvflare/app_opt/pt/fedopt.py:157-182) calls torch's single-tensor optimizers, whose
``exp_avg_sq.sqrt()`` (torch/optim/adam.py:545; NAdam, RAdam, RMSprop, Adagrad alike) is torch CPU's unary sqrt
kernel.  torch 2.10 with MKL computes it with MKL VML vsSqrt (ATen vml.h, IMPLEMENT_VML_MKL(sqrt, Sqrt)), which
on the AVX-512 path is NOT the correctly rounded vsqrtps: it is one Newton step from the VRSQRT14PS estimate
(tools/sqrt_probe.c; ~0.5 % of results 1 ulp low).  The device epilogue reproduces either:

* ``"torch_cpu"`` -- the restated vsSqrt (fedavg_arith.h ``sqrt_torch_cpu``) with the estimate table captured where
  the golden FedOpt fixtures were generated (``data/rsqrt14_avx512.bin``, 2 x 2^15 estimates), which the kernel
  evaluates as 64 exact line segments (fedavg_rsqrt14.h, tools/make_rsqrt14_segments.py);
* ``"ieee"`` -- the correctly rounded sqrt (torch builds / CPUs whose vsSqrt rounds correctly).

``mode()`` follows ``$NVFLARE_AMD_TORCH_SQRT`` (``torch_cpu`` | ``ieee`` | ``auto``, the default): ``auto`` asks this
host's torch for the sqrt of ``data/sqrt_vectors.npz``'s probe values (8407 inputs, 6400 of them where the two
differ) and picks the one it matches bit for bit, ``ieee`` when it matches neither (then the FedOpt parameters
carry the documented sqrt bound)."""

from __future__ import annotations

import os
import threading
from typing import Optional

import numpy as np

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
TABLE_FILE = os.path.join(DATA, "rsqrt14_avx512.bin")
VECTORS_FILE = os.path.join(DATA, "sqrt_vectors.npz")
MODES = ("torch_cpu", "ieee")

_lock = threading.RLock()
_detected: Optional[str] = None
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
    """``"torch_cpu"`` if this host's torch.sqrt gives the restated vsSqrt on every probe value, ``"ieee"`` if it
    gives the correctly rounded sqrt on every one, else ``"unmatched"``."""
    global _detected
    with _lock:
        if _detected is None:
            import torch

            v = np.load(VECTORS_FILE, allow_pickle=False)
            got = torch.from_numpy(np.ascontiguousarray(v["x"])).sqrt().numpy().view(np.uint32)
            if np.array_equal(got, v["torch_cpu"].view(np.uint32)):
                _detected = "torch_cpu"
            elif np.array_equal(got, v["ieee"].view(np.uint32)):
                _detected = "ieee"
            else:
                _detected = "unmatched"
        return _detected


def mode() -> str:
    """The sqrt the device server optimizer reproduces (module docstring)."""
    env = os.environ.get("NVFLARE_AMD_TORCH_SQRT", "auto").strip().lower()
    if env in MODES:
        return env
    if env != "auto":
        raise ValueError(f"NVFLARE_AMD_TORCH_SQRT={env!r}: expected torch_cpu, ieee or auto")
    d = detect()
    return d if d in MODES else "ieee"


def epilogue_flag(sqrt_mode: Optional[str] = None) -> int:
    """``fedavg_epilogue.torch_sqrt`` for a step: 1 in ``torch_cpu`` mode, else 0 (the correctly rounded sqrt)."""
    m = sqrt_mode or mode()
    if m not in MODES:
        raise ValueError(f"sqrt mode {m!r}: expected one of {MODES}")
    return int(m == "torch_cpu")
