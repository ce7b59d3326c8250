"""Which fp32 sqrt the reference's server optimizer computes -- torch CPU's on this host.

The FedOpt server step (nvflare/app_opt/pt/fedopt.py:157-182) calls torch's single-tensor optimizers, whose
``exp_avg_sq.sqrt()`` (torch/optim/adam.py:545; NAdam, RAdam, RMSprop, Adagrad alike) is torch CPU's unary sqrt
kernel.  torch 2.10 with MKL computes it with MKL VML vsSqrt (ATen vml.h, IMPLEMENT_VML_MKL(sqrt, Sqrt)), which is
NOT the correctly rounded sqrt, and MKL picks its code path by CPU.  The device epilogue reproduces:

* ``"torch_cpu"`` -- the AVX-512 path (Intel hosts; where the golden FedOpt fixtures were generated): one Newton step
  from the VRSQRT14PS estimate (tools/sqrt_probe.c; ~0.5 % of results 1 ulp low), restated in fedavg_arith.h
  ``sqrt_torch_cpu`` with the captured estimate table (``data/rsqrt14_avx512.bin``, 2 x 2^15 estimates) evaluated as
  64 exact line segments (fedavg_rsqrt14.h, tools/make_rsqrt14_segments.py);
* ``"torch_cpu_amd"`` -- the SSE4.2 / AVX path MKL runs on the GPU pool's AMD EPYC hosts (and on any CPU where MKL takes
  it): a coupled Newton step in plain fp32 from the CPU's RSQRTPS estimate (~16 % of results +-1 ulp), restated in
  fedavg_arith.h ``sqrt_mkl_rsqrtps``.  RSQRTPS is vendor-specific, so the estimate table is THIS host's, captured at
  run time (``host_rsqrtps_table``: the C-ABI's fedavg_host_rsqrtps_table over every fp32 of [1, 4)) and uploaded to
  each device context (DeviceContext.load_rsqrtps); the sequence equals MKL's own kernel on all 2^32 inputs with this
  container's RSQRTPS and the box's torch.sqrt on all 2^32 inputs with the box's (tools/sqrt_mkl_sse_check.py,
  profiles/r03/final/sqrt_check_torch_all.log; that table is the fixture tests/golden/rsqrtps_amd_epyc9575f.bin);
* ``"ieee"`` -- the correctly rounded sqrt (torch builds / CPUs whose vsSqrt rounds correctly).

``mode()`` follows ``$NVFLARE_AMD_TORCH_SQRT`` (``torch_cpu`` | ``torch_cpu_amd`` | ``ieee`` | ``auto``, the default):
``auto`` asks this host's torch for the sqrt of ``data/sqrt_vectors.npz``'s probe values (6400 inputs where the AVX-512
path and the correctly rounded sqrt differ, 3072 where the box's SSE path differs from both, and inputs where they
agree) plus 65,536 seeded positive normals, and picks the one it matches bit for bit: the AVX-512 and correctly rounded
candidates from the stored results, the SSE candidate recomputed with this host's RSQRTPS (``sqrt_sse_restated``);
``ieee`` when it matches none (then the FedOpt parameters carry the documented sqrt bound)."""

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
_rsqrtps: Optional[np.ndarray] = None


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


def host_rsqrtps_table() -> np.ndarray:
    """THIS CPU's RSQRTPS estimates as the device indexes them (8192 uint16: mantissa bits 22..11 for x in [1, 2)
    then [2, 4), one per top-12-bit mantissa), captured by the C-ABI (fedavg_host_rsqrtps_table, no device needed);
    raises FedAvgError when the CPU's estimate does not have that shape."""
    global _rsqrtps
    with _lock:
        if _rsqrtps is None:
            import ctypes

            from . import _native as N

            t = np.zeros(8192, dtype=np.uint16)
            N.call("fedavg_host_rsqrtps_table", ctypes.c_void_p(t.ctypes.data), ctypes.c_size_t(t.size))
            t.flags.writeable = False
            _rsqrtps = t
        return _rsqrtps


def sqrt_sse_restated(x: np.ndarray, table: np.ndarray) -> np.ndarray:
    """MKL vsSqrt's SSE4.2 / AVX kernel with RSQRTPS ``table`` (fedavg_arith.h sqrt_mkl_rsqrtps), for detection: every
    operation a separately rounded fp32 numpy operation, as the kernel's plain SSE arithmetic; zero, subnormals, the
    top 4095 finite values, inf, NaN and negatives take the correctly rounded callout."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    b = x.view(np.uint32)
    inside = (b >= 0x00800000) & (b <= 0x7F7FF000)
    e = (b >> 23).astype(np.int64) - 127
    p = e & 1
    k = (e - p) // 2
    t = table.astype(np.uint32)[(p.astype(np.uint32) << 12) | ((b & 0x7FFFFF) >> 11)]
    yb = ((0x3F000000 | (t << 11)).astype(np.int64) - k * 8388608).astype(np.uint32)
    y = np.where(inside, yb, np.uint32(0x3F800000)).view(np.float32)
    half = np.float32(0.5)
    with np.errstate(all="ignore"):
        s_ = x * y
        h = y * half
        r = half - s_ * h
        s1 = s_ * r + s_
        h1 = h * r + h
        res = (x - s1 * s1) * h1 + s1
        return np.where(inside, res, np.sqrt(x)).astype(np.float32)


def _probe_values():
    v = np.load(VECTORS_FILE, allow_pickle=False)
    rng = np.random.default_rng(20261017)
    extra = rng.integers(0x00800000, 0x7F7FF001, 65536, dtype=np.uint32).view(np.float32)
    return v, extra


def detect(host_sqrt=None) -> str:
    """The mode (``MODES``) whose results this host's torch.sqrt gives on every probe value, else ``"unmatched"``.
    ``host_sqrt``: the fp32 sqrt to identify in place of torch CPU's (a test hook; the result is then not cached)."""
    global _detected
    with _lock:
        custom = host_sqrt is not None
        if _detected is not None and not custom:
            return _detected
        if not custom:
            import torch

            def host_sqrt(a):
                return torch.from_numpy(np.ascontiguousarray(a)).sqrt().numpy()

        v, extra = _probe_values()
        x = np.ascontiguousarray(v["x"])
        got = np.asarray(host_sqrt(x), dtype=np.float32).view(np.uint32)
        found = "unmatched"
        for m in ("torch_cpu", "ieee"):
            if np.array_equal(got, v[m].view(np.uint32)):
                found = m
                break
        else:
            try:
                tab = host_rsqrtps_table()
            except Exception as e:  # noqa: BLE001 - a CPU whose RSQRTPS the device cannot restate: no SSE candidate
                logging.getLogger(__name__).info("no RSQRTPS table for this CPU (%s)", e)
                tab = None
            if tab is not None and np.array_equal(got, sqrt_sse_restated(x, tab).view(np.uint32)):
                got_x = np.asarray(host_sqrt(extra), dtype=np.float32).view(np.uint32)
                if np.array_equal(got_x, sqrt_sse_restated(extra, tab).view(np.uint32)):
                    found = "torch_cpu_amd"
        if not custom:
            _detected = found
        return found


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
                "(neither MKL's AVX-512 path nor its SSE path with this CPU's RSQRTPS)", ", ".join(MODES[:-1]))
    return "ieee"


def epilogue_flag(sqrt_mode: Optional[str] = None) -> int:
    """``fedavg_epilogue.torch_sqrt`` (FEDAVG_SQRT_*) for a step in the given (default: this host's) mode."""
    from nvflare_amd import _native as N

    m = sqrt_mode or mode()
    if m not in MODES:
        raise ValueError(f"sqrt mode {m!r}: expected one of {MODES}")
    return {"torch_cpu": N.FEDAVG_SQRT_TORCH_AVX512, "torch_cpu_amd": N.FEDAVG_SQRT_TORCH_AMD,
            "ieee": N.FEDAVG_SQRT_IEEE}[m]
