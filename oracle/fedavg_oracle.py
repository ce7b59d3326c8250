"""CPU oracle for the FedAvg weighted-aggregation hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module.  It is the checker, never the thing measured or shipped: ``nvflare_amd`` (the product) never
imports it.

Three restatements of ``WeightedAggregationHelper.add`` / ``get_result``
(``nvflare/app_common/aggregators/weighted_aggregation_helper.py:153-240``), all bit-exact with the
reference on the golden vectors in ``tests/golden/`` (pinned by ``tests/test_oracle_golden.py``):

* ``fedavg_c``            -- plain C restatement (``oracle/fedavg_oracle.c``), element by element in
                             arrival order; optionally multi-threaded over elements (OpenMP).
* ``numpy_mode_reference`` -- the numpy branch as numpy ops (``:188-193``, ``:210-214``, ``:236``).
* ``torch_mode_reference`` -- the torch branch as torch CPU ops (``:181-187``, ``:203-209``, ``:233``).
* ``torch16_vector_reference`` -- the torch branch for float16 / bfloat16 tensors, restated in numpy
                             with explicit roundings: torch CPU's vectorised kernels compute in fp32
                             (mul / div with the scalar as float, add_ as one fp32 fma with alpha cast to
                             the tensor dtype) and round to 16 bits after each op.  Pinned bitwise on the
                             elements torch computes on its vector path (tests/golden/dtype_cases.*).

Plus ``synth_values``: the host twin of the device synthetic-input generator used by ``bench.py`` for
full-size spot checks.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_fedavg.so")
_lib = None

MODE_NUMPY = 0
MODE_TORCH = 1
FIN_NONE = 0
FIN_NUMPY_SCALE = 1
FIN_TORCH_DIV = 2


def build(force: bool = False) -> str:
    """Compile the C restatement with ``oracle/Makefile`` (gcc, -ffp-contract=off)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        for name, ct in (("oracle_fedavg_f32", ctypes.c_float), ("oracle_fedavg_f64", ctypes.c_double)):
            fn = getattr(lib, name)
            fn.restype = None
            fn.argtypes = [
                ctypes.POINTER(ctypes.c_void_p),
                ctypes.c_int,
                ctypes.POINTER(ctypes.c_double),
                ctypes.c_int,
                ctypes.c_int,
                ctypes.c_int,
                ctypes.c_double,
                ctypes.c_void_p,
                ctypes.c_void_p,
                ctypes.c_size_t,
                ctypes.c_int,
            ]
        lib.oracle_synth_value.restype = ctypes.c_float
        lib.oracle_synth_value.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        lib.oracle_synth_fill_f32.restype = None
        lib.oracle_synth_fill_f32.argtypes = [
            ctypes.c_uint64,
            ctypes.c_uint64,
            ctypes.c_void_p,
            ctypes.c_size_t,
            ctypes.c_void_p,
        ]
        _lib = lib
    return _lib


def fedavg_c(
    rows: Sequence[np.ndarray],
    weights: Sequence[float],
    mode: int,
    weighted: bool = True,
    fin: Optional[int] = None,
    count: Optional[float] = None,
    acc_in: Optional[np.ndarray] = None,
    nthreads: int = 1,
) -> np.ndarray:
    """C restatement: weighted arrival-order accumulate, then the mode's finalisation.

    ``rows`` are the client arrays in arrival order (same dtype, float32 or float64, same size).
    ``count`` defaults to the fp64 arrival-order sum of ``weights`` (``weighted_aggregation_helper.py:201,216``).
    ``fin`` defaults to the mode's ``get_result`` step.
    """
    lib = load()
    dtype = np.dtype(rows[0].dtype) if rows else np.dtype(acc_in.dtype)
    if dtype == np.float32:
        fn = lib.oracle_fedavg_f32
    elif dtype == np.float64:
        fn = lib.oracle_fedavg_f64
    else:
        raise TypeError(f"oracle supports float32/float64 rows, got {dtype}")
    rows = [np.ascontiguousarray(r, dtype=dtype).reshape(-1) for r in rows]
    n = rows[0].size if rows else acc_in.size
    for r in rows:
        if r.size != n:
            raise ValueError("all rows must have the same size")
    if count is None:
        count = 0.0
        for i, w in enumerate(weights):
            count = w if i == 0 else count + w
    if fin is None:
        fin = FIN_TORCH_DIV if mode == MODE_TORCH else FIN_NUMPY_SCALE
    K = len(rows)
    ptrs = (ctypes.c_void_p * max(K, 1))(*[r.ctypes.data for r in rows])
    w = (ctypes.c_double * max(K, 1))(*[float(x) for x in weights])
    out = np.empty(n, dtype=dtype)
    acc_ptr = None
    if acc_in is not None:
        acc_in = np.ascontiguousarray(acc_in, dtype=dtype).reshape(-1)
        acc_ptr = acc_in.ctypes.data
    elif K == 0:
        raise ValueError("need at least one row or an acc_in")
    fn(ptrs, K, w, int(mode), int(bool(weighted)), int(fin), float(count), acc_ptr, out.ctypes.data, n, int(nthreads))
    return out


def numpy_mode_reference(rows, weights, weighted: bool = True, count: Optional[float] = None):
    """numpy branch restated with numpy ops (``weighted_aggregation_helper.py:188-193,210-214,236``)."""
    total = None
    c = None
    for v, w in zip(rows, weights):
        if total is None:
            total = v * w if weighted else v.copy()
            c = w
        else:
            total = total + v * w if weighted else total + v
            c = c + w
    if count is not None:
        c = count
    return total * (1.0 / c)


def torch_mode_reference(rows, weights, weighted: bool = True, count: Optional[float] = None):
    """torch branch restated with torch CPU ops (``weighted_aggregation_helper.py:181-187,203-209,233``).

    ``rows`` are CPU torch tensors.  Uses all of torch's intra-op threads (the CPU baseline mode)."""
    total = None
    c = None
    for v, w in zip(rows, weights):
        if total is None:
            total = v.mul(w) if weighted else v.clone()
            c = w
        else:
            if weighted:
                total.add_(v, alpha=w)
            else:
                total.add_(v)
            c = c + w
    if count is not None:
        c = count
    return total.div_(c)


def bf16_round(x) -> np.ndarray:
    """fp32 -> value of the nearest bfloat16, as fp32 (c10::BFloat16 round_to_nearest_even; NaN -> 0x7FC0)."""
    x = np.asarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    r = np.where(np.isnan(x), np.uint32(0x7FC00000), r)
    return r.view(np.float32)


def round16(x, fmt: str) -> np.ndarray:
    """fp32 -> value of the nearest ``fmt`` ("float16" | "bfloat16") number, as fp32 (round to nearest even)."""
    x = np.asarray(x, dtype=np.float32)
    if fmt == "bfloat16":
        return bf16_round(x)
    with np.errstate(over="ignore"):
        return x.astype(np.float16).astype(np.float32)


def bf16_bits_to_f32(bits) -> np.ndarray:
    return (np.asarray(bits, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16_bits(x) -> np.ndarray:
    return (bf16_round(x).view(np.uint32) >> 16).astype(np.uint16)


def torch16_scalar_mask(n: int, threads: int = 1, grain: int = 32768, block: int = 32) -> np.ndarray:
    """Elements of an n-element float16 / bfloat16 ``add_`` that torch CPU runs through its scalar loop
    (third-party torch 2.x, restated): TensorIteratorBase::for_each keeps tensors below ``grain`` (and
    single-thread runs) in one range, else at::parallel_for (ATen/ParallelOpenMP.h) cuts [0, n) into ranges of
    ceil(n / min(threads, ceil(n / grain))) elements; cpu_kernel_vec's vectorized_loop (ATen/native/cpu/Loops.h)
    covers each range in blocks of ``block`` elements (2 vectors; 32 on the AVX2 / AVX512 builds) and leaves
    the last (length mod block) to basic_loop.  block 0: no vector kernel (every element scalar)."""
    mask = np.zeros(n, dtype=bool)
    if n <= 0:
        return mask
    if n < grain or threads <= 1:
        ranges = [(0, n)]
    else:
        nt = min(threads, -(-n // grain))
        chunk = -(-n // nt)
        ranges = [(b, min(b + chunk, n)) for b in range(0, n, chunk)]
    for b, e in ranges:
        mask[(b if block <= 0 else b + (e - b) // block * block):e] = True
    return mask


def torch16_reference(rows, weights, fmt: str, weighted: bool = True, count: Optional[float] = None,
                      threads: int = 1, block: int = 32, mask: Optional[np.ndarray] = None):
    """torch branch for ``fmt`` tensors (weighted_aggregation_helper.py:181-187, :203-209, :233) as torch CPU
    computes it, both loops: ``torch16_vector_reference`` on the vectorised elements, and on the elements of
    ``torch16_scalar_mask`` the scalar loop's c10::Half / c10::BFloat16 add_ step
        T = r(T + r(v * r(float32(w))))        (operator* and operator+ round to the format)
    (mul and div_ compute the same in both loops).  ``mask`` overrides the scalar elements."""
    rows = [np.asarray(v, dtype=np.float32) for v in rows]
    if mask is None:
        mask = torch16_scalar_mask(rows[0].size if rows else 0, threads, block=block)
    with np.errstate(over="ignore", invalid="ignore"):
        total, c = None, None
        for v, w in zip(rows, weights):
            if total is None:
                total = round16(v * np.float32(w), fmt) if weighted else v.copy()
                c = w
            else:
                if weighted:
                    a = round16(np.float32(w), fmt)
                    vec = round16((v.astype(np.float64) * np.float64(a) + total.astype(np.float64)).astype(np.float32),
                                  fmt)
                    sc = round16(total + round16(v * np.float32(a), fmt), fmt)
                    total = np.where(mask, sc, vec)
                else:
                    total = round16(total + v, fmt)
                c = c + w
        if count is not None:
            c = count
        return round16(total / np.float32(c), fmt)


def torch16_vector_reference(rows, weights, fmt: str, weighted: bool = True, count: Optional[float] = None):
    """torch branch for ``fmt`` tensors (weighted_aggregation_helper.py:181-187, :203-209, :233), as torch
    CPU's vectorised kernels compute it.  ``rows``: fp32 arrays holding ``fmt`` values; returns fp32 values
    of the ``fmt`` result.

    first  T = r(v * float32(w))            mul_kernel, reduced float with a CPU scalar: opmath fp32
    step   T = r(fma32(v, r(float32(w)), T)) ufunc add: alpha.to<scalar_t>(), Vectorized fmadd in fp32
    unweighted step T = r(T + v)
    final  T = r(T / float32(count))         div_true_kernel, reduced float with a CPU scalar
    (fma32 is evaluated exactly in fp64 -- the product of two 16-bit values is exact there -- then rounded
    once to fp32.)"""
    with np.errstate(over="ignore", invalid="ignore"):
        total, c = None, None
        for v, w in zip(rows, weights):
            v = np.asarray(v, dtype=np.float32)
            if total is None:
                total = round16(v * np.float32(w), fmt) if weighted else v.copy()
                c = w
            else:
                if weighted:
                    a = np.float64(round16(np.float32(w), fmt))
                    total = round16((v.astype(np.float64) * a + total.astype(np.float64)).astype(np.float32), fmt)
                else:
                    total = round16(total + v, fmt)
                c = c + w
        if count is not None:
            c = count
        return round16(total / np.float32(c), fmt)


def synth_values(seed: int, row: int, cols: np.ndarray) -> np.ndarray:
    """Host twin of the device generator ``fedavg_fill_synthetic_f32`` (bit-identical values)."""
    lib = load()
    cols = np.ascontiguousarray(cols, dtype=np.uint64)
    out = np.empty(cols.size, dtype=np.float32)
    lib.oracle_synth_fill_f32(int(seed), int(row), cols.ctypes.data, cols.size, out.ctypes.data)
    return out


def synth_weights(K: int):
    """Synthetic per-client weights of SURVEY.md section 8d: aggregation_weight 1.0 x NUM_STEPS (1 + 37k mod 100)."""
    return [1.0 * float(1 + (37 * k) % 100) for k in range(K)]


# ---------------------------------------------------------------------------------------------------
# server-optimizer epilogues (rows a9/a10): see oracle_epilogue_apply in fedavg_oracle.c
# ---------------------------------------------------------------------------------------------------
EPI_NONE, EPI_ADD_BASE, EPI_SGD, EPI_ADAM, EPI_ADAGRAD, EPI_RMSPROP, EPI_ADAMAX, EPI_NADAM, EPI_RADAM, EPI_RPROP, EPI_ASGD = range(11)


class _Epi(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int),
        ("first_step", ctypes.c_int),
        ("nesterov", ctypes.c_int),
        ("maximize", ctypes.c_int),
        ("decoupled_weight_decay", ctypes.c_int),
        ("lr", ctypes.c_double),
        ("momentum", ctypes.c_double),
        ("dampening", ctypes.c_double),
        ("weight_decay", ctypes.c_double),
        ("beta1", ctypes.c_double),
        ("beta2", ctypes.c_double),
        ("eps", ctypes.c_double),
        ("step", ctypes.c_double),
        ("amsgrad", ctypes.c_int),
        ("lr_decay", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("centered", ctypes.c_int),
        ("momentum_decay", ctypes.c_double),
        ("mu_product", ctypes.c_double),
        ("etaminus", ctypes.c_double),
        ("etaplus", ctypes.c_double),
        ("step_size_min", ctypes.c_double),
        ("step_size_max", ctypes.c_double),
        ("eta", ctypes.c_double),
        ("mu", ctypes.c_double),
        ("lambd", ctypes.c_double),
        ("sqrt_table", ctypes.c_void_p),
        ("rsqrtps_table", ctypes.c_void_p),
    ]


_SQRT_TABLE_FILE = os.path.join(os.path.dirname(_HERE), "nvflare_amd", "data", "rsqrt14_avx512.bin")
_sqrt_table = None


def sqrt_table() -> np.ndarray:
    """The VRSQRT14PS estimates behind torch CPU's sqrt (captured by tools/sqrt_probe.c where the golden FedOpt
    fixtures were generated): 2 x 2^15 uint32 results for x in [1, 2) then [2, 4), one per top-15-bit mantissa,
    as the uint16 mantissa bits 22..7 oracle_sqrt_torch_cpu indexes (every entry has exponent 126 and its low 7
    mantissa bits clear -- checked here)."""
    global _sqrt_table
    if _sqrt_table is None:
        raw = np.fromfile(_SQRT_TABLE_FILE, dtype=np.uint32)
        if raw.size != 65536 or np.any((raw >> 23) != 126) or np.any(raw & 0x7F):
            raise ValueError(f"{_SQRT_TABLE_FILE}: not a VRSQRT14 table")
        _sqrt_table = np.ascontiguousarray(((raw >> 7) & 0xFFFF).astype(np.uint16))
    return _sqrt_table


def sqrt_torch_cpu(x) -> np.ndarray:
    """torch CPU's fp32 sqrt restated (oracle_sqrt_torch_cpu in fedavg_oracle.c), elementwise."""
    lib = load()
    fn = lib.oracle_sqrt_torch_cpu_n
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    tab = sqrt_table()
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    fn(tab.ctypes.data, x.ctypes.data, x.size, out.ctypes.data)
    return out


def sqrt_torch_cpu_sse2(x) -> np.ndarray:
    """torch CPU's fp32 sqrt where MKL takes its SSE2 path (AMD hosts; oracle_sqrt_mkl_sse2), elementwise."""
    lib = load()
    fn = lib.oracle_sqrt_mkl_sse2_n
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    fn(x.ctypes.data, x.size, out.ctypes.data)
    return out


_RSQRTPS_BOX_FILE = os.path.join(os.path.dirname(_HERE), "tests", "golden", "rsqrtps_amd_epyc9575f.bin")
_rsqrtps = None
_rsqrtps_box = None


def rsqrtps_table() -> np.ndarray:
    """RSQRTPS of THIS host CPU (oracle_host_rsqrtps_table; the product captures its own, fedavg_host_rsqrtps_table):
    2 x 4096 uint16, mantissa bits 22..11 of the estimate for x in [1, 2) then [2, 4), one per top-12-bit mantissa."""
    global _rsqrtps
    if _rsqrtps is None:
        lib = load()
        fn = lib.oracle_host_rsqrtps_table
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p]
        t = np.zeros(8192, np.uint16)
        bad = fn(t.ctypes.data)
        if bad:
            raise ValueError(f"this CPU's RSQRTPS is not a 12-bit estimate in [0.5, 1) ({bad} blocks)")
        _rsqrtps = t
    return _rsqrtps


def rsqrtps_table_box() -> np.ndarray:
    """RSQRTPS of the GPU pool's AMD EPYC 9575F hosts, captured there in round 3 (tools/rsqrtps_dump.c,
    tools/make_rsqrtps_table.py): the fixture tests/golden/rsqrtps_amd_epyc9575f.bin, which pins the restatement to
    that host's torch.sqrt (tests/golden/sqrt_amd_box.npz)."""
    global _rsqrtps_box
    if _rsqrtps_box is None:
        t = np.fromfile(_RSQRTPS_BOX_FILE, dtype=np.uint16)
        if t.size != 8192 or np.any(t > 0xFFF):
            raise ValueError(f"{_RSQRTPS_BOX_FILE}: not an RSQRTPS table")
        _rsqrtps_box = np.ascontiguousarray(t)
    return _rsqrtps_box


def sqrt_torch_cpu_amd(x, table: Optional[np.ndarray] = None) -> np.ndarray:
    """torch CPU's fp32 sqrt where MKL takes vsSqrt's SSE4.2 / AVX kernel (the AMD hosts; oracle_sqrt_mkl_rsqrtps) with
    THIS CPU's RSQRTPS table, or ``table`` (another CPU's, e.g. the AMD box's fixture rsqrtps_table_box())."""
    lib = load()
    fn = lib.oracle_sqrt_mkl_rsqrtps_n
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    tab = np.ascontiguousarray(rsqrtps_table() if table is None else table, dtype=np.uint16)
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    fn(tab.ctypes.data, x.ctypes.data, x.size, out.ctypes.data)
    return out


SQRT_FUNCS = {"torch_cpu": sqrt_torch_cpu, "torch_cpu_amd": sqrt_torch_cpu_amd, "ieee": np.sqrt}


def epilogue_apply(delta, kind, p=None, m=None, v=None, base=None, vmax=None, torch_cpu_sqrt=False,
                   rsqrtps=None, **hp):
    """Apply an epilogue to the aggregated update `delta` (fp32).  p/m/v (and vmax with amsgrad=1) are
    updated IN PLACE (copies are the caller's business); returns `out` for NONE/ADD_BASE and p otherwise.
    ``torch_cpu_sqrt``: which sqrt -- False / "ieee" the correctly rounded one, True / "torch_cpu" torch CPU's
    AVX-512 vsSqrt (oracle_sqrt_torch_cpu), "torch_cpu_amd" its SSE4.2 / AVX path on the AMD hosts
    (oracle_sqrt_mkl_rsqrtps with ``rsqrtps`` or THIS host's RSQRTPS table)."""
    lib = load()
    fn = lib.oracle_epilogue_apply
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_Epi)] + [ctypes.c_void_p] * 6
    delta = np.ascontiguousarray(delta, dtype=np.float32).reshape(-1)
    e = _Epi()
    e.kind = kind
    for k, val in hp.items():
        setattr(e, k, val)
    if torch_cpu_sqrt not in (False, True, "ieee", "torch_cpu", "torch_cpu_amd"):
        raise ValueError(f"torch_cpu_sqrt={torch_cpu_sqrt!r}")
    if torch_cpu_sqrt is True or torch_cpu_sqrt == "torch_cpu":
        e.sqrt_table = sqrt_table().ctypes.data
    elif torch_cpu_sqrt == "torch_cpu_amd":
        tab = np.ascontiguousarray(rsqrtps_table() if rsqrtps is None else rsqrtps, dtype=np.uint16)
        e.rsqrtps_table = tab.ctypes.data
    out = np.empty_like(delta)

    def ptr(a):
        return None if a is None else a.ctypes.data

    if (e.amsgrad or e.centered) and vmax is None:
        raise ValueError("amsgrad / centered need vmax")
    fn(delta.ctypes.data, delta.size, ctypes.byref(e), ptr(p), ptr(m), ptr(v), ptr(vmax), ptr(base), out.ctypes.data)
    return out if kind in (EPI_NONE, EPI_ADD_BASE) else p


# ---------------------------------------------------------------------------------------------------
# dequantisation (row f4): see oracle_dequantize in fedavg_oracle.c
# ---------------------------------------------------------------------------------------------------
Q_F16, Q_BF16, Q_BLOCKWISE8, Q_FP4, Q_NF4, Q_ADA_U8, Q_ADA_U16 = 1, 2, 3, 4, 5, 6, 7


def dequantize(qtype, q, n, absmax=None, code=None, blocksize=0, norm=0.0, level=1.0, offset=0.0, has_norm=True):
    """Dequantize n elements of payload q (numpy) into a new float32 array."""
    lib = load()
    fn = lib.oracle_dequantize
    fn.restype = None
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                   ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
    q = np.ascontiguousarray(q)
    out = np.empty(n, np.float32)
    am = None if absmax is None else np.ascontiguousarray(absmax, dtype=np.float32)
    cd = None if code is None else np.ascontiguousarray(code, dtype=np.float32)
    fn(int(qtype), q.ctypes.data, int(n), None if am is None else am.ctypes.data, None if cd is None else cd.ctypes.data,
       int(blocksize), float(norm), float(level), float(offset), int(bool(has_norm)), out.ctypes.data)
    return out
