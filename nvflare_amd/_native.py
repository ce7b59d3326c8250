"""ctypes binding of libnvflare_amd_fedavg.so (include/nvflare_amd_fedavg.h).

There is no CPU fallback: if the HIP library is missing or cannot be loaded, every entry point raises.
``import torch`` happens first when torch is importable, so that the process has ONE HIP runtime:
torch ships its own ``libamdhip64.so.7`` and the dynamic loader then binds this library's
``libamdhip64.so.7`` dependency to the already-loaded copy (same SONAME).
"""

from __future__ import annotations

import ctypes
import os
import threading

from ._build import LIB_PATH

try:  # share torch's HIP runtime when torch is present (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

FEDAVG_F32 = 0
FEDAVG_F64 = 1
FEDAVG_I32 = 2
FEDAVG_I64 = 3
FEDAVG_F16 = 4
FEDAVG_BF16 = 5
FEDAVG_U8 = 6
FEDAVG_I8 = 7
FEDAVG_I16 = 8
FEDAVG_BOOL = 9
FEDAVG_U16 = 10
FEDAVG_U32 = 11
FEDAVG_U64 = 12

FEDAVG_OP_NUMPY = 0
FEDAVG_OP_TORCH = 1
FEDAVG_OP_UNWEIGHTED = 2
FEDAVG_OP_TORCH_DEVICE = 3  # torch-ROCm arithmetic of device-resident tensors

FEDAVG_FIN_NONE = 0
FEDAVG_FIN_SCALE = 1
FEDAVG_FIN_DIV = 2
FEDAVG_FIN_RECIP = 3  # torch-ROCm div_ by a CPU scalar: multiply by the opmath reciprocal

ABI_VERSION = 9  # include/nvflare_amd_fedavg.h FEDAVG_ABI_VERSION

# fedavg_epilogue.torch_sqrt (enum fedavg_sqrt)
FEDAVG_SQRT_IEEE = 0
FEDAVG_SQRT_TORCH_AVX512 = 1
FEDAVG_SQRT_TORCH_AMD = 2

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_size_t = ctypes.c_size_t
c_u64 = ctypes.c_uint64
c_double = ctypes.c_double
c_float = ctypes.c_float

# name -> argtypes (every function returns int rc, except the two noted)
_SIGNATURES = {
    "fedavg_device_count": [ctypes.POINTER(c_int)],
    "fedavg_create": [c_int, ctypes.POINTER(c_void_p)],
    "fedavg_destroy": [c_void_p],
    "fedavg_device_info": [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t)],
    "fedavg_set_stream": [c_void_p, c_void_p],
    "fedavg_get_stream": [c_void_p, ctypes.POINTER(c_void_p)],
    "fedavg_malloc": [c_void_p, c_size_t, ctypes.POINTER(c_void_p)],
    "fedavg_free": [c_void_p, c_void_p],
    "fedavg_h2d": [c_void_p, c_void_p, c_void_p, c_size_t],
    "fedavg_h2d_tiled": [c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_void_p, c_size_t],
    "fedavg_d2d_tiled": [c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_void_p, c_size_t],
    "fedavg_h2d_tiled_multi": [c_void_p, c_void_p, c_size_t, c_size_t, c_int, ctypes.POINTER(c_size_t),
                               ctypes.POINTER(c_void_p), ctypes.POINTER(c_size_t)],
    "fedavg_d2h": [c_void_p, c_void_p, c_void_p, c_size_t],
    "fedavg_d2h_multi": [c_void_p, c_void_p, c_void_p, c_int, ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t),
                         ctypes.POINTER(c_size_t)],
    "fedavg_host_register": [c_void_p, c_void_p, c_size_t],
    "fedavg_host_unregister": [c_void_p, c_void_p],
    "fedavg_d2d": [c_void_p, c_void_p, c_void_p, c_size_t],
    "fedavg_memset": [c_void_p, c_void_p, c_int, c_size_t],
    "fedavg_sync": [c_void_p],
    "fedavg_accumulate": [
        c_void_p,  # ctx
        ctypes.POINTER(c_void_p),  # rows
        ctypes.POINTER(c_double),  # weights
        c_int,  # k_rows
        c_void_p,  # acc_in
        c_void_p,  # out
        c_size_t,  # n
        c_int,  # in_dtype
        c_int,  # acc_dtype
        c_int,  # op
        c_int,  # fin
        c_double,  # count
    ],
    "fedavg_accumulate_tiled": [
        c_void_p,  # ctx
        ctypes.POINTER(c_void_p),  # bases
        ctypes.POINTER(c_double),  # weights
        c_int,  # k_rows
        c_size_t,  # tile_elems
        c_size_t,  # tile_stride
        c_size_t,  # begin
        c_size_t,  # end
        c_void_p,  # acc_in
        c_void_p,  # out
        c_int,  # op
        c_int,  # fin
        c_double,  # count
    ],
    "fedavg_mark": [c_void_p, c_size_t],
    "fedavg_marks_reset": [c_void_p],
    "fedavg_d2h_marked": [c_void_p, c_void_p, c_void_p, c_size_t],
    "fedavg_accumulate_tiled16": [
        c_void_p,  # ctx
        c_int,  # fmt
        ctypes.POINTER(c_void_p),  # bases
        ctypes.POINTER(c_double),  # weights
        c_int,  # k_rows
        c_size_t,  # tile_elems
        c_size_t,  # tile_stride
        c_size_t,  # begin
        c_size_t,  # end
        c_void_p,  # acc_in
        c_void_p,  # out
        c_int,  # op
        c_int,  # fin
        c_double,  # count
    ],
    "fedavg_accumulate_tiled16_tails": [
        c_void_p,  # ctx
        c_int,  # fmt
        ctypes.POINTER(c_void_p),  # bases
        ctypes.POINTER(c_double),  # weights
        c_int,  # k_rows
        c_size_t,  # tile_elems
        c_size_t,  # tile_stride
        c_size_t,  # begin
        c_size_t,  # end
        c_void_p,  # acc_in
        c_void_p,  # out
        c_int,  # op
        c_int,  # fin
        c_double,  # count
        c_void_p,  # tails (int64, host)
        c_size_t,  # n_tails
    ],
    "fedavg_accumulate_tiled64": [
        c_void_p,  # ctx
        ctypes.POINTER(c_void_p),  # bases
        ctypes.POINTER(c_double),  # weights
        c_int,  # k_rows
        c_size_t,  # tile_elems
        c_size_t,  # tile_stride
        c_size_t,  # begin
        c_size_t,  # end
        c_void_p,  # acc_in
        c_void_p,  # out
        c_int,  # op
        c_int,  # fin
        c_double,  # count
    ],
    "fedavg_accumulate_tiled_epi": [
        c_void_p,  # ctx
        ctypes.POINTER(c_void_p),  # bases
        ctypes.POINTER(c_double),  # weights
        c_int,  # k_rows
        c_size_t,  # tile_elems
        c_size_t,  # tile_stride
        c_size_t,  # begin
        c_size_t,  # end
        c_void_p,  # acc_in
        c_void_p,  # out
        c_int,  # op
        c_int,  # fin
        c_double,  # count
        c_void_p,  # const fedavg_epilogue*
    ],
    "fedavg_set_timing": [c_void_p, c_int],
    "fedavg_last_kernel_ms": [c_void_p, ctypes.POINTER(c_float)],
    "fedavg_timing_begin": [c_void_p],
    "fedavg_timing_end": [c_void_p, ctypes.POINTER(c_float)],
    "fedavg_set_launch": [c_void_p, c_int, c_int],
    "fedavg_launch_count": [c_void_p, ctypes.POINTER(ctypes.c_uint64)],
    "fedavg_set_variant": [c_void_p, c_int],
    "fedavg_set_tile": [c_void_p, c_int],
    "fedavg_fill_synthetic_f32": [c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_u64, c_u64, c_u64],
    "fedavg_gather_f32": [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
    "fedavg_sqrt_f32": [c_void_p, c_void_p, c_void_p, c_size_t, c_int],
    "fedavg_host_rsqrtps_table": [c_void_p, c_size_t],  # v9: this CPU's RSQRTPS (host only)
    "fedavg_set_rsqrtps_table": [c_void_p, c_void_p, c_size_t],  # v9: the table FEDAVG_SQRT_TORCH_AMD reads
    "fedavg_dequantize": [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_size_t, c_size_t],
}
EXPORTED = ["fedavg_last_error", "fedavg_abi_version", "fedavg_struct_size", *_SIGNATURES.keys()]


FEDAVG_EPI_NONE = 0
FEDAVG_EPI_ADD_BASE = 1
FEDAVG_EPI_SGD = 2
FEDAVG_EPI_ADAM = 3
FEDAVG_EPI_ADAGRAD = 4
FEDAVG_EPI_RMSPROP = 5
FEDAVG_EPI_ADAMAX = 6
FEDAVG_EPI_NADAM = 7
FEDAVG_EPI_RADAM = 8
FEDAVG_EPI_RPROP = 9
FEDAVG_EPI_ASGD = 10


class Epilogue(ctypes.Structure):
    """struct fedavg_epilogue (include/nvflare_amd_fedavg.h)."""

    _fields_ = [
        ("kind", c_int),
        ("first_step", c_int),
        ("nesterov", c_int),
        ("maximize", c_int),
        ("decoupled_weight_decay", c_int),
        ("lr", c_double),
        ("momentum", c_double),
        ("dampening", c_double),
        ("weight_decay", c_double),
        ("beta1", c_double),
        ("beta2", c_double),
        ("eps", c_double),
        ("step", c_double),
        ("param", c_void_p),
        ("state1", c_void_p),
        ("state2", c_void_p),
        ("base", c_void_p),
        ("amsgrad", c_int),
        ("state3", c_void_p),
        ("lr_decay", c_double),
        ("alpha", c_double),
        ("centered", c_int),
        ("momentum_decay", c_double),
        ("mu_product", c_double),
        ("etaminus", c_double),
        ("etaplus", c_double),
        ("step_size_min", c_double),
        ("step_size_max", c_double),
        ("eta", c_double),
        ("mu", c_double),
        ("lambd", c_double),
        ("torch_sqrt", c_int),  # v8: FEDAVG_SQRT_* (nvflare_amd/torch_sqrt.py epilogue_flag)
    ]


FEDAVG_Q_F16 = 1
FEDAVG_Q_BF16 = 2
FEDAVG_Q_BLOCKWISE8 = 3
FEDAVG_Q_FP4 = 4
FEDAVG_Q_NF4 = 5
FEDAVG_Q_ADA_U8 = 6
FEDAVG_Q_ADA_U16 = 7


class Quant(ctypes.Structure):
    """struct fedavg_quant (include/nvflare_amd_fedavg.h)."""

    _fields_ = [
        ("qtype", c_int),
        ("has_norm", c_int),
        ("blocksize", c_size_t),
        ("absmax", c_void_p),
        ("code", c_void_p),
        ("norm", c_double),
        ("level", c_double),
        ("offset", c_double),
    ]


class FedAvgError(RuntimeError):
    """An error reported by the HIP library (its fedavg_last_error string)."""


_lib = None
_lib_lock = threading.Lock()


def lib_path() -> str:
    return os.environ.get("NVFLARE_AMD_FEDAVG_LIB", LIB_PATH)


def load():
    """Load the HIP library (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not os.path.exists(path):
            raise FedAvgError(
                f"HIP library {path} is missing; build it with `python -m nvflare_amd._build` "
                "(hipcc --offload-arch=gfx950). nvflare_amd has no CPU fallback."
            )
        lib = ctypes.CDLL(path)
        lib.fedavg_last_error.restype = ctypes.c_char_p
        lib.fedavg_last_error.argtypes = []
        lib.fedavg_abi_version.restype = c_int
        lib.fedavg_abi_version.argtypes = []
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = c_int
            fn.argtypes = argtypes
        if lib.fedavg_abi_version() != ABI_VERSION:
            raise FedAvgError(f"ABI mismatch: library {lib.fedavg_abi_version()} != python {ABI_VERSION}")
        lib.fedavg_struct_size.restype = c_size_t
        lib.fedavg_struct_size.argtypes = [c_int]
        for which, struct in enumerate((Epilogue, Quant)):
            if lib.fedavg_struct_size(which) != ctypes.sizeof(struct):
                raise FedAvgError(f"ABI mismatch: library sizeof({struct.__name__}) = "
                                  f"{lib.fedavg_struct_size(which)} != python {ctypes.sizeof(struct)}")
        _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().fedavg_last_error().decode(errors="replace")
        raise FedAvgError(f"{what}: {msg}" if what else msg)


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def device_count() -> int:
    n = c_int(0)
    call("fedavg_device_count", ctypes.byref(n))
    return n.value
