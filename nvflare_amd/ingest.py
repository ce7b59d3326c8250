"""Ingest without intermediate host copies.

A client's weights reach the server as serialized bytes: FOBS numpy payloads (``np.save`` format,
``app_common/decomposers/numpy_decomposers.py:98-107``), safetensors payloads for torch tensors
(``app_opt/pt/decomposers.py:122-132``), or -- with tensor disk offload -- safetensors files on disk that
the aggregation helper materialises one key at a time (``app_opt/pt/lazy_tensor_dict.py:70-90``,
``weighted_aggregation_helper.py:170-175``).  The reference decodes each into a fresh array / tensor (one
full host copy, plus page faults on the new memory) and the GPU path then copies it again into the
pinned staging ring.  Here the bytes are parsed in place instead:

* ``recompose_npy`` / ``recompose_safetensors``: array / tensor VIEWS over the received buffer (header
  parsed, no copy); the aggregator stages them straight from the message bytes into the pinned ring.
* ``MappedTensor``: a disk-offloaded ``_LazyRef`` resolved to a read-only mmap of its safetensors file;
  the engine copies the tensor's bytes from the page cache into the ring (``fedavg_h2d_tiled_multi``)
  without materialising a tensor.  Anything that is not a parseable safetensors file keeps the
  reference's ``materialize()``.

Views over ``bytes`` are read-only: consumers that write into decoded arrays in place must use the
reference decomposers (the aggregator never writes into its inputs, weighted_aggregation_helper.py:181-199).
"""

from __future__ import annotations

import io
import json
import mmap
import os
import struct
import warnings
from typing import Any, Dict, Optional, Tuple

import numpy as np

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

# safetensors dtype tags (https://github.com/huggingface/safetensors, format spec: 8-byte little-endian header
# length, JSON header {name: {dtype, shape, data_offsets: [begin, end]}}, then the byte buffer)
_ST_NP = {
    "F64": np.float64, "F32": np.float32, "F16": np.float16, "I64": np.int64, "I32": np.int32, "I16": np.int16,
    "I8": np.int8, "U8": np.uint8, "BOOL": np.bool_, "U16": np.uint16, "U32": np.uint32, "U64": np.uint64,
}


def _st_torch_dtype(tag: str):
    if torch is None:
        raise TypeError("torch is required for safetensors payloads")
    table = {"F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
             "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
             "BOOL": torch.bool}
    if tag not in table:
        raise TypeError(f"safetensors dtype {tag} not supported")
    return table[tag]


def parse_safetensors_header(buf) -> Tuple[int, Dict[str, Any]]:
    """(offset of the byte buffer, header dict without __metadata__) of a safetensors blob or mmap."""
    if len(buf) < 8:
        raise ValueError("not a safetensors payload (shorter than 8 bytes)")
    (n,) = struct.unpack_from("<Q", buf, 0)
    if n > len(buf) - 8:
        raise ValueError("not a safetensors payload (header length past the end)")
    header = json.loads(bytes(buf[8:8 + n]).decode("utf-8"))
    header.pop("__metadata__", None)
    return 8 + n, header


def recompose_npy(data) -> np.ndarray:
    """``np.load(BytesIO(data), allow_pickle=False)`` as a view over ``data`` (numpy_decomposers.py:105-107).

    Object arrays (which np.load refuses without pickle anyway) and malformed payloads fall back to np.load."""
    f = io.BytesIO(data)
    try:
        version = np.lib.format.read_magic(f)
        if version == (1, 0):
            shape, fortran, dtype = np.lib.format.read_array_header_1_0(f)
        elif version in ((2, 0), (3, 0)):
            shape, fortran, dtype = np.lib.format.read_array_header_2_0(f)
        else:
            raise ValueError(f"npy version {version}")
    except ValueError:
        return np.load(io.BytesIO(data), allow_pickle=False)
    if dtype.hasobject:
        return np.load(io.BytesIO(data), allow_pickle=False)
    count = int(np.prod(shape, dtype=np.int64)) if shape else 1
    arr = np.frombuffer(data, dtype=dtype, count=count, offset=f.tell())
    if fortran:
        return arr.reshape(shape[::-1]).T
    return arr.reshape(shape)


def recompose_safetensors(data) -> Dict[str, Any]:
    """``safetensors.torch.load(data)`` as tensor views over ``data`` (app_opt/pt/decomposers.py:127-132)."""
    start, header = parse_safetensors_header(data)
    out = {}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)  # torch.frombuffer on a read-only buffer
        for name, info in header.items():
            b, e = info["data_offsets"]
            dt = _st_torch_dtype(info["dtype"])
            shape = tuple(info["shape"])
            n = int(np.prod(shape, dtype=np.int64)) if shape else 1
            if n == 0:
                out[name] = torch.empty(shape, dtype=dt)
                continue
            t = torch.frombuffer(data, dtype=dt, count=n, offset=start + b)
            out[name] = t.reshape(shape)
    return out


class MappedTensor:
    """A safetensors tensor read in place from a read-only mmap of its file (the disk-offload ``_LazyRef``).

    The aggregation engine stages ``host_view()`` straight into the pinned ring; ``materialize()`` gives the
    reference's tensor (a copy) to anyone else."""

    __slots__ = ("path", "key", "tag", "dtype", "shape", "nbytes", "_offset", "_ref")

    def __init__(self, path: str, key: str, ref=None):
        self.path = path
        self.key = key
        self._ref = ref  # the originating _LazyRef keeps its temp directory alive
        with open(path, "rb") as f:
            with mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as mm:
                start, header = parse_safetensors_header(mm)
        if key not in header:
            raise KeyError(f"{key!r} not in {path}")
        info = header[key]
        self.tag = info["dtype"]
        self.dtype = _st_torch_dtype(self.tag)
        self.shape = tuple(info["shape"])
        b, e = info["data_offsets"]
        self._offset = start + b
        self.nbytes = e - b

    def host_view(self) -> Tuple[Any, int, int]:
        """(keep-alive object, address, nbytes) of the tensor's bytes in a fresh read-only mapping."""
        fd = os.open(self.path, os.O_RDONLY)
        try:
            mm = mmap.mmap(fd, 0, access=mmap.ACCESS_READ)
        finally:
            os.close(fd)
        view = np.frombuffer(mm, dtype=np.uint8, count=self.nbytes, offset=self._offset)
        return (mm, view), (view.ctypes.data if self.nbytes else 0), self.nbytes

    def materialize(self):
        if self._ref is not None and hasattr(self._ref, "materialize"):
            return self._ref.materialize()
        from safetensors import safe_open

        with safe_open(self.path, framework="pt") as f:
            return f.get_tensor(self.key)

    def __repr__(self) -> str:
        return f"MappedTensor({self.path!r}, key={self.key!r}, {self.tag}, shape={self.shape})"


def as_mapped(v) -> Optional[MappedTensor]:
    """A MappedTensor for a disk-offload lazy reference (``file_path`` + ``key`` + ``materialize``, as
    lazy_tensor_dict.py:60-77's _LazyRef), None for anything else or an unreadable file."""
    if isinstance(v, MappedTensor):
        return v
    path = getattr(v, "file_path", None)
    key = getattr(v, "key", None)
    if not (isinstance(path, str) and isinstance(key, str) and callable(getattr(v, "materialize", None))):
        return None
    try:
        m = MappedTensor(path, key, ref=v)
        _st_torch_dtype(m.tag)
        return m
    except (OSError, ValueError, KeyError, TypeError):
        return None
