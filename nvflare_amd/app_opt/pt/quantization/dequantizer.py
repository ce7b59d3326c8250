"""Drop-in ``ModelDequantizer`` (server task-result filter) that dequantizes on the MI355X (row f4).

Reference: ``nvflare/app_opt/pt/quantization/dequantizer.py:31-224``.  Same filter contract (WEIGHTS /
WEIGHT_DIFF DXOs, ``PROCESSED_ALGORITHM`` names the format, ``quant_state`` / ``source_datatype`` meta,
which are removed afterwards), the same skip rules (bool tensors; quantization bits >= source bits) and the
same result container and dtype.  The per-format arithmetic runs in ``fedavg_dequantize``:

* ``lazy=False`` (default, the reference's behaviour): every quantized tensor is dequantized on the GPU
  and returned to the host as the numpy array / torch tensor the reference would produce;
* ``lazy=True``: tensors become ``QuantizedPayload`` values that the drop-in aggregator dequantizes
  straight into its HBM slots -- the staging copy moves the compressed bytes (4x / 8x fewer than fp32 for
  blockwise8 / 4-bit).  Anything else that reads the DXO sees objects with ``materialize()``, which NVFlare's
  own ``WeightedAggregationHelper`` calls (``weighted_aggregation_helper.py:170-175``).

bitsandbytes (which the reference uses for blockwise8 / float4 / normfloat4) is not needed: its kernels'
arithmetic is restated in ``nvflare_amd/csrc/fedavg_dequant.hip``.  ``adaquant`` payloads compressed with
bz2 are decompressed on the host (a byte-stream format) and dequantized on the device.
"""

from __future__ import annotations

import bz2
import re
from typing import Optional, Union

import numpy as np

from .... import _native as N
from ....compat import DXO, DataKind, DXOFilter, FLContext, MetaKey, Shareable
from ....quantized import QuantizedPayload

QUANTIZATION_TYPE = ["FLOAT16", "BLOCKWISE8", "FLOAT4", "NORMFLOAT4", "ADAQUANT"]  # constant.py
_BNB_BLOCKWISE8_BLOCKSIZE = 4096  # bitsandbytes dequantize_blockwise default (dequantizer.py:114 passes none)


def _torch():
    import torch

    return torch


def _to_np(a) -> np.ndarray:
    torch = _torch()
    if isinstance(a, torch.Tensor):
        return a.detach().cpu().contiguous().numpy()
    return np.asarray(a)


class ModelDequantizer(DXOFilter):
    def __init__(self, lazy: bool = False, device: Optional[int] = None):
        data_kinds = [DataKind.WEIGHTS, DataKind.WEIGHT_DIFF]
        super().__init__(supported_data_kinds=data_kinds, data_kinds_to_filter=data_kinds)
        self.lazy = bool(lazy)
        self.device = device
        self.logger.info("Using model dequantizer (MI355X).")

    # -------------------------------------------------------------------------------------------------
    def payload_for(self, values, qstate: dict, quantization_type: str, source_data_type: str,
                    source_format: str) -> Optional[QuantizedPayload]:
        """The device payload standing for one quantized tensor, or None when the reference keeps the
        value as it is (adaquant tensors that were never quantized)."""
        # fp32 values from the device; fp16 results are one RNE cast of them (numpy astype / torch .half()),
        # bf16 results (torch only -- numpy has no bf16) one .bfloat16() after materialize
        out_dtype = np.dtype(np.float16) if source_data_type == "float16" else np.dtype(np.float32)
        common = dict(container=source_format, device=self.device)
        if quantization_type == "float16":
            v = _to_np(values)
            return QuantizedPayload(N.FEDAVG_Q_F16, v.view(np.uint16), v.shape, out_dtype=out_dtype, **common)
        if quantization_type == "blockwise8":
            v = _to_np(values)
            return QuantizedPayload(N.FEDAVG_Q_BLOCKWISE8, v.view(np.uint8), v.shape, out_dtype=out_dtype,
                                    absmax=_to_np(qstate["absmax"]), code=_to_np(qstate["code"]),
                                    blocksize=_BNB_BLOCKWISE8_BLOCKSIZE, **common)
        if quantization_type in ("float4", "normfloat4"):
            if "nested_absmax" in qstate or "state2" in qstate:
                absmax = self._nested_absmax(qstate)
            else:
                absmax = _to_np(qstate["absmax"])
            shape = tuple(int(s) for s in qstate["shape"])
            # bitsandbytes dequantizes to QuantState.dtype; the reference then casts to the source dtype
            qt = N.FEDAVG_Q_FP4 if quantization_type == "float4" else N.FEDAVG_Q_NF4
            return QuantizedPayload(qt, _to_np(values).view(np.uint8), shape, out_dtype=out_dtype, absmax=absmax,
                                    blocksize=int(qstate["blocksize"]), **common)
        if quantization_type == "adaquant":
            if not qstate:
                return None
            shape = tuple(int(s) for s in qstate["tensor_shape"])
            offset = float(qstate["offset"])
            if source_data_type != "float32":
                raise TypeError("nvflare_amd: adaquant dequantization runs for float32 sources "
                                f"(got {source_data_type}; the reference rounds fp64 -> {source_data_type} once)")
            if "norm" not in qstate:
                return QuantizedPayload(N.FEDAVG_Q_ADA_U8, np.zeros(0, np.uint8), shape, out_dtype=out_dtype,
                                        offset=offset, has_norm=False, **common)
            if "compressed_tensor" in qstate:
                raw = bz2.decompress(_to_np(qstate["compressed_tensor"]).tobytes())
                q = np.frombuffer(raw, dtype=np.dtype(qstate["new_dtype"]))
            else:
                q = _to_np(values)
            qt = N.FEDAVG_Q_ADA_U8 if q.dtype.itemsize == 1 else N.FEDAVG_Q_ADA_U16
            return QuantizedPayload(qt, np.ascontiguousarray(q), shape, out_dtype=out_dtype, norm=float(qstate["norm"]),
                                    level=float(qstate["quantization_level"]), offset=offset, **common)
        raise ValueError(f"Invalid quantization type: {quantization_type}, valid: {QUANTIZATION_TYPE}")

    def _nested_absmax(self, qstate: dict) -> np.ndarray:
        """bitsandbytes compress_statistics: absmax itself blockwise-8 quantized, plus an offset."""
        nested = QuantizedPayload(N.FEDAVG_Q_BLOCKWISE8, _to_np(qstate["absmax"]).view(np.uint8),
                                  _to_np(qstate["absmax"]).shape, container="numpy",
                                  absmax=_to_np(qstate["nested_absmax"]), code=_to_np(qstate["nested_quant_map"]),
                                  blocksize=int(qstate["nested_blocksize"]), device=self.device)
        return nested.materialize() + np.float32(qstate["nested_offset"])

    def dequantization(self, params: dict, quant_state: dict, quantization_type: str, source_datatype: dict,
                       fl_ctx: FLContext):
        """dequantizer.py:47-185 with the arithmetic on the device."""
        n_params = len(params)
        self.log_info(fl_ctx, f"Running dequantization on {n_params} variables")
        n_quant = 0
        for name in list(params.keys()):
            source_data_type = source_datatype[name]
            if source_data_type == "bool":
                continue
            if quantization_type != "adaquant":
                source_bits = int(re.findall(r"\d+", source_data_type)[0])
                quant_bits = int(re.findall(r"\d+", quantization_type)[0])
                if quant_bits >= source_bits:
                    self.log_info(fl_ctx, f"Skipping dequantization for {name}, quantization bit {quantization_type}"
                                          f" >= source data bit {source_data_type}")
                    continue
            values = params[name]
            torch = _torch()
            if isinstance(values, np.ndarray):
                source_format = "numpy"
            elif isinstance(values, torch.Tensor):
                source_format = "torch"
            else:
                raise ValueError(f"Invalid source data type: {type(values)}, valid: numpy or torch")
            n_quant += 1
            payload = self.payload_for(values, quant_state.get(name) or {}, quantization_type, source_data_type,
                                       source_format)
            if payload is None:  # adaquant left this tensor as it was: only the dtype cast applies
                params[name] = self._cast(values, source_format, source_data_type)
            elif self.lazy and payload.out_dtype == np.float32:
                params[name] = payload
            else:
                params[name] = payload.materialize()
                if source_data_type == "bfloat16":
                    params[name] = params[name].bfloat16()
        self.log_info(fl_ctx, f"Dequantized {n_quant}/{n_params} params on the device ({'lazy' if self.lazy else 'eager'}).")
        return params

    @staticmethod
    def _cast(values, source_format: str, source_data_type: str):
        if source_format == "numpy":
            if source_data_type in ("float32", "float16"):
                return values.astype(np.dtype(source_data_type))
            return values
        return {"float32": values.float, "float16": values.half, "bfloat16": values.bfloat16}.get(
            source_data_type, lambda: values)()

    def process_dxo(self, dxo: DXO, shareable: Shareable, fl_ctx: FLContext) -> Union[None, DXO]:
        self.log_info(fl_ctx, "Running dequantization...")
        quantization_type = dxo.get_meta_prop(key=MetaKey.PROCESSED_ALGORITHM, default=None)
        if quantization_type is None or quantization_type.upper() not in QUANTIZATION_TYPE:
            raise ValueError(f"Invalid quantization type: {quantization_type}, valid: {QUANTIZATION_TYPE}")
        source_datatype = dxo.get_meta_prop(key="source_datatype", default=None)
        dxo.data = self.dequantization(params=dxo.data, quant_state=dxo.meta["quant_state"],
                                       quantization_type=quantization_type.lower(), source_datatype=source_datatype,
                                       fl_ctx=fl_ctx)
        dxo.remove_meta_props([MetaKey.PROCESSED_ALGORITHM, "quant_state", "source_datatype", "quantized_flag"])
        dxo.update_shareable(shareable)
        self.log_info(fl_ctx, "Dequantized back to original precision")
        return dxo
