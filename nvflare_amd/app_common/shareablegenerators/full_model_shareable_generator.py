"""Drop-in ``FullModelShareableGenerator`` whose WEIGHT_DIFF apply runs on the MI355X (row a9).

Reference: ``nvflare/app_common/shareablegenerators/full_model_shareable_generator.py:23-83``.  Same
surface and behaviour (``system_panic`` without a base model, ValueError for other data kinds, META
from the DXO).  ``weights[k] = weights[k] + diff[k]`` for float32 numpy-array / CPU-tensor pairs of equal
shape is computed by the HIP kernel (one fp32 add, bit-identical); anything else -- integer buffers,
python numbers, mixed containers -- keeps the reference's own host arithmetic.
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from ...compat import (
    AppConstants,
    DataKind,
    FLContext,
    ModelLearnable,
    ModelLearnableKey,
    Shareable,
    ShareableGenerator,
    from_shareable,
    model_learnable_to_dxo,
)
from ...deferred import DeferredAggregate, materialize_deferred
from ...engine import is_torch_tensor
from ._device_apply import DeviceAdder


def _fp32_host_view(v):
    """(numpy view, is_torch) for a float32 numpy array or CPU torch tensor; None otherwise."""
    if isinstance(v, np.ndarray) and v.dtype == np.float32 and v.ndim > 0:  # numpy 0-d + 0-d gives a scalar
        return v, False
    if is_torch_tensor(v) and v.device.type == "cpu" and str(v.dtype) == "torch.float32" and not v.requires_grad:
        return v.detach().contiguous().numpy(), True
    return None


def _apply_deferred(weights: Dict, diff: Dict, keys) -> list:
    """Keys whose difference is a pending DeferredAggregate (aggregator ``defer_result=True``) and whose
    base is an fp32 host array of the same container: aggregated and added in one launch
    (DeferredRound.fused_apply), so the difference never crosses PCIe.  Returns the keys left to do."""
    import torch

    by_round = {}
    for k in keys:
        d = diff[k]
        if not isinstance(d, DeferredAggregate) or not d.round.fusable(d.name):
            continue
        vb = _fp32_host_view(weights[k])
        if vb is None or vb[1] != (d.container == "torch"):
            continue
        by_round.setdefault(id(d.round), (d.round, {}))[1][d.name] = (k, vb[0], vb[1])
    done = set()
    for rnd, items in by_round.values():
        res = rnd.fused_apply({name: base for name, (_, base, _) in items.items()})
        for name, r in res.items():
            k, _, is_torch = items[name]
            weights[k] = torch.from_numpy(r) if is_torch else r
            done.add(k)
    return [k for k in keys if k not in done]


def apply_weight_diff(adder: DeviceAdder, weights: Dict, diff: Dict, keys=None) -> Dict:
    """weights[k] = weights[k] + diff[k] for k in keys (default: every key of diff); GPU for fp32 pairs."""
    import torch

    keys = list(diff) if keys is None else list(keys)
    keys = _apply_deferred(weights, diff, keys)
    dev_pairs, dev_keys, dev_torch = [], [], []
    for k in keys:
        b, d = weights[k], materialize_deferred(diff[k])
        vb, vd = _fp32_host_view(b), _fp32_host_view(d)
        if vb is not None and vd is not None and vb[1] == vd[1] and vb[0].shape == vd[0].shape:
            dev_pairs.append((vb[0], vd[0]))
            dev_keys.append(k)
            dev_torch.append(vb[1])
        else:
            weights[k] = b + d  # reference arithmetic for non-fp32 / mixed values
    for k, r, t in zip(dev_keys, adder.add(dev_pairs), dev_torch):
        weights[k] = torch.from_numpy(r) if t else r
    return weights


class FullModelShareableGenerator(ShareableGenerator):
    def __init__(self, device: Optional[int] = None):
        """Args: device: HIP device index for the WEIGHT_DIFF apply (default $NVFLARE_AMD_DEVICE or 0)."""
        super().__init__()
        self._adder = DeviceAdder(device)

    def learnable_to_shareable(self, model_learnable: ModelLearnable, fl_ctx: FLContext) -> Shareable:
        return model_learnable_to_dxo(model_learnable).to_shareable()

    def shareable_to_learnable(self, shareable: Shareable, fl_ctx: FLContext) -> ModelLearnable:
        if not isinstance(shareable, Shareable):
            raise TypeError("shareable must be Shareable, but got {}.".format(type(shareable)))
        base_model = fl_ctx.get_prop(AppConstants.GLOBAL_MODEL)
        dxo = from_shareable(shareable)
        if dxo.data_kind == DataKind.WEIGHT_DIFF:
            if not base_model:
                self.system_panic(reason="No global base model needed for processing WEIGHT_DIFF!", fl_ctx=fl_ctx)
                return base_model
            weights = base_model[ModelLearnableKey.WEIGHTS]
            if dxo.data is not None:
                apply_weight_diff(self._adder, weights, dxo.data)
        elif dxo.data_kind == DataKind.WEIGHTS:
            if not base_model:
                base_model = ModelLearnable()
            weights = dxo.data
            if not weights:
                self.log_info(fl_ctx, "No model weights found. Model will not be updated.")
            else:
                base_model[ModelLearnableKey.WEIGHTS] = weights
        else:
            raise ValueError(
                "data_kind should be either DataKind.WEIGHTS or DataKind.WEIGHT_DIFF, but got {}".format(dxo.data_kind)
            )
        base_model[ModelLearnableKey.META] = dxo.get_meta_props()
        return base_model
