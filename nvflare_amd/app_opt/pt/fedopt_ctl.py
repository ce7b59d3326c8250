"""GPU drop-in for the server step of ``nvflare.app_opt.pt.fedopt_ctl.FedOpt`` (the FedAvg-workflow FedOpt
controller).

Reference (fedopt_ctl.py:113-176): after each round's FedAvg aggregation, ``update_model`` calls
``optimizer_update``, which sets ``param.grad = torch.tensor(-1.0 * model_diff[name])`` for the parameters in
the aggregate, runs ``optimizer.step()`` and the lr scheduler, and returns ``torch_model.state_dict()``. Each
entry is then converted with ``.detach().cpu().numpy()``, and keys of the aggregate that are not trained
parameters (batch-norm statistics) get the FedAvg update ``global_model.params[key] + value``.

Here ``optimizer_update`` steps the parameters with the HIP fused-epilogue kernel through the same
``DeviceServerOptimizer`` as the SAG generator (app_opt/pt/fedopt.py): SGD / Adam / AdamW (amsgrad
included) with torch's single-tensor rounding, the optimizer object kept for its ``param_groups`` and
``state``. The new parameters come back in one D2H of the flat parameter buffer instead of a ``.cpu()`` per
tensor. A difference that is a ``DeferredAggregate`` of a round still staged on the device is aggregated and
stepped in the same launch.

``DeviceFedOptUpdate`` holds these two methods and needs only the attributes the reference controller
sets in ``run()`` (``torch_model``, ``optimizer``, ``lr_scheduler``, ``device``, ``current_round``, ``info``).
``FedOpt`` combines it with the reference controller when ``nvflare`` is importable, so a job swaps only
the class path.
"""

from __future__ import annotations

import time
import warnings
from typing import Dict, List, Optional, Tuple

import torch

from ...compat import HAVE_NVFLARE
from .fedopt import DeviceServerOptimizer, PTFedOptModelShareableGenerator, hip_device_index


class DeviceFedOptUpdate:
    """``optimizer_update`` / ``update_model`` of the reference FedOpt controller, stepped on the MI355X."""

    _device_opt: Optional[DeviceServerOptimizer] = None

    def _device_optimizer(self) -> DeviceServerOptimizer:
        dev = self._device_opt
        if dev is None or dev.optimizer is not self.optimizer or not dev.is_bound():
            dev = DeviceServerOptimizer(self.torch_model, self.optimizer, hip_device_index(self.device))
            self._device_opt = dev
        return dev

    def optimizer_update(self, model_diff: Dict) -> Tuple[Dict, List[str]]:
        """fedopt_ctl.py:113-139: the server step on g = -diff for the parameters in ``model_diff``."""
        dev = self._device_optimizer()
        self.torch_model.train()
        self.optimizer.zero_grad()
        updated_params = dev.step(model_diff)
        if self.lr_scheduler is not None:
            with warnings.catch_warnings():  # the step ran on the device, not through optimizer.step()
                warnings.simplefilter("ignore", UserWarning)
                self.lr_scheduler.step()
        return self.torch_model.state_dict(), updated_params

    def _weights_to_host(self, weights: Dict) -> Dict:
        dev = self._device_opt
        if dev is not None and all(isinstance(v, torch.Tensor) for v in weights.values()):
            return PTFedOptModelShareableGenerator._to_host(weights, preserve_torch=False, dev=dev)
        return {k: v.detach().cpu().numpy() for k, v in weights.items()}

    def update_model(self, global_model, aggr_result):
        """fedopt_ctl.py:141-176: new global params = stepped trainable parameters (+ the model's other
        state), FedAvg ``base + diff`` for the aggregate's other keys; meta and metrics of the aggregate."""
        model_diff = aggr_result.params

        start = time.time()
        weights, updated_params = self.optimizer_update(model_diff)
        secs = time.time() - start

        start = time.time()
        weights = self._weights_to_host(weights)
        secs_detach = time.time() - start

        n_fedavg = 0
        for key, value in model_diff.items():
            if key not in updated_params:
                weights[key] = global_model.params[key] + value
                n_fedavg += 1

        self.info(
            f"FedOpt ({type(self.optimizer)} {self.device}) server model update "
            f"round {self.current_round}, "
            f"{type(self.lr_scheduler)} "
            f"lr: {self.optimizer.param_groups[-1]['lr']}, "
            f"fedopt layers: {len(updated_params)}, "
            f"fedavg layers: {n_fedavg}, "
            f"update: {secs} secs., detach: {secs_detach} secs.",
        )

        global_model.params = weights
        global_model.meta = aggr_result.meta
        global_model.metrics = aggr_result.metrics
        return global_model


_ReferenceFedOpt = None
if HAVE_NVFLARE:
    try:
        from nvflare.app_opt.pt.fedopt_ctl import FedOpt as _ReferenceFedOpt
    except Exception:  # the workflow package needs more of nvflare than the API types
        _ReferenceFedOpt = None

if _ReferenceFedOpt is not None:

    class FedOpt(DeviceFedOptUpdate, _ReferenceFedOpt):
        """``nvflare.app_opt.pt.fedopt_ctl.FedOpt`` with its server step on the MI355X (same arguments;
        ``device`` names the HIP device, "cuda:N")."""

else:

    class FedOpt:  # pragma: no cover - needs the NVFlare workflow runtime
        def __init__(self, *args, **kwargs):
            raise ImportError("nvflare_amd FedOpt controller: the FedAvg workflow needs the nvflare package; "
                              "DeviceFedOptUpdate holds the device server step on its own")
