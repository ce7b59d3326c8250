"""Host logic of the FedOpt controller drop-in (nvflare_amd/app_opt/pt/fedopt_ctl.py) with the server step
mocked, as the reference's own tests/unit_test/app_opt/pt/pt_fedopt_ctl_test.py does: ``update_model`` keeps
the aggregate's meta and metrics (None included), takes the stepped parameters from ``optimizer_update``
and gives the aggregate's other keys the FedAvg ``base + diff`` update (fedopt_ctl.py:141-176)."""

from unittest.mock import MagicMock

import numpy as np

from nvflare_amd.app_opt.pt.fedopt_ctl import DeviceFedOptUpdate
from nvflare_amd.compat import FLModel


class _HostWeight:
    """Stands in for a tensor of the model's state_dict (detach / cpu / numpy)."""

    def __init__(self, value):
        self.value = value

    def detach(self):
        return self

    def cpu(self):
        return self

    def numpy(self):
        return self.value


def _controller():
    c = object.__new__(DeviceFedOptUpdate)
    c.current_round = 3
    c.device = "cuda:0"
    c.optimizer = MagicMock(param_groups=[{"lr": 0.1}])
    c.lr_scheduler = None
    c.info = MagicMock()
    c.optimizer_update = MagicMock(side_effect=lambda diff: ({"trainable": _HostWeight(np.float32(1.5))}, ["trainable"]))
    return c


def test_update_model_keeps_aggregate_meta_metrics_and_fedavgs_other_keys():
    c = _controller()
    global_model = FLModel(params={"trainable": 1.0, "batch_norm": np.float32(10.0)}, metrics={"old": -1.0},
                           meta={"old_meta": "before"})
    aggr = FLModel(params={"trainable": 0.5, "batch_norm": np.float32(2.0)}, metrics={"loss": 0.25},
                   meta={"nr_aggregated": 2})
    out = c.update_model(global_model, aggr)
    assert out.params["trainable"] == 1.5
    assert out.params["batch_norm"] == 12.0
    assert out.meta == aggr.meta and out.metrics == aggr.metrics
    c.optimizer_update.assert_called_once_with(aggr.params)
    assert "fedopt layers: 1, fedavg layers: 1" in c.info.call_args[0][0]

    cleared = FLModel(params={"trainable": 0.5, "batch_norm": np.float32(2.0)}, metrics=None, meta={"nr_aggregated": 2})
    assert c.update_model(global_model, cleared).metrics is None
