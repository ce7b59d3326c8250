"""FedOpt generator configuration and error paths (fedopt.py:30-155), host only."""

import numpy as np
import pytest
import torch

from golden_util import fedopt_model
from nvflare_amd.app_opt.pt.fedopt import PTFedOptModelShareableGenerator, build_component_from_args, hip_device_index
from nvflare_amd.compat import DXO, AppConstants, DataKind, EventType, FLContext, Learnable, make_model_learnable


def test_constructor_validation():
    with pytest.raises(TypeError):
        PTFedOptModelShareableGenerator(optimizer_args=[1])
    with pytest.raises(TypeError):
        PTFedOptModelShareableGenerator(lr_scheduler_args="x")
    g = PTFedOptModelShareableGenerator()
    assert g.optimizer_args == {"path": "torch.optim.SGD", "args": {"lr": 1.0}}


def test_device_index_rule(monkeypatch):
    monkeypatch.delenv("NVFLARE_AMD_DEVICE", raising=False)
    assert hip_device_index("cuda:3") == 3
    assert hip_device_index(2) == 2
    assert hip_device_index("cpu") == 0
    assert hip_device_index(None) == 0
    monkeypatch.setenv("NVFLARE_AMD_DEVICE", "5")
    assert hip_device_index("cpu") == 5


def test_build_component_from_args():
    p = [torch.nn.Parameter(torch.zeros(2))]
    opt = build_component_from_args({"class_path": "torch.optim.Adam", "args": {"params": p, "lr": 0.1}})
    assert isinstance(opt, torch.optim.Adam) and opt.param_groups[0]["lr"] == 0.1
    with pytest.raises(ValueError):
        build_component_from_args({"args": {}})


class _Panics:
    def __init__(self, gen):
        self.reasons = []
        gen.system_panic = lambda reason, fl_ctx: self.reasons.append(reason)


def test_start_run_panics_without_model():
    g = PTFedOptModelShareableGenerator(source_model="missing")
    p = _Panics(g)
    g.handle_event(EventType.START_RUN, FLContext())
    assert p.reasons == ["Model is not available"]
    g2 = PTFedOptModelShareableGenerator(source_model=object())
    p2 = _Panics(g2)
    g2.handle_event(EventType.START_RUN, FLContext())
    assert "torch.nn.Module" in p2.reasons[0]


def test_shareable_checks_panic_before_any_device_work():
    g = PTFedOptModelShareableGenerator(source_model=fedopt_model())
    p = _Panics(g)
    ctx = FLContext()
    out = g.shareable_to_learnable(DXO(DataKind.WEIGHTS, data={"w": np.zeros(2, np.float32)}).to_shareable(), ctx)
    assert isinstance(out, Learnable) and "WEIGHT_DIFF" in p.reasons[-1]
    s = DXO(DataKind.WEIGHT_DIFF, data={}, meta={"PROCESSED_ALGORITHM": "x"}).to_shareable()
    g.shareable_to_learnable(s, ctx)
    assert "processed by x" in p.reasons[-1]
    g.shareable_to_learnable(DXO(DataKind.WEIGHT_DIFF, data={}).to_shareable(), ctx)
    assert p.reasons[-1] == "No global base model!"
    ctx.set_prop(AppConstants.GLOBAL_MODEL, make_model_learnable({}, {}))


@pytest.mark.parametrize("kind", ["Rprop", "ASGD"])
def test_bad_difference_fails_before_lazy_state(kind):
    """A difference torch would refuse at ``param.grad = ...`` (other dtype / size) fails the step before
    Rprop / ASGD state is made (fedopt.py lazy init ran ahead of the checks)."""
    from nvflare_amd import _native as N
    from nvflare_amd.app_opt.pt.fedopt import DeviceServerOptimizer, _Slot

    a = torch.nn.Parameter(torch.zeros(3, 4))
    b = torch.nn.Parameter(torch.zeros(5))
    opt = getattr(torch.optim, kind)([a, b], lr=0.1)
    so = DeviceServerOptimizer.__new__(DeviceServerOptimizer)  # host logic only: no device buffers
    so.optimizer = opt
    so.kind = N.FEDAVG_EPI_RPROP if kind == "Rprop" else N.FEDAVG_EPI_ASGD
    so.slots = [_Slot("a", a, 0, 12), _Slot("b", b, 64, 5)]
    so.by_name = {s.name: s for s in so.slots}
    bad_cases = [
        {"a": np.zeros((3, 4), np.float32), "b": np.zeros(5, np.float64)},  # dtype
        {"a": np.zeros((4, 3), np.float32), "b": np.zeros(5, np.float32)},  # size
        {"a": torch.zeros(3, 4, dtype=torch.float16)},
    ]
    for diff in bad_cases:
        with pytest.raises(RuntimeError, match="assigned grad has data of a different"):
            so.step(diff)
        assert not any(s.state_initialised for s in so.slots)
        assert all(s.step == 0.0 for s in so.slots)
