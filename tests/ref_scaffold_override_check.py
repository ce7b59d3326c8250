"""Run by tests/test_cpu_reference_suite.py under tests/ref_suite_plugin.py (real NVFlare API classes from the
mounted reference; not collected on its own): the drop-in Scaffold controller moves only the reference's own
aggregation functions to the device.  A subclass overriding ``aggregate_fn`` keeps it, as the reference's
``BaseFedAvg.aggregate`` would call ``self.aggregate_fn`` (base_fedavg.py:251-252) -- ADVICE r02."""

import numpy as np

from nvflare.apis.fl_context import FLContext
from nvflare.app_common.abstract.fl_model import FLModel
from nvflare_amd.app_common.workflows.scaffold import Scaffold


def _ctl(cls):
    ctl = cls(num_clients=2, num_rounds=1)
    ctl.fl_ctx = FLContext()  # as the reference's own SCAFFOLD tests set it up (fedavg_test.py:1159-1160)
    ctl.info = ctl.warning = lambda *a, **k: None
    return ctl


def _results():
    return [FLModel(params={"w": np.full(3, float(i + 1), np.float32)}, meta={"NUM_STEPS_CURRENT_ROUND": 1},
                    current_round=0) for i in range(2)]


def test_subclass_aggregate_fn_is_kept():
    calls = []

    class Custom(Scaffold):
        @staticmethod
        def aggregate_fn(results):
            calls.append(len(results))
            return FLModel(params={"w": np.zeros(3, np.float32)})

    ctl = _ctl(Custom)
    out = ctl.aggregate(_results())
    assert calls == [2]
    assert np.array_equal(out.params["w"], np.zeros(3, np.float32))


def test_instance_aggregate_fn_is_kept():
    """An instance-level override (``self.aggregate_fn = fn``) runs as given, as the reference's
    ``self.aggregate_fn`` lookup would run it."""
    calls = []

    def fn(results):
        calls.append(len(results))
        return FLModel(params={"w": np.full(3, 7.0, np.float32)})

    ctl = _ctl(Scaffold)
    ctl.aggregate_fn = fn
    out = ctl.aggregate(_results())
    assert calls == [2]
    assert np.array_equal(out.params["w"], np.full(3, 7.0, np.float32))


def test_default_aggregate_fn_runs_on_the_device():
    ctl = _ctl(Scaffold)
    out = ctl.aggregate(_results())
    assert np.array_equal(out.params["w"], np.full(3, 1.5, np.float32))
