"""pytest plugin (TEST INFRASTRUCTURE): run the REFERENCE's own unit tests for the aggregation path against the
drop-in classes, on the CPU, with ``tests/fake_device.FakeDeviceContext`` standing in for the MI355X.

Used only by tests/test_cpu_reference_suite.py in the build container, where the reference tree is mounted
(NVFLARE_REF_ROOT); nothing of it is copied.  ``nvflare`` is imported through the same namespace shim as
tests/golden/make_golden.py (``import nvflare`` itself needs ``cryptography``), so the drop-in's compat layer
binds the REAL NVFlare DXO / Shareable / FLContext / Aggregator classes.  Each collected test module then sees
the drop-in's ``InTimeAccumulateWeightedAggregator`` / ``WeightedAggregationHelper`` / ``AggregationStatsKey``
/ metric helpers in place of the reference's."""

import os
import sys
import types

sys.dont_write_bytecode = True  # the reference tree is read-only input: never leave __pycache__ in it

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _install_shim(ref_root: str) -> None:
    for name, sub in (("nvflare", "nvflare"), ("nvflare.app_opt", "nvflare/app_opt"), ("nvflare.app_opt.pt", "nvflare/app_opt/pt")):
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.__path__ = [os.path.join(ref_root, sub)]
            sys.modules[name] = m
    if ref_root not in sys.path:
        sys.path.insert(0, ref_root)


def _swapping() -> bool:
    return os.environ.get("FEDAVG_REF_SUITE_SWAP", "1") == "1"  # 0: run the reference as is (baseline)


def pytest_configure(config):
    _install_shim(os.environ["NVFLARE_REF_ROOT"])
    config._fedavg_swapped = []
    config._fedavg_fake = None
    if not _swapping():
        return
    for p in (REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import nvflare_amd.compat as compat
    import nvflare_amd.device as device
    from fake_device import FakeDeviceContext

    assert compat.HAVE_NVFLARE, "the drop-in must bind the real NVFlare classes here"
    fake = FakeDeviceContext()
    device.DeviceContext.get = classmethod(lambda cls, d=None: fake)
    config._fedavg_fake = fake


def pytest_collection_modifyitems(session, config, items):
    if not _swapping():
        return
    from nvflare_amd.app_common.aggregators import intime_accumulate_model_aggregator as intime
    from nvflare_amd.app_common.aggregators import weighted_aggregation_helper as wah

    swap = {
        "InTimeAccumulateWeightedAggregator": intime.InTimeAccumulateWeightedAggregator,
        "WeightedAggregationHelper": wah.WeightedAggregationHelper,
        "AggregationStatsKey": wah.AggregationStatsKey,
        "_is_aggregatable_metric_value": wah._is_aggregatable_metric_value,
        "filter_aggregatable_metrics": wah.filter_aggregatable_metrics,
    }
    mods = {item.module for item in items if getattr(item, "module", None) is not None}
    # the reference FedAvg controller builds its in-time helper from its own module namespace (fedavg.py:205)
    for name in ("nvflare.app_common.workflows.fedavg", "nvflare.app_common.workflows.base_fedavg"):
        if name in sys.modules:
            mods.add(sys.modules[name])
    for mod in mods:
        for name, obj in swap.items():
            if hasattr(mod, name):
                setattr(mod, name, obj)
                config._fedavg_swapped.append(f"{mod.__name__}.{name}")
    # FedAvgLR takes its helper as a constructor default built at import (lr/fedavg.py:45): the drop-in
    # usage is ``FedAvgLR(aggregator=WeightedAggregationHelper(...))``; here the default itself is swapped
    lr = sys.modules.get("nvflare.app_common.workflows.lr.fedavg")
    if lr is not None:
        init = lr.FedAvgLR.__init__
        defaults = tuple(wah.WeightedAggregationHelper() if type(d).__name__ == "WeightedAggregationHelper" else d
                         for d in init.__defaults__)
        if defaults != init.__defaults__:
            init.__defaults__ = defaults
            config._fedavg_swapped.append("nvflare.app_common.workflows.lr.fedavg.FedAvgLR(aggregator=)")
    # the reference's SCAFFOLD tests import ``Scaffold`` / ``scaffold_aggregate_fn`` from the workflow module
    # inside each test (fedavg_test.py:1098-1700): swap the module's names for the drop-in's
    try:
        import nvflare.app_common.workflows.scaffold as ref_scaffold
    except Exception:  # a reference without the FLModel SCAFFOLD workflow
        ref_scaffold = None
    if ref_scaffold is not None:
        from nvflare_amd.app_common.workflows import scaffold as dropin_scaffold

        for name in ("Scaffold", "scaffold_aggregate_fn"):
            setattr(ref_scaffold, name, getattr(dropin_scaffold, name))
            config._fedavg_swapped.append(f"{ref_scaffold.__name__}.{name}")


def pytest_sessionfinish(session, exitstatus):
    """Evidence for the outer test: which names were swapped and how many fake-device launches ran."""
    out = os.environ.get("FEDAVG_REF_SUITE_REPORT")
    if out:
        import json

        cfg = session.config
        with open(out, "w") as f:
            json.dump({"swapped": cfg._fedavg_swapped,
                       "launches": len(cfg._fedavg_fake.launches) if cfg._fedavg_fake is not None else 0,
                       "exitstatus": int(exitstatus)}, f)
