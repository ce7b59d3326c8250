"""The reference's OWN unit tests for the aggregation path, run against the drop-in (CPU, fake device).

Runs ``tests/unit_test/app_common/aggregators/{in_time_accumulate_weighted_aggregator,weighted_aggregation_
helper}_test.py`` from the mounted reference tree (NVFlare, read in place, nothing copied) in a subprocess,
with tests/ref_suite_plugin.py binding the real NVFlare API classes and swapping the reference's aggregator /
helper for the drop-in's; the device is tests/fake_device.py (the kernels' per-element sequence restated by
the oracle), so this checks the drop-in's API, validation, bookkeeping and stats against the reference's
own expectations -- the kernels themselves are checked on the GPU (tests/test_gpu_*.py).  Skipped where the
reference tree is absent (e.g. on the GPU box)."""

import json
import os
import subprocess
import sys
import xml.etree.ElementTree as ET

import pytest

REF = os.environ.get("NVFLARE_REF_ROOT", "/root/reference")
SUITE = [os.path.join(REF, "tests/unit_test/app_common/aggregators", f)
         for f in ("in_time_accumulate_weighted_aggregator_test.py", "weighted_aggregation_helper_test.py")]
HERE = os.path.dirname(os.path.abspath(__file__))
FEDAVG_WORKFLOW = os.path.join(REF, "tests/unit_test/app_common/workflow/fedavg_test.py")


def _run(tmp_path, files, swap, tag):
    report = tmp_path / f"report_{tag}.json"
    junit = tmp_path / f"junit_{tag}.xml"
    env = dict(os.environ, NVFLARE_REF_ROOT=REF, PYTHONDONTWRITEBYTECODE="1", FEDAVG_REF_SUITE_REPORT=str(report),
               FEDAVG_REF_SUITE_SWAP="1" if swap else "0", PYTHONPATH=os.pathsep.join([HERE, os.path.dirname(HERE)]))
    env.pop("NVFLARE_AMD_FORCE_STANDINS", None)
    proc = subprocess.run([sys.executable, "-m", "pytest", "-p", "ref_suite_plugin", "-p", "no:cacheprovider",
                           f"--rootdir={tmp_path}", f"--junitxml={junit}", "-q", *files], cwd=str(tmp_path), env=env,
                          capture_output=True, text=True, timeout=600)
    outcomes = {}
    for case in ET.parse(junit).getroot().iter("testcase"):
        status = "passed"
        for child in case:
            if child.tag in ("failure", "error"):
                status = "failed"
            elif child.tag == "skipped":
                status = "skipped"
        outcomes[f"{case.get('classname')}::{case.get('name')}"] = status
    return proc, json.loads(report.read_text()), outcomes


@pytest.mark.skipif(not all(os.path.exists(p) for p in SUITE), reason="reference tree not mounted")
def test_reference_unit_tests_pass_against_dropin(tmp_path):
    proc, rep, outcomes = _run(tmp_path, SUITE, True, "aggregators")
    tail = (proc.stdout + proc.stderr)[-3000:]
    assert proc.returncode == 0, tail
    assert any(s.endswith(".InTimeAccumulateWeightedAggregator") for s in rep["swapped"]), rep
    assert any(s.endswith(".WeightedAggregationHelper") for s in rep["swapped"]), rep
    assert rep["launches"] > 0, rep  # the drop-in's engine did the aggregation
    assert len(outcomes) >= 79 and set(outcomes.values()) == {"passed"}, tail


@pytest.mark.skipif(not os.path.exists(FEDAVG_WORKFLOW), reason="reference tree not mounted")
def test_reference_fedavg_workflow_tests_same_outcome(tmp_path):
    """workflow/fedavg_test.py with the drop-in helper inside the reference FedAvg controller (fedavg.py:205):
    every test ends exactly as it does for the reference itself (10 of them fail in this container for both,
    on ``cryptography`` imports outside the aggregation path -- SURVEY.md section 8c)."""
    _, _, ref = _run(tmp_path, [FEDAVG_WORKFLOW], False, "ref")
    _, rep, ours = _run(tmp_path, [FEDAVG_WORKFLOW], True, "dropin")
    assert any("workflows.fedavg.WeightedAggregationHelper" in s for s in rep["swapped"]), rep
    assert "nvflare.app_common.workflows.scaffold.scaffold_aggregate_fn" in rep["swapped"], rep
    assert "nvflare.app_common.workflows.scaffold.Scaffold" in rep["swapped"], rep
    assert sum("TestScaffold" in k and v == "passed" for k, v in ours.items()) >= 8, ours
    assert ours == ref
    assert sum(v == "passed" for v in ours.values()) >= 100


FEDAVG_LR = os.path.join(REF, "tests/unit_test/app_common/workflow/fedavg_lr_test.py")


@pytest.mark.skipif(not os.path.exists(FEDAVG_LR), reason="reference tree not mounted")
def test_reference_fedavg_lr_tests_same_outcome(tmp_path):
    """workflow/fedavg_lr_test.py with the drop-in helper as FedAvgLR's aggregator (lr/fedavg.py:45,157-164;
    fp64 gradient / Hessian keys through the engine's fp64 arena): every test ends as it does for the
    reference."""
    _, _, ref = _run(tmp_path, [FEDAVG_LR], False, "ref")
    _, rep, ours = _run(tmp_path, [FEDAVG_LR], True, "dropin")
    assert "nvflare.app_common.workflows.lr.fedavg.FedAvgLR(aggregator=)" in rep["swapped"], rep
    assert rep["launches"] > 0, rep
    assert ours == ref
    assert sum(v == "passed" for v in ours.values()) >= 20, ours


FEDOPT_CTL = os.path.join(REF, "nvflare/app_opt/pt/fedopt_ctl.py")

_COMPOSE = r"""
import os, sys
sys.dont_write_bytecode = True
from ref_suite_plugin import _install_shim
_install_shim(os.environ["NVFLARE_REF_ROOT"])
import nvflare_amd.compat as compat
assert compat.HAVE_NVFLARE
from nvflare.app_opt.pt.fedopt_ctl import FedOpt as Ref
from nvflare_amd.app_opt.pt.fedopt_ctl import DeviceFedOptUpdate, FedOpt
assert issubclass(FedOpt, Ref) and issubclass(FedOpt, DeviceFedOptUpdate)
assert FedOpt.update_model is DeviceFedOptUpdate.update_model
assert FedOpt.optimizer_update is DeviceFedOptUpdate.optimizer_update
assert FedOpt.run is Ref.run
from nvflare.app_common.workflows import scaffold as ref_scaffold
from nvflare_amd.app_common.workflows import scaffold as dropin_scaffold
assert issubclass(dropin_scaffold.Scaffold, ref_scaffold.Scaffold)
assert dropin_scaffold._reference_scaffold_fn is ref_scaffold.scaffold_aggregate_fn
ctl = dropin_scaffold.Scaffold(num_clients=2, num_rounds=1, aggregation_device=0)
seen = []
ctl._device_scaffold_fn = lambda results: seen.append("scaffold")
ctl._device_fedavg_fn = lambda results: seen.append("fedavg")
import nvflare.app_common.workflows.base_fedavg as bf
bf.BaseFedAvg.aggregate = lambda self, results, aggregate_fn=None: aggregate_fn(results)
ctl.aggregate([], aggregate_fn=ref_scaffold.scaffold_aggregate_fn)
ctl.aggregate([])
mine = lambda results: seen.append("own")
ctl.aggregate([], aggregate_fn=mine)
assert seen == ["scaffold", "fedavg", "own"], seen
print("composed")
"""


@pytest.mark.skipif(not os.path.exists(FEDOPT_CTL), reason="reference tree not mounted")
def test_fedopt_controller_composes_with_reference_controller():
    """With the real nvflare importable, the drop-in FedOpt controller IS the reference controller (its run(),
    FedAvg rounds, constructor) with the device server step in place of optimizer_update / update_model; the
    drop-in Scaffold controller routes the reference's aggregation functions (and only those) to the device."""
    env = dict(os.environ, NVFLARE_REF_ROOT=REF, PYTHONDONTWRITEBYTECODE="1",
               PYTHONPATH=os.pathsep.join([HERE, os.path.dirname(HERE)]))
    env.pop("NVFLARE_AMD_FORCE_STANDINS", None)
    proc = subprocess.run([sys.executable, "-c", _COMPOSE], env=env, capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0 and "composed" in proc.stdout, (proc.stdout + proc.stderr)[-3000:]


SCAFFOLD_CHECK = os.path.join(HERE, "ref_scaffold_override_check.py")


@pytest.mark.skipif(not os.path.exists(FEDAVG_WORKFLOW), reason="reference tree not mounted")
def test_dropin_scaffold_keeps_subclass_aggregate_fn(tmp_path):
    """The drop-in Scaffold under the real NVFlare classes: a subclass's own or an instance-level aggregate_fn runs as given, the
    reference's default goes to the device (tests/ref_scaffold_override_check.py)."""
    proc, _, outcomes = _run(tmp_path, [SCAFFOLD_CHECK], True, "scaffold_override")
    assert proc.returncode == 0, (proc.stdout + proc.stderr)[-3000:]
    assert len(outcomes) == 3 and set(outcomes.values()) == {"passed"}, outcomes
