"""bench.py's client-sharded entry under its watchdog (CPU; the measurement itself is stubbed): a stuck exchange
ends the process with the line measured so far printed once, an exception becomes an error entry, and a line
already printed is not printed again."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUCK = r"""
import sys, time
sys.path.insert(0, {root!r})
import bench
bench.run_client_sharded = lambda *a, **k: time.sleep(30)
args = bench.parse(["--also", "4x", "--watchdog-s", "0.3"])
line, also, state = {{"metric": "m", "value": 1.0}}, [], {{"printed": {printed}}}
bench.client_sharded_entry(args, 2, 0, 0, line, also, state)
print("NOT REACHED")
"""


def _run(printed):
    p = subprocess.run([sys.executable, "-c", STUCK.format(root=ROOT, printed=printed)], capture_output=True,
                       text=True, timeout=60)
    return p.returncode, [ln for ln in p.stdout.splitlines() if ln.strip()]


def test_stuck_entry_prints_line_once_and_exits():
    rc, out = _run(False)
    assert rc == 0 and len(out) == 1, out
    d = json.loads(out[0])
    assert d["value"] == 1.0 and "watchdog" in d["also"][0]["error"]


def test_stuck_teardown_after_print_does_not_print_again():
    rc, out = _run(True)
    assert rc == 0 and out == []


def test_exception_becomes_error_entry():
    sys.path.insert(0, ROOT)
    import bench

    def boom(*a, **k):
        raise RuntimeError("exchange failed")

    saved = bench.run_client_sharded
    bench.run_client_sharded = boom
    try:
        args = bench.parse(["--also", "4x", "--watchdog-s", "30"])
        also = []
        failed, dog = bench.client_sharded_entry(args, 2, 0, 0, {}, also, {})
        dog.cancel()
    finally:
        bench.run_client_sharded = saved
    assert failed is False and "RuntimeError: exchange failed" in also[0]["error"]


def test_host_resident_entry_on_fake_device(monkeypatch):
    """The 2h entry (config 2 from pageable host arrays to a host result through the drop-in helper) on the fake
    device: every element of the result is compared with the oracle, and the summary carries the PCIe-inclusive
    fields."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    from fake_device import fake_engine

    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    def helper(local):
        h = WeightedAggregationHelper(device=local)
        h._engine = fake_engine()
        return h

    monkeypatch.setattr(bench, "make_host_helper", helper)
    args = bench.parse(["--also", "2h", "--host-resident-params", "10001", "--steps", "2", "--warmup", "1"])
    also = []
    failed, dog = bench.guarded_entry(args, 1, 0, 0, {}, also, {}, bench.HOST_RESIDENT)
    dog.cancel()
    e = also[0]
    assert failed is False, e
    assert e["spot_check"]["compared"] == 10001 and e["spot_check"]["mismatches"] == 0
    assert e["steps"] == 2 and e["config"]["clients"] == 8 and e["value"] > 0
    assert "host-resident" in e["baseline_config"] and "custom" in e["baseline_config"]


def test_host_sharded_entry_needs_two_gpus_and_summarises_strong():
    """The 2s entry (one process over all N GPUs' buckets) skips at N = 1; its summary counts the model once."""
    sys.path.insert(0, ROOT)
    import bench

    args = bench.parse(["--also", "2s", "--host-resident-params", "10001"])
    also = []
    failed, dog = bench.guarded_entry(args, 1, 0, 0, {}, also, {}, bench.HOST_SHARDED)
    dog.cancel()
    assert failed is False and "needs >= 2 GPUs" in also[0]["skipped"]
    r = {"K": 8, "P": 1000, "wall": 0.5, "steps": 5, "warmup": 3, "sharded": True, "accept_s": 0.08, "drain_s": 0.005,
         "result_type": "ndarray", "devices": 4, "spot_check": None}
    e = bench.summarize_host_resident(args, 4, r)
    assert e["scaling"] == "strong" and e["config"]["devices"] == 4 and e["config"]["params_total"] == 1000
    assert abs(e["value"] - 4.0 * 8 * 1000 / 0.1 / 2**30) < 0.01
    r["sharded"] = False
    assert abs(bench.summarize_host_resident(args, 4, r)["value"] - 4 * 4.0 * 8 * 1000 / 0.1 / 2**30) < 0.01
