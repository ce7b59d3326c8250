"""bench.py's default run at N = 1 -- the line the driver records every round -- on the fake device:
besides config 3 (the value) it carries config 2 device-resident, config 5 with the FedOpt hand-out pull timed, and,
because config 4 does not fit one GPU, ONE GPU's share of the 8-GPU split of config 4 labelled as the share (instead of
a skip); the CPU baseline runs after every GPU entry, and every entry records the GPU state it ran at (here: not
available, the fake device has no GPU)."""

import contextlib
import io
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from bench_fake_rank import install, small_presets  # noqa: E402


@pytest.fixture
def undo_install(monkeypatch):
    """install() patches bench, torch.cuda and DeviceContext for the whole process: have monkeypatch put every one back
    after the test (other tests in this process parse bench's real presets)."""
    import torch

    import bench
    from nvflare_amd import device as device_mod

    monkeypatch.setattr(bench, "PRESETS", dict(bench.PRESETS))
    for name in ("dist_setup", "make_host_helper", "run_client_sharded"):
        monkeypatch.setattr(bench, name, getattr(bench, name))
    for name in ("synchronize", "empty_cache"):
        monkeypatch.setattr(torch.cuda, name, getattr(torch.cuda, name))
    monkeypatch.setattr(device_mod.DeviceContext, "get", device_mod.DeviceContext.__dict__["get"])
    threads = torch.get_num_threads()  # install() runs torch on one thread
    yield
    torch.set_num_threads(threads)


@pytest.mark.timeout(300)
def test_default_run_at_one_gpu(monkeypatch, undo_install):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    bench = install(0, 1)
    monkeypatch.setattr(bench, "dist_setup", lambda args: (1, 0, 0))
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(0)
    # room for every preset but config 4's 256-client slab (as one MI355X holds configs 2, 3, 5 but not config 4)
    monkeypatch.setattr(ctx, "total_bytes", bench.HEADROOM + (8 << 20))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--steps", "2", "--warmup", "1", "--host-resident-params", "10001", "--spot-check", "64",
                    "--cpu-baseline-s", "0.2", "--cpu-sample-params", "4096"])
    lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    small = small_presets(1)
    assert d["n_gpus"] == 1 and d["spot_check"]["mismatches"] == 0

    def name(e):
        return e.get("baseline_config") or e["config"]["baseline_config"]

    names = [name(e) for e in d["also"]]
    # 2h / 2s / 4x: 2s and 4x skip at one GPU (nothing to split / exchange); every device-resident entry is measured
    measured = [e for e in d["also"] if "roofline" in e]
    assert len(measured) == 3, names
    c2 = next(e for e in measured if e["config"]["clients"] == small[2]["clients"])
    assert c2["config"]["params_total"] == small[2]["params"] and c2["spot_check"]["mismatches"] == 0
    c4 = next(e for e in measured if e["config"]["clients"] == small[4]["clients"])
    from nvflare_amd.sharding import bucket_ranges

    lo, hi = max(bucket_ranges(small[4]["params"], 8), key=lambda b: b[1] - b[0])
    assert "ONE GPU's share of the 8-GPU split" in name(c4)
    assert c4["config"]["share"] == {"of_params_total": small[4]["params"], "gpus": 8, "bucket": [lo, hi]}
    assert c4["config"]["params_total"] == hi - lo and c4["spot_check"]["mismatches"] == 0
    assert c4["value"] == pytest.approx(4.0 * small[4]["clients"] * (hi - lo) / (c4["ms_per_step"] / 1e3) / 2**30,
                                        rel=2e-3, abs=0.006)
    c5 = next(e for e in measured if e["config"]["epilogue"] == "adam")
    assert c5["handout_pull"]["bytes_per_gpu_rank0"] == 4 * small[5]["params"]
    assert not any("skipped" in e and "config 4" in name(e) and "client-sharded" not in name(e) for e in d["also"])
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["n_gpus_in_run"] == 1
    assert set(d["gpu_state"]) == {"before", "main_timed", "after"}
