"""The 2s entry's deployment -- ONE server process whose drop-in helper splits every key over all the node's GPUs
(WeightedAggregationHelper(devices=[0..7]), nvflare_amd/sharding.py) -- rehearsed on eight fake devices (VERDICT r05
item 7): every device stages its bucket of every client from the shard pool's own threads, in parallel, and the
assembled result is the oracle's bit for bit; and a device whose staging never returns ends bench.py's 2s entry through
the watchdog (the line measured so far printed, the entry marked timed out, every rank exits), not a hang."""

import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from fake_device import FakeDeviceContext  # noqa: E402

T = 4096


def _sharded_helper(devices):
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper
    from nvflare_amd.sharding import ShardedFedAvg

    h = WeightedAggregationHelper(devices=devices)
    old = h._engine
    sh = ShardedFedAvg(list(devices))
    for eng in sh.engines:
        eng._ctx = FakeDeviceContext()
    h._engine = sh
    if hasattr(old, "release"):
        old.release()
    return h, sh


def test_eight_devices_stage_in_parallel_and_match_the_oracle(oracle):
    h, sh = _sharded_helper(list(range(8)))
    seen = {}  # bucket -> thread names that staged into it
    lock = threading.Lock()
    for b, eng in enumerate(sh.engines):
        ctx = eng._ctx
        for name in ("h2d_tiled_multi", "h2d_ptr", "h2d"):
            orig = getattr(ctx, name)

            def wrapped(*a, _orig=orig, _b=b, **k):
                with lock:
                    seen.setdefault(_b, set()).add(threading.current_thread().name)
                time.sleep(0.002)  # long enough for the eight staging threads to overlap
                return _orig(*a, **k)

            setattr(ctx, name, wrapped)
    K, P = 8, 8 * 3 * T + 123  # every bucket non-empty, a ragged last one
    rng = np.random.default_rng(5)
    clients = [rng.standard_normal(P).astype(np.float32) for _ in range(K)]
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    for k in range(K):
        h.add({"w": clients[k]}, ws[k], f"site-{k}", 0)
    got = h.get_result()["w"]
    want = oracle.fedavg_c(clients, ws, oracle.MODE_NUMPY)
    assert np.asarray(got).view(np.uint32).tolist() == want.view(np.uint32).tolist()
    assert sorted(seen) == list(range(8))  # every device staged its bucket
    names = set().union(*seen.values())
    assert all(n.startswith("nvflare-amd-shard") for n in names), names
    assert len(names) >= 2  # the buckets were staged from several pool threads at once


@pytest.mark.timeout(300)
def test_a_stalled_device_ends_the_2s_entry_through_the_watchdog(tmp_path):
    env = dict(os.environ, NVFLARE_AMD_BENCH_WORKER_SCRIPT=os.path.join(ROOT, "tests", "bench_fake_rank.py"),
               NVFLARE_AMD_FAKE_STALL_DEVICE="3", NVFLARE_AMD_BENCH_GPU_STATE="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1",
                        "--host-resident-params", "40001", "--spot-check", "64", "--watchdog-s", "8",
                        "--cpu-baseline-s", "0.2", "--cpu-sample-params", "4096"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert time.monotonic() - t0 < 200
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    d = json.loads(lines[0])
    s2 = [e for e in d["also"] if "one process over all GPUs" in (e.get("baseline_config") or "")]
    assert len(s2) == 1 and "watchdog" in s2[0].get("error", ""), d["also"]
    # the entries before it were measured and kept
    assert any("host-resident updates" in (e.get("baseline_config") or "") for e in d["also"])
