"""bench.py's default run at N = 8 -- the line the driver's first 8-GPU scaling run prints -- rehearsed on the CPU
(VERDICT r03 item 4): eight gloo ranks run ``bench.main()`` with every default ``also`` entry on the fake device
(tests/fake_device.FakeBenchContext: the kernels restated by the oracle), the BASELINE presets shrunk so the oracle
finishes in seconds.  The line's structure is what is checked: config 3's value counts 4 K P N (weak), configs 5 and
4 split one model into eight buckets (strong), 2h / 2s / 4x are present, spot checks are summed over the ranks, and
every entry's spot check is clean.  The client-sharded (4x) measurement itself needs HIP streams; its collectives
run here through a stand-in with the same call sequence (the exchange is tests/test_cpu_client_shards.py's)."""

import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 8
T = 4096
SMALL = {2: dict(clients=8, params=3 * T + 5, epilogue="none", scaling="weak"),
         3: dict(clients=64, params=2 * T + 12, epilogue="none", scaling="weak"),
         4: dict(clients=256, params=WORLD * 2 * T + 100, epilogue="none", scaling="strong"),
         5: dict(clients=64, params=WORLD * T + 36, epilogue="adam", scaling="strong")}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD), RANK=str(rank),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import contextlib
    import io

    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    import bench
    from fake_device import FakeBenchContext, FakeDeviceContext, fake_engine

    from nvflare_amd import device as device_mod
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper
    from nvflare_amd.sharding import ShardedFedAvg

    ctx = FakeBenchContext(device=rank)

    def dist_setup(args):
        dist.init_process_group(backend="gloo")
        return WORLD, rank, rank

    def make_host_helper(local, devices=None):
        if devices:
            h = WeightedAggregationHelper(devices=devices)
            old = h._engine
            sh = ShardedFedAvg(list(devices))
            for eng in sh.engines:
                eng._ctx = FakeDeviceContext()
            h._engine = sh
            if hasattr(old, "release"):
                old.release()
            return h
        h = WeightedAggregationHelper(device=local)
        h._engine = fake_engine()
        return h

    def run_client_sharded(args, world, rank_, local, K, P, seed):
        """The 4x entry's collectives (fit vote, barriers, max / sum over ranks) with stand-in device times."""
        from nvflare_amd.client_shards import ExchangePlan

        clients = [len(range(s, K, world)) for s in range(world)]
        plan = ExchangePlan(P, clients)
        if bench.sum_over_ranks(world, [0])[0]:
            return {"skipped": "does not fit"}
        steps, warmup = max(1, min(args.steps, 5)), max(1, min(args.warmup, 1))
        bench.dist_barrier(world)
        wall = bench.max_over_ranks(world, 1e-3 * steps)
        sampled, mism, differ = bench.sum_over_ranks(world, [10, 0, 0])
        return {"K": K, "P": plan.bucket_len(rank_), "P_total": P, "wall": wall, "steps": steps, "warmup": warmup,
                "kernel_ms": 0.5, "all_to_all_ms": 1.0, "overlapped_ms": 1.1,
                "all_to_all_bytes_out_rank0": 4.0 * (sum(plan.send_splits(rank_)) - plan.send_splits(rank_)[rank_]),
                "bits_equal_serial": differ == 0,
                "spot_check": {"sampled": sampled, "mismatches": mism + differ, "ranks": world, "oracle": "stand-in"},
                "clients_per_rank": clients, "max_peer_bytes": 1 << 28, "min_kernel_tiles": 2048}

    bench.dist_setup = dist_setup
    bench.make_host_helper = make_host_helper
    bench.run_client_sharded = run_client_sharded
    bench.PRESETS.clear()
    bench.PRESETS.update(SMALL)
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.empty_cache = lambda *a, **k: None
    device_mod.DeviceContext.get = classmethod(lambda cls, device=None: ctx)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--gpus", str(WORLD), "--steps", "2", "--warmup", "1", "--host-resident-params", "10001",
                    "--spot-check", "64"])
    with open(os.path.join(out_dir, f"rank{rank}.out"), "w") as f:
        f.write(buf.getvalue())


@pytest.mark.timeout(600)
def test_default_run_at_eight_ranks(tmp_path):
    port = _free_port()
    mp.start_processes(_rank, args=(port, str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    outs = [open(tmp_path / f"rank{r}.out").read() for r in range(WORLD)]
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and all(not o.strip() for o in outs[1:]), outs
    d = json.loads(lines[0])
    K3, P3 = SMALL[3]["clients"], SMALL[3]["params"]
    assert d["n_gpus"] == WORLD and d["scaling"] == "weak" and d["steps"] == 2
    # value = 4 K P N steps / wall: weak scaling counts every rank's own P-param bucket
    wall = d["ms_per_step"] / 1e3
    assert d["value"] == pytest.approx(4.0 * K3 * P3 * WORLD / wall / 2**30, rel=2e-3, abs=0.006)
    assert d["spot_check"]["mismatches"] == 0 and d["spot_check"]["ranks"] == WORLD
    assert d["spot_check"]["sampled"] >= WORLD * 64
    def name(e):
        return e.get("baseline_config") or e["config"]["baseline_config"]

    assert len(d["also"]) == 5, [name(e) for e in d["also"]]
    assert not any("skipped" in e or "error" in e for e in d["also"]), d["also"]
    c5 = next(e for e in d["also"] if e["config"].get("epilogue") == "adam")
    c4 = next(e for e in d["also"] if e["config"].get("clients") == 256 and "client-sharded" not in name(e))
    for e, cfg in ((c5, SMALL[5]), (c4, SMALL[4])):  # strong: one model split into eight buckets, counted once
        assert e["scaling"] == "strong" and e["n_gpus"] == WORLD
        assert e["config"]["params_total"] == cfg["params"]
        assert e["spot_check"]["mismatches"] == 0 and e["spot_check"]["ranks"] == WORLD
        assert e["value"] == pytest.approx(4.0 * cfg["clients"] * cfg["params"] / (e["ms_per_step"] / 1e3) / 2**30,
                                           rel=2e-3, abs=0.006)
    h2 = [e for e in d["also"] if "host-resident updates" in name(e)]
    s2 = [e for e in d["also"] if "ONE server process" in name(e)]
    x4 = [e for e in d["also"] if "client-sharded" in name(e)]
    assert len(h2) == len(s2) == len(x4) == 1, [name(e) for e in d["also"]]
    assert h2[0]["scaling"] == "weak" and h2[0]["spot_check"]["mismatches"] == 0 and h2[0]["spot_check"]["ranks"] == WORLD
    assert s2[0]["scaling"] == "strong" and s2[0]["config"]["devices"] == WORLD and s2[0]["spot_check"]["mismatches"] == 0
    assert x4[0]["spot_check"]["ranks"] == WORLD and x4[0]["bits_equal_serial"]
