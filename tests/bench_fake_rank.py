"""One rank of bench.main() on the fake device (test infrastructure, CPU only): the stubs the N-rank rehearsals install
in every rank process before calling bench.main() -- tests/test_cpu_bench_world8.py (ranks started by the test, env
set by it) and tests/test_cpu_bench_spawn.py (ranks started by bench.py's own launch_ranks, env set by it; this file
is then the rank's script, NVFLARE_AMD_BENCH_WORKER_SCRIPT).

The kernels are restated by the oracle (fake_device.FakeBenchContext), the BASELINE presets are shrunk so the oracle
finishes in seconds, every process group is gloo, and the client-sharded (4x) entry's collectives run through a
stand-in with the same call sequence (its exchange is tests/test_cpu_client_shards.py's)."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T = 4096


def small_presets(world):
    return {2: dict(clients=8, params=3 * T + 5, epilogue="none", scaling="weak"),
            3: dict(clients=64, params=2 * T + 12, epilogue="none", scaling="weak"),
            4: dict(clients=256, params=world * 2 * T + 100, epilogue="none", scaling="strong"),
            5: dict(clients=64, params=world * T + 36, epilogue="adam", scaling="strong")}


def install(rank, world):
    """Point bench at the fake device for this rank; returns the bench module."""
    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.setdefault("OMP_NUM_THREADS", "1")
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
        assert int(os.environ["WORLD_SIZE"]) == world and int(os.environ["RANK"]) == rank
        dist.init_process_group(backend="gloo")
        return world, rank, rank

    def make_host_helper(local, devices=None):
        if devices:
            h = WeightedAggregationHelper(devices=devices)
            old = h._engine
            sh = ShardedFedAvg(list(devices))
            for eng in sh.engines:
                eng._ctx = FakeDeviceContext()
            stall = os.environ.get("NVFLARE_AMD_FAKE_STALL_DEVICE")  # tests/test_cpu_host_sharded8.py: a device whose
            if stall is not None:  # staging copies never return (the 2s entry must end through the watchdog)
                import time

                def stalled(*a, **k):
                    time.sleep(3600)

                ctx_ = sh.engines[int(stall)]._ctx
                ctx_.h2d_tiled_multi = ctx_.h2d_ptr = ctx_.h2d = stalled
            h._engine = sh
            if hasattr(old, "release"):
                old.release()
            return h
        h = WeightedAggregationHelper(device=local)
        h._engine = fake_engine()
        return h

    def run_client_sharded(args, world_, rank_, local, K, P, seed):
        """The 4x entry's collectives (fit vote, barriers, max / sum over ranks) with stand-in device times."""
        from nvflare_amd.client_shards import ExchangePlan

        clients = [len(range(s, K, world_)) for s in range(world_)]
        plan = ExchangePlan(P, clients)
        if bench.sum_over_ranks(world_, [0])[0]:
            return {"skipped": "does not fit"}
        steps, warmup = max(1, min(args.steps, 5)), max(1, min(args.warmup, 1))
        bench.dist_barrier(world_)
        wall = bench.max_over_ranks(world_, 1e-3 * steps)
        sampled, mism, differ = bench.sum_over_ranks(world_, [10, 0, 0])
        return {"K": K, "P": plan.bucket_len(rank_), "P_total": P, "wall": wall, "steps": steps, "warmup": warmup,
                "kernel_ms": 0.5, "all_to_all_ms": 1.0, "overlapped_ms": 1.1,
                "all_to_all_bytes_out_rank0": 4.0 * (sum(plan.send_splits(rank_)) - plan.send_splits(rank_)[rank_]),
                "bits_equal_serial": differ == 0,
                "spot_check": {"sampled": sampled, "mismatches": mism + differ, "ranks": world_, "oracle": "stand-in"},
                "clients_per_rank": clients, "max_peer_bytes": 1 << 28, "min_kernel_tiles": 2048}

    bench.dist_setup = dist_setup
    bench.make_host_helper = make_host_helper
    bench.run_client_sharded = run_client_sharded
    bench.PRESETS.clear()
    bench.PRESETS.update(small_presets(world))
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.empty_cache = lambda *a, **k: None
    device_mod.DeviceContext.get = classmethod(lambda cls, device=None: ctx)
    return bench


if __name__ == "__main__":  # a rank started by bench.launch_ranks: the env carries RANK / WORLD_SIZE / MASTER_*
    _bench = install(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]))
    _bench.main(sys.argv[1:])
