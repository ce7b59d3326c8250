#!/usr/bin/env python3
"""Benchmark of the MI355X FedAvg weighted aggregation (BASELINE.json metric).

One step = one aggregation: the arrival-ordered weighted accumulate-and-finalise kernel over K
device-resident client rows of P fp32 params -> P fp32 results (weighted_aggregation_helper.py:153-240,
torch-mode arithmetic by default).  Inputs are resident in HBM before the timed region starts.

  python bench.py [--gpus N --steps K --warmup W]          # default: 64 clients x 1e9 params, 1 GPU
  torchrun --nproc-per-node N bench.py --gpus N ...        # weak scaling: each GPU aggregates its own
                                                           # 1e9-param bucket, no data-path collective

Prints ONE JSON line (rank 0).  value = GiB/s aggregated = 4*K*P*N*steps / t / 2^30 with t the max over
ranks of the barrier+synchronize bracketed wall time.  roofline.achieved uses the algorithmic bytes of one
aggregation (4*K*P + 4*P) over its device time measured with HIP events on the stream the kernels run on
(one aggregation = roofline.launches_per_step launches of the burst kernel; launch_us_avg is the
per-launch time a rocprofv3 --stats average compares with).  cpu_baseline times the oracle restatement
(torch CPU ops, all threads) on a bounded sample of the same workload, and the same leg spot-checks
sampled device outputs bit-exactly against the oracle (test infrastructure; never the measured path).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "GiB/s aggregated (device-resident FedAvg, K clients × P fp32 params); % HBM peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=float, default=1e9, help="fp32 params per GPU bucket")
    ap.add_argument("--mode", choices=["torch", "numpy"], default="torch")
    ap.add_argument("--blocks-per-cu", type=int, default=0,
                    help="0 = library default (burst kernel: 1 at >= 32 clients, else 2; fused: 1 at >= 64)")
    ap.add_argument("--unroll", type=int, default=0, help="0 = library default (4)")
    ap.add_argument("--variant", type=int, default=0,
                    help="kernel variant bits (include/nvflare_amd_fedavg.h fedavg_set_variant; 0 = burst kernel)")
    ap.add_argument("--tile", type=int, default=4096, help="slab tile width (elements)")
    ap.add_argument("--epilogue", choices=["none", "add_base", "sgd", "adam", "adamax", "nadam", "radam"], default="none",
                    help="fused server update (config 5 = adam: FedOpt Adam on the aggregated deltas)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-params", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--spot-check", type=int, default=4096, help="sampled outputs checked against the oracle")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per launch from a separate rocprofv3 --pmc pass (default: profiles/pmc_traffic.json "
                         "when its config matches this run)")
    ap.add_argument("--seed", type=int, default=1000)
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    if world > 1:
        import torch.distributed as dist

        if os.environ.get("NVFLARE_AMD_BENCH_SHARED_DEVICE") == "1":
            # rehearsal of the multi-rank flow on a one-GPU box: every rank on cuda:0, barriers and the
            # max-over-ranks timing over gloo (RCCL refuses two ranks on one device); never a measurement
            local = 0
            torch.cuda.set_device(0)
            dist.init_process_group(backend="gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    return world, rank, local


def barrier_sync(world, ctx):
    import torch

    ctx.sync()
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(world, value: float) -> float:
    """MAX over ranks (RCCL on GPUs; gloo in the CPU tests).  Timing only -- no data-path collective."""
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(world, values):
    """Element-wise SUM over ranks of a few host integers (spot-check counts)."""
    if world == 1:
        return list(values)
    import torch
    import torch.distributed as dist

    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor(list(values), dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]


def rank_bucket(rank: int, P: int):
    """Weak scaling: rank r aggregates global params [r*P, (r+1)*P) of every client (sharding.bucket_ranges
    with equal per-GPU buckets); returns the generator column offset of the bucket."""
    return rank * P


def cpu_baseline_and_spot_check(args, ctx, K, out_buf, weights, count, P, col0, op, baseline=True):
    """Oracle leg (test infrastructure): time the reference restatement on the host (``baseline``: rank 0 at
    N=1 only), then check sampled device outputs of this rank's bucket bit-for-bit against the oracle computed
    from the host twin of the generator."""
    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import fedavg_oracle as orc

    res = {}
    # -- spot check at full size -----------------------------------------------------------------
    if args.spot_check > 0:
        rng = np.random.default_rng(7)
        idx = np.unique(np.concatenate([rng.integers(0, P, args.spot_check, dtype=np.int64), [0, P - 1]]))
        host_rows = [orc.synth_values(args.seed, k, (idx + col0).astype(np.uint64)) for k in range(K)]
        mode = orc.MODE_TORCH if op == 1 else orc.MODE_NUMPY
        exp = orc.fedavg_c(host_rows, weights, mode)
        got = ctx.gather_f32(out_buf.ptr, idx.astype(np.uint64))
        mism = int(np.count_nonzero(exp.view(np.uint32) != got.view(np.uint32)))
        res["spot_check"] = {"sampled": int(idx.size), "mismatches": mism, "oracle": "oracle/fedavg_oracle.c"}
    # -- CPU baseline: the reference's torch CPU op sequence on a bounded sample ------------------
    if baseline and not args.no_cpu_baseline:
        Ps = int(min(args.cpu_sample_params, P))
        gen = [np.random.default_rng(1000 + k).standard_normal(Ps, dtype=np.float32) for k in range(K)]
        trows = [torch.from_numpy(g) for g in gen]
        threads = torch.get_num_threads()
        reps, t_tot = 0, 0.0
        while t_tot < 10.0 and reps < 2000:
            t0 = time.perf_counter()
            if op == 1:
                orc.torch_mode_reference(trows, weights)
            else:
                orc.numpy_mode_reference(gen, weights)
            t_tot += time.perf_counter() - t0
            reps += 1
        gibs = 4.0 * K * Ps * reps / t_tot / 2**30
        # single-thread numpy restatement (the numpy-job path) for context
        t0 = time.perf_counter()
        orc.numpy_mode_reference(gen, weights)
        t_np = time.perf_counter() - t0
        res["cpu_baseline"] = {
            "value": round(gibs, 3),
            "unit": "GiB/s",
            "cores": threads if op == 1 else 1,
            "kind": "port",
            "sample": f"{K} clients x {Ps} fp32 params (numpy default_rng(1000+k) N(0,1)), "
                      f"{'torch CPU mul/add_(alpha)/div_' if op == 1 else 'numpy v*w / t+v*w / t*(1/c)'} "
                      f"restatement of weighted_aggregation_helper.py:181-236, {reps} reps in {t_tot:.1f}s",
            "numpy_single_thread_GiBs": round(4.0 * K * Ps / t_np / 2**30, 3),
            "host_cpu_count": os.cpu_count(),
            "host_cpu_model": _cpu_model(),
        }
    return res


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(args, K, P):
    """HBM bytes per launch measured by rocprofv3 PMC passes of this same command (profiles/pmc_traffic.json),
    only when that measurement's configuration is this run's."""
    if args.traffic_bytes is not None:
        return args.traffic_bytes, "--traffic-bytes"
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, None
    want = {"clients": K, "params": P, "tile": args.tile, "mode": args.mode, "epilogue": args.epilogue}
    for r in rec.get("records", []):
        cfg = dict(r.get("config", {}))
        cfg.setdefault("epilogue", "none")
        if all(cfg.get(k) == v for k, v in want.items()):
            return float(r["bytes_per_launch"]), "profiles/pmc_traffic.json"
    return None, None


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from nvflare_amd import _native as N
    from nvflare_amd.device import DeviceContext, TiledLayout

    ctx = DeviceContext.get(local)
    ctx.set_launch(args.blocks_per_cu, args.unroll)
    ctx.set_variant(args.variant)
    K = int(args.clients)
    P = int(args.params)
    op = N.FEDAVG_OP_TORCH if args.mode == "torch" else N.FEDAVG_OP_NUMPY
    fin = N.FEDAVG_FIN_DIV if args.mode == "torch" else N.FEDAVG_FIN_SCALE
    col0 = rank_bucket(rank, P)  # weak scaling: rank r owns param bucket [r*P, (r+1)*P)

    free, total = ctx.mem_info()
    lay = TiledLayout(args.tile, K)  # the engine's slab layout: K client slots interleaved per tile
    need = lay.slab_elems(P) * 4 + P * 4
    if need > free:
        raise SystemExit(f"rank {rank}: workload needs {need / 2**30:.1f} GiB, device has {free / 2**30:.1f} GiB free")

    end = (P + 3) // 4 * 4
    slab = ctx.alloc(lay.slab_elems(P) * 4)
    epi_bufs = {"none": 1, "add_base": 1, "sgd": 2}.get(args.epilogue, 3)  # out | p+buf | p+m+v
    state = [ctx.alloc(end * 4) for _ in range(epi_bufs)]
    out = state[0]
    bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]
    for k, base in enumerate(bases):
        ctx.fill_synthetic_f32(base, P, args.seed, k, col0, lay.tile, lay.tile_stride)
    ctx.sync()
    # per-client weights: aggregation_weight 1.0 x NUM_STEPS_CURRENT_ROUND = 1 + (37k mod 100)
    weights = [1.0 * float(1 + (37 * k) % 100) for k in range(K)]
    count = None
    for w in weights:
        count = w if count is None else count + w

    epi = None
    if args.epilogue != "none":
        for j, b in enumerate(state):  # initial params (or base weights), zero optimizer state
            if j == 0:
                ctx.fill_synthetic_f32(b.ptr, end, args.seed + 7, 0, col0)
            else:
                ctx.memset(b.ptr, 0, end * 4)
        epi = N.Epilogue()
        epi.kind = {"add_base": N.FEDAVG_EPI_ADD_BASE, "sgd": N.FEDAVG_EPI_SGD, "adam": N.FEDAVG_EPI_ADAM,
                    "adamax": N.FEDAVG_EPI_ADAMAX, "nadam": N.FEDAVG_EPI_NADAM, "radam": N.FEDAVG_EPI_RADAM}[args.epilogue]
        if args.epilogue == "add_base":
            epi.base = out.ptr
        elif args.epilogue == "sgd":
            epi.param, epi.state1 = state[0].ptr, state[1].ptr
            epi.lr, epi.momentum = 1.0, 0.9
        else:
            epi.param, epi.state1, epi.state2 = state[0].ptr, state[1].ptr, state[2].ptr
            epi.lr, epi.beta1, epi.beta2, epi.eps = 1e-3, 0.9, 0.999, 1e-8
            epi.momentum_decay, epi.mu_product = 4e-3, 1.0  # NAdam (mu_product held at its first-step value)
        ctx.sync()
    n_step = [0]

    def step():
        if epi is None:
            ctx.accumulate_tiled(bases, weights, lay.tile, lay.tile_stride, 0, end, out.ptr, op, fin, count)
            return
        n_step[0] += 1
        epi.step = float(n_step[0])
        epi.first_step = int(n_step[0] == 1)
        ctx.accumulate_tiled_epi(bases, weights, lay.tile, lay.tile_stride, 0, end,
                                 out.ptr if args.epilogue == "add_base" else None, op, fin, count, epi)

    for _ in range(args.warmup):
        step()
    barrier_sync(world, ctx)

    n_launch0 = ctx.launch_count()
    ctx.timing_begin()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier_sync(world, ctx)
    t1 = time.perf_counter()
    ev_ms = ctx.timing_end()
    launches_per_step = (ctx.launch_count() - n_launch0) / args.steps

    wall = max_over_ranks(world, t1 - t0)
    kernel_ms = ev_ms / args.steps
    kernel_ms_max = max_over_ranks(world, kernel_ms)

    extra = {}
    if args.epilogue != "none":
        args.spot_check = 0  # the spot check covers the plain aggregation output only
    if world == 1:
        extra = cpu_baseline_and_spot_check(args, ctx, K, out, weights, count, P, col0, op)
    else:  # every rank checks its own bucket; the counts are summed (no CPU baseline at N > 1)
        extra = cpu_baseline_and_spot_check(args, ctx, K, out, weights, count, P, col0, op, baseline=False)
        if "spot_check" in extra:
            sampled, mism = sum_over_ranks(world, [extra["spot_check"]["sampled"], extra["spot_check"]["mismatches"]])
            extra["spot_check"].update(sampled=sampled, mismatches=mism, ranks=world)

    if rank == 0:
        bytes_step = 4.0 * K * P * world  # aggregated client bytes per step, all ranks
        value = bytes_step * args.steps / wall / 2**30
        epi_bytes = {"none": 4.0, "add_base": 8.0, "sgd": 16.0}.get(args.epilogue, 24.0)
        alg_bytes_launch = 4.0 * K * P + epi_bytes * P
        traffic, traffic_src = pmc_traffic(args, K, P)
        achieved = alg_bytes_launch / (kernel_ms / 1e3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: device counter-hash generator (Irwin-Hall(4) ~N(0,1)), host twin in oracle/",
            "config": {
                "workload": f"{K} clients x {P} fp32 params per GPU, weighted FedAvg, {args.mode}-mode arithmetic"
                            + ("" if args.epilogue == "none" else f", fused {args.epilogue} server update"),
                "epilogue": args.epilogue,
                "clients": K,
                "params_per_gpu": P,
                "mode": args.mode,
                "parallelism": f"param-bucket shards x{world}, no data-path collective",
                "layout": f"tiled slab, {lay.tile}-element tiles x {K} slots",
                "kernel": (("fedavg_tiles_burst_f32x4 (results staged on chip, stored as chip-wide bursts; "
                            + ("8 register-held tiles per block per launch)" if args.variant & 32
                               else "8 register- + 10 LDS-held tiles per block per launch, one block per CU)"
                               if K >= 32 and not args.variant & 64
                               else "8 register- + 4 LDS-held tiles per block per launch)"))
                           if epi is None and args.variant & 11 == 0
                           else "fedavg_tiles_epi_burst_f32x4" if epi is not None and args.variant & 12 == 0
                           else "fedavg_tiles_epi_f32x4" if epi is not None else "fedavg_tiles_f32x4"),
            },
            "pct_hbm_peak": round(100.0 * achieved / HBM_PEAK_GBS, 2),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel_ms_avg": round(kernel_ms, 4),
                "kernel_ms_avg_max_rank": round(kernel_ms_max, 4),
                "alg_bytes_per_launch": alg_bytes_launch,
                # one aggregation = launches_per_step kernel launches (the burst kernel: one per 8 tiles per
                # block); kernel_ms_avg and alg_bytes_per_launch are per aggregation, launch_us_avg is the
                # per-launch figure a rocprofv3 --stats average compares with
                "launches_per_step": launches_per_step,
                "launch_us_avg": round(kernel_ms * 1e3 / max(launches_per_step, 1), 2),
            },
        }
        if "cpu_baseline" in extra:
            line["cpu_baseline"] = extra["cpu_baseline"]
        else:
            line["cpu_baseline"] = None
        if "spot_check" in extra:
            line["spot_check"] = extra["spot_check"]
        print(json.dumps(line), flush=True)
    failed = bool(extra.get("spot_check", {}).get("mismatches"))  # summed over ranks: every rank agrees
    if failed and rank == 0:
        print("SPOT CHECK FAILED", file=sys.stderr)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    if failed:
        sys.exit(3)


if __name__ == "__main__":
    main()
