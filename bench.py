#!/usr/bin/env python3
"""Benchmark of the MI355X FedAvg weighted aggregation (BASELINE.json metric).

One step = one aggregation: the arrival-ordered weighted accumulate-and-finalise kernel over K
device-resident client rows of P fp32 params -> P fp32 results (weighted_aggregation_helper.py:153-240,
torch-mode arithmetic by default).  Inputs are resident in HBM before the timed region starts.

  python bench.py [--gpus N --steps K --warmup W]          # default: BASELINE config 3, 64 clients x 1e9 params;
                                                           # N > 1: starts N rank processes itself (launch_ranks)
  torchrun --nproc-per-node N bench.py --gpus N ...        # the same N ranks under torchrun (WORLD_SIZE set)
  python bench.py --config {2,3,4,5}                       # BASELINE.json configs[1..4] (presets below)

Scaling.  The path shards by parameter bucket:
  weak   (configs 2, 3 -- single-GPU configs): every rank aggregates its own P-param bucket of the K clients
  strong (configs 4, 5 -- "sharded across 8", "1->8 GPUs"): a fixed global model of P params is split by
         sharding.bucket_ranges(P, N); rank r aggregates bucket r of every client.
After the main measurement the default run also measures, in the same process, BASELINE configs 5 and 4 under
strong scaling (``--also``; config 4 needs >= 2 GPUs: 358 GB of client updates do not fit one 288 GB HBM), and
config 4 once more as a multi-GPU server would ingest it ("4x": client g's whole update on GPU g mod N, RCCL
all-to-all of the buckets overlapped with the kernels, nvflare_amd/client_shards.py; serial and overlapped device
times side by side, under a watchdog so a stuck collective cannot cost the line), and config 2 once more as the
server receives it ("2h": pageable host arrays through the drop-in helper's add / get_result, H2D and D2H included --
north_star's PCIe-inclusive rate, each rank on its own GPU and PCIe link; "2s": the same round in ONE process whose
helper splits every key over all N GPUs, as a single NVFlare server process drives a node), and embeds them in the
line's ``also`` list -- so one N-GPU run records configs 2, 3, 4 and 5 at that N.

Prints ONE JSON line (rank 0).  value = GiB/s aggregated = 4*K*P_total*steps / t / 2^30 with t the max over
ranks of the barrier+synchronize bracketed wall time (P_total = P*N weak, P strong).  roofline.achieved uses the
algorithmic bytes of one aggregation on one GPU (4*K*P_gpu + 4*P_gpu, or + the epilogue's state bytes) over
its device time measured with HIP events on the stream the kernels run on (one aggregation =
roofline.launches_per_step launches of the burst kernel; launch_us_avg is the per-launch time a rocprofv3
--stats average compares with).  cpu_baseline times the oracle restatement (torch CPU ops) on a bounded
sample of the same workload, and the same leg spot-checks sampled device outputs bit-exactly against the
oracle (test infrastructure; never the measured path).
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

# BASELINE.json configs[1..4] (configs[0] is the CPU plumbing job, tests/sag_harness.py)
PRESETS = {
    2: dict(clients=8, params=125_000_000, epilogue="none", scaling="weak"),
    3: dict(clients=64, params=1_000_000_000, epilogue="none", scaling="weak"),
    4: dict(clients=256, params=350_000_000, epilogue="none", scaling="strong"),
    5: dict(clients=64, params=1_000_000_000, epilogue="adam", scaling="strong"),
}
PRESET_NAMES = {
    2: "BASELINE config 2: 8 clients x 125M fp32 params, weighted FedAvg on 1 MI355X",
    3: "BASELINE config 3: 64 clients x 1B fp32 params, single-GPU HBM-resident aggregation",
    4: "BASELINE config 4: 256 clients x 350M fp32 params, param buckets sharded across the GPUs",
    5: "BASELINE config 5: FedOpt server optimizer (Adam on aggregated deltas), 64 clients x 1B params",
}
SHARE_GPUS = 8  # config 4 on fewer GPUs than it fits: one GPU's share of this many (BASELINE: "across 8 MI355X")
CLIENT_SHARDED = 40  # --also token "4x": config 4 through the client-sharded exchange (run_client_sharded)
HOST_RESIDENT = 20  # --also token "2h": config 2 with host-resident updates and result (run_host_resident)
HOST_SHARDED = 21  # --also token "2s": the same round in ONE process over all N GPUs' buckets (run_host_resident)
WATCHDOG_S = 240.0  # each guarded entry's limit: a stuck collective must not cost the measured line
EPI_STATE_BYTES = {"none": 4.0, "add_base": 8.0, "sgd": 16.0}  # per param beyond the 4*K client reads; else 24
HEADROOM = 2 << 30  # device bytes left free beside a workload (runtime, gather buffers)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, choices=sorted(PRESETS), default=3,
                    help="BASELINE.json workload preset (clients, params, epilogue, scaling); flags below override")
    ap.add_argument("--clients", type=int, default=None)
    ap.add_argument("--params", type=float, default=None,
                    help="fp32 params: per GPU under weak scaling, of the whole model under strong scaling")
    ap.add_argument("--global-params", type=float, default=None, help="--scaling strong --params N")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None)
    ap.add_argument("--also", default="auto",
                    help="extra strong-scaling BASELINE configs measured after the main one, in the same line "
                         "(comma list of 4 / 5 / 4x = config 4 through the client-sharded RCCL exchange / "
                         "2h = config 2 from host-resident updates to a host result, PCIe included, every rank / "
                         "2s = the same round in one process over all N GPUs' parameter buckets; "
                         "2 = config 2 device-resident (weak); "
                         "'auto' = 2,5,4,2h,2s,4x for the default config 3 run; 'none')")
    ap.add_argument("--client-sharded-params", type=float, default=None,
                    help="model size of the 4x entry (default: config 4's 350M; smaller for one-GPU rehearsals)")
    ap.add_argument("--host-resident-params", type=float, default=None,
                    help="params per GPU of the 2h entry (default: config 2's 125M)")
    ap.add_argument("--watchdog-s", type=float, default=WATCHDOG_S, help="limit of the 4x and 2h entries")
    ap.add_argument("--rank-timeout-s", type=float, default=RANK_TIMEOUT_S,
                    help="--gpus N without torchrun: limit of the N rank processes this run starts")
    ap.add_argument("--mode", choices=["torch", "numpy"], default="torch")
    ap.add_argument("--blocks-per-cu", type=int, default=0,
                    help="0 = library default (burst kernel: 1 at >= 32 clients, else 2; fused: 1 at >= 64)")
    ap.add_argument("--unroll", type=int, default=0, help="0 = library default (4)")
    ap.add_argument("--variant", type=int, default=0,
                    help="kernel variant bits (include/nvflare_amd_fedavg.h fedavg_set_variant; 0 = burst kernel)")
    ap.add_argument("--tile", type=int, default=4096, help="slab tile width (elements)")
    ap.add_argument("--epilogue", choices=["none", "add_base", "sgd", "adam", "adamax", "nadam", "radam"], default=None,
                    help="fused server update (config 5 = adam: FedOpt Adam on the aggregated deltas)")
    ap.add_argument("--entry-warmup-s", type=float, default=0.5,
                    help="the also entries' untimed warmup lasts at least this long (the main entry runs exactly "
                         "--warmup steps): a short entry after an idle gap (a D2H, a fill) otherwise times the GPU "
                         "while its clocks ramp back up (round 6: config 4's share at 1 666 MHz gfx, 85.7 %% against "
                         "88.5 %% warm)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-s", type=float, default=8.0, help="seconds of CPU work the baseline times")
    ap.add_argument("--cpu-sample-params", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--spot-check", type=int, default=4096, help="sampled outputs checked against the oracle")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per aggregation from a separate rocprofv3 --pmc pass (default: "
                         "profiles/pmc_traffic.json when its config matches this run)")
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--sqrt", choices=["auto", "torch_cpu", "torch_cpu_amd", "ieee"], default="auto",
                    help="sqrt of the fused optimizer step: the product default (auto: the sqrt this host's torch "
                         "computes, nvflare_amd/torch_sqrt.py), torch CPU's restated vsSqrt of the Intel or the AMD hosts, or the "
                         "correctly rounded one")
    args = ap.parse_args(argv)
    preset = PRESETS[args.config]
    if args.global_params is not None:
        args.params, args.scaling = args.global_params, "strong"
    for k in ("clients", "params", "epilogue", "scaling"):
        if getattr(args, k) is None:
            setattr(args, k, preset[k])
    args.clients, args.params = int(args.clients), int(args.params)
    explicit = any(f in (argv if argv is not None else sys.argv[1:])
                   for f in ("--clients", "--params", "--global-params", "--scaling", "--epilogue"))
    args.preset_exact = not explicit
    if args.also == "auto":
        args.also = "2,5,4,2h,2s,4x" if (args.config == 3 and not explicit) else "none"
    tokens = {"4x": CLIENT_SHARDED, "2h": HOST_RESIDENT, "2s": HOST_SHARDED}
    args.also = [] if args.also in ("", "none") else [tokens.get(x.strip()) or int(x) for x in args.also.split(",")]
    return args


RANK_TIMEOUT_S = 1800.0  # the self-launched ranks' limit (python bench.py --gpus N without torchrun)
RANK_GRACE_S = 60.0  # after one rank fails: how long the others get to end on their own before they are killed


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """``python bench.py --gpus N`` with no WORLD_SIZE in the environment: start N rank
    processes of this same script, one per GPU, the way ``torchrun --nproc-per-node N`` would (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), and print rank 0's JSON line.  This process makes no GPU call
    (it has not imported torch): it only starts the ranks, so nothing re-executes a process that touched the GPU.
    The other ranks' stdout goes to stderr; every rank's stderr passes through (progress).  Returns the exit code: 0,
    the first failing rank's code (the others then get RANK_GRACE_S to end before they are killed), or 124 when the
    ranks have not finished within --rank-timeout-s (all killed).  The ranks never outlive this process: each is
    started with PR_SET_PDEATHSIG = SIGKILL, and SIGTERM / SIGINT here kill them before this process exits."""
    import signal
    import subprocess
    import threading

    world = args.gpus
    script = os.environ.get("NVFLARE_AMD_BENCH_WORKER_SCRIPT") or os.path.abspath(__file__)  # a test seam
    argv = list(sys.argv[1:] if argv is None else argv)
    base_env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
                    LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", NVFLARE_AMD_BENCH_LAUNCHED="1")
    base_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC on this pool
    procs, lines = [], []

    def pump(p, rank):
        for raw in p.stdout:
            line = raw.decode(errors="replace")
            if rank == 0 and line.startswith("{"):  # the result line; library chatter (gloo, RCCL) goes to stderr
                lines.append(line)
                sys.stdout.write(line)
                sys.stdout.flush()
            else:
                sys.stderr.write(f"[rank {rank}] {line}")

    def die_with_parent():  # Linux PR_SET_PDEATHSIG: a rank is killed when this process dies, however it dies
        try:
            import ctypes

            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)
        except OSError:
            pass

    # every rank first (no thread runs while preexec_fn does), then their output pumps
    for r in range(world):
        env = dict(base_env, RANK=str(r), LOCAL_RANK=str(r))
        p = subprocess.Popen([sys.executable, "-u", script, *argv], env=env, stdout=subprocess.PIPE,
                             start_new_session=True,  # its own process group: killed as a whole on failure
                             preexec_fn=die_with_parent)
        procs.append((p, threading.Thread(target=pump, args=(p, r), daemon=True)))
    for _, t in procs:
        t.start()

    def kill_all():
        for p, _ in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass

    def on_signal(signum, frame):  # the driver's own time limit (SIGTERM) or ^C: the ranks go with this process
        kill_all()
        sys.stderr.write(f"bench: signal {signum}; the ranks were killed\n")
        os._exit(128 + signum)

    old_handlers = {}
    if threading.current_thread() is threading.main_thread():
        for sig in (signal.SIGTERM, signal.SIGINT):
            old_handlers[sig] = signal.signal(sig, on_signal)

    deadline = time.monotonic() + args.rank_timeout_s
    code, failed_at = 0, None
    try:
        while True:
            states = [p.poll() for p, _ in procs]
            bad = [(r, c) for r, c in enumerate(states) if c not in (None, 0)]
            if bad and code == 0:
                r, code = bad[0]
                failed_at = time.monotonic()
                print(f"bench: rank {r} exited with {code}; the other ranks get {RANK_GRACE_S:g} s", file=sys.stderr)
            if all(c is not None for c in states):
                break
            now = time.monotonic()
            if now > deadline or (failed_at is not None and now - failed_at > RANK_GRACE_S):
                if failed_at is None:
                    code = 124
                    print(f"bench: the ranks did not finish within {args.rank_timeout_s:g} s; killed", file=sys.stderr)
                kill_all()
                break
            time.sleep(0.2)
    finally:
        kill_all()
        for p, t in procs:
            p.wait()
            t.join(timeout=5)
        for sig, h in old_handlers.items():
            signal.signal(sig, h)
    if code == 0 and len(lines) != 1:
        print("bench: rank 0 printed no result line", file=sys.stderr)
        code = 1
    return code


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
    """Element-wise SUM over ranks of a few host integers (spot-check counts, feasibility votes)."""
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


def rank_span(scaling: str, rank: int, world: int, P: int):
    """(first global param, params) of rank r's bucket: weak -- its own P; strong -- bucket r of a P-param
    model split by sharding.bucket_ranges (whole 4096-element tiles, sizes within one tile of each other)."""
    if scaling == "weak":
        return rank_bucket(rank, P), P
    from nvflare_amd.sharding import bucket_ranges

    lo, hi = bucket_ranges(P, world)[rank]
    return lo, hi - lo


def synth_weights(K):
    """aggregation_weight 1.0 x NUM_STEPS_CURRENT_ROUND = 1 + (37k mod 100)."""
    return [1.0 * float(1 + (37 * k) % 100) for k in range(K)]


def arrival_count(weights):
    count = None
    for w in weights:
        count = w if count is None else count + w
    return count


ADAM_HP = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8)


def sqrt_mode(args) -> str:
    """The fused optimizer step's sqrt (nvflare_amd/torch_sqrt.py): the product default unless --sqrt says."""
    from nvflare_amd import torch_sqrt

    return torch_sqrt.mode() if args.sqrt == "auto" else args.sqrt


def spot_check(args, ctx, K, P, col0, op, epilogue, bufs, n_steps, seed):
    """Sampled device outputs of this rank's bucket against the oracle computed from the host twin of the
    generator (test infrastructure): the plain aggregation's output, or for the fused Adam step the parameter and
    both moments after every step the run made."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import fedavg_oracle as orc

    if args.spot_check <= 0 or epilogue not in ("none", "adam"):
        return None
    rng = np.random.default_rng(7)
    idx = np.unique(np.concatenate([rng.integers(0, P, args.spot_check, dtype=np.int64), [0, P - 1]]))
    cols = (idx + col0).astype(np.uint64)
    weights = synth_weights(K)
    mode = orc.MODE_TORCH if op == 1 else orc.MODE_NUMPY
    d = orc.fedavg_c([orc.synth_values(seed, k, cols) for k in range(K)], weights, mode)
    if epilogue == "none":
        got = ctx.gather_f32(bufs[0].ptr, idx.astype(np.uint64))
        mism = int(np.count_nonzero(d.view(np.uint32) != got.view(np.uint32)))
        return {"sampled": int(idx.size), "mismatches": mism, "oracle": "oracle/fedavg_oracle.c"}
    p = orc.synth_values(seed + 7, 0, cols)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    sq = sqrt_mode(args)
    for s in range(1, n_steps + 1):
        orc.epilogue_apply(d, orc.EPI_ADAM, p=p, m=m, v=v, step=float(s), torch_cpu_sqrt=sq, **ADAM_HP)
    mism = 0
    for buf, host in zip(bufs, (p, m, v)):
        got = ctx.gather_f32(buf.ptr, idx.astype(np.uint64))
        mism += int(np.count_nonzero(host.view(np.uint32) != got.view(np.uint32)))
    return {"sampled": int(idx.size) * 3, "mismatches": mism,
            "oracle": f"oracle/fedavg_oracle.c (aggregation + {n_steps} Adam steps; p, exp_avg, exp_avg_sq; "
                      f"{ {'torch_cpu': 'torch CPU (Intel host)', 'torch_cpu_amd': 'torch CPU (AMD host)'}.get(sq, 'correctly rounded')} sqrt)"}


def cpu_baseline(args, K, P, op):
    """The reference's op sequence restated on the host (oracle, test infrastructure) on a bounded sample of the
    workload: torch CPU mul / add_(alpha) / div_ with torch's intra-op threads, and numpy single-threaded."""
    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import fedavg_oracle as orc

    weights = synth_weights(K)
    Ps = int(min(args.cpu_sample_params, P))
    gen = [np.random.default_rng(1000 + k).standard_normal(Ps, dtype=np.float32) for k in range(K)]
    trows = [torch.from_numpy(g) for g in gen]
    threads, cg_cpus, cg_file, affinity = baseline_threads()
    prev_threads = torch.get_num_threads()

    def timed(limit_s):
        reps, t_tot = 0, 0.0
        while t_tot < limit_s and reps < 2000:
            t0 = time.perf_counter()
            if op == 1:
                orc.torch_mode_reference(trows, weights)
            else:
                orc.numpy_mode_reference(gen, weights)
            t_tot += time.perf_counter() - t0
            reps += 1
        return reps, t_tot

    torch.set_num_threads(threads)
    try:
        reps, t_tot = timed(getattr(args, "cpu_baseline_s", 8.0))
    finally:
        torch.set_num_threads(prev_threads)
    gibs = 4.0 * K * Ps * reps / t_tot / 2**30
    t0 = time.perf_counter()  # single-thread numpy restatement (the numpy-job path) for context
    orc.numpy_mode_reference(gen, weights)
    t_np = time.perf_counter() - t0
    omp = os.environ.get("OMP_NUM_THREADS")
    if cg_cpus is not None:
        reason = (f"min(affinity {affinity}, ceil(cgroup quota {cg_cpus:g} CPUs from {cg_file})): the CPUs this "
                  f"process may use ({os.cpu_count()} on the host)")
    else:
        reason = (f"no cgroup CPU quota; min(affinity {affinity}, OMP_NUM_THREADS={omp} or torch's default "
                  f"{prev_threads}) ({os.cpu_count()} on the host)")
    return {
        "value": round(gibs, 3),
        "unit": "GiB/s",
        "cores": threads if op == 1 else 1,
        "kind": "port",
        "sample": f"{K} clients x {Ps} fp32 params (numpy default_rng(1000+k) N(0,1)), "
                  f"{'torch CPU mul/add_(alpha)/div_' if op == 1 else 'numpy v*w / t+v*w / t*(1/c)'} "
                  f"restatement of weighted_aggregation_helper.py:181-236, {reps} reps in {t_tot:.1f}s",
        "numpy_single_thread_GiBs": round(4.0 * K * Ps / t_np / 2**30, 3),
        "torch_threads": threads,
        "host_cpu_count": os.cpu_count(),
        "affinity_cpus": affinity,
        "cgroup_cpus": round(cg_cpus, 3) if cg_cpus is not None else None,
        "cgroup_quota_file": cg_file,
        "omp_num_threads_env": omp,
        "cores_reason": reason,
        "host_cpu_model": _cpu_model(),
    }


def cgroup_cpu_quota(root="/sys/fs/cgroup", proc_cgroup="/proc/self/cgroup"):
    """CPUs this process's cgroup may use (quota / period, the smallest along its cgroup path), or None when no quota
    is set.  cgroup v2: <root>/<path>/cpu.max ("max 100000" | "1600000 100000"); v1: cpu.cfs_quota_us and
    cpu.cfs_period_us under the cpu (or cpu,cpuacct) hierarchy.  Returns (cpus as a float, the file it came from)."""
    v2, v1 = None, None
    try:
        with open(proc_cgroup) as f:
            for line in f:
                parts = line.rstrip("\n").split(":", 2)
                if len(parts) != 3:
                    continue
                if parts[0] == "0" and parts[1] == "":
                    v2 = parts[2]
                elif "cpu" in parts[1].split(","):
                    v1 = (parts[1], parts[2])
    except OSError:
        pass

    def walk(base, rel):
        rel = rel.strip("/")
        parts = rel.split("/") if rel else []
        for i in range(len(parts), -1, -1):
            yield os.path.join(base, *parts[:i])

    best = None
    if v2 is not None:
        for d in walk(root, v2):
            try:
                with open(os.path.join(d, "cpu.max")) as f:
                    q, p = f.read().split()[:2]
            except (OSError, ValueError):
                continue
            if q != "max" and float(p) > 0:
                c = float(q) / float(p)
                if best is None or c < best[0]:
                    best = (c, os.path.join(d, "cpu.max"))
    if v1 is not None:
        for ctrl in (v1[0], "cpu,cpuacct", "cpu"):
            for d in walk(os.path.join(root, ctrl), v1[1]):
                try:
                    with open(os.path.join(d, "cpu.cfs_quota_us")) as f:
                        q = int(f.read())
                    with open(os.path.join(d, "cpu.cfs_period_us")) as f:
                        p = int(f.read())
                except (OSError, ValueError):
                    continue
                if q > 0 and p > 0:
                    c = q / p
                    if best is None or c < best[0]:
                        best = (c, os.path.join(d, "cpu.cfs_quota_us"))
            if best is not None:
                break
    return best


def baseline_threads():
    """Threads for the CPU baseline: min(affinity CPUs, ceil(cgroup quota)) when the cgroup sets a
    quota -- a process that sees 256 CPUs but may use 16 thrashes at 256 threads -- else min(affinity,
    OMP_NUM_THREADS or torch's default).  Returns (threads, cgroup cpus or None, quota file or None, affinity)."""
    import math

    import torch

    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    if quota is not None:
        return max(1, min(affinity, math.ceil(quota[0] - 1e-9))), quota[0], quota[1], affinity
    omp = os.environ.get("OMP_NUM_THREADS")
    want = int(omp) if omp and omp.isdigit() and int(omp) > 0 else torch.get_num_threads()
    return max(1, min(affinity, want)), None, None, affinity


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(args, K, P, epilogue):
    """HBM bytes per aggregation measured by rocprofv3 PMC passes of this same command
    (profiles/pmc_traffic.json), only when that measurement's configuration is this run's."""
    if args.traffic_bytes is not None:
        return args.traffic_bytes, "--traffic-bytes"
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, None
    want = {"clients": K, "params": P, "tile": args.tile, "mode": args.mode, "epilogue": epilogue, "dtype": "fp32"}
    for r in rec.get("records", []):
        cfg = dict(r.get("config", {}))
        cfg.setdefault("epilogue", "none")
        cfg.setdefault("dtype", "fp32")  # 16-bit records (tools/bench_narrow.py lines) never stand for a bench line
        if all(cfg.get(k) == v for k, v in want.items()):
            return float(r["bytes_per_launch"]), "profiles/pmc_traffic.json"
    return None, None


def gpu_monitor(local):
    """tools/gpu_state.GpuMonitor for this rank's GPU, or None when switched off
    (NVFLARE_AMD_BENCH_GPU_STATE=0) or unavailable; never fails the run."""
    if os.environ.get("NVFLARE_AMD_BENCH_GPU_STATE", "1") == "0":
        return None
    try:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from tools.gpu_state import GpuMonitor

        return GpuMonitor(local)
    except Exception:  # noqa: BLE001 -- measurement context only
        return None


def gpu_sampler(args):
    """A context manager sampling this rank's GPU state over a timed region (``None`` inside when off)."""
    import contextlib

    mon = getattr(args, "gpu_monitor", None)
    return mon.sample() if mon is not None else contextlib.nullcontext(None)


def gpu_snapshot(args):
    mon = getattr(args, "gpu_monitor", None)
    return mon.snapshot() if mon is not None else None


def handout_pull(args, ctx, world, param_buf, P, reps=3):
    """The FedOpt hand-out pull timed: after the server step the new weights leave for the clients
    as an independent host copy -- ShardedServerOptimizer.to_host -> _pull (nvflare_amd/app_opt/pt/sharded_fedopt.py),
    one fedavg_d2h_multi per GPU of its parameter bucket into one page-locked host array, every GPU over its own PCIe
    link at once (here: every rank its bucket, in parallel); at N = 1 DeviceServerOptimizer's single-device pull.  The
    host array is page-locked once before the timed pulls (the pool reuses it across rounds).  Returns the max over
    ranks of the median pull time."""
    from nvflare_amd.device import HostArenaPool

    pool = HostArenaPool(depth=1)
    host = pool.take(P, pin=ctx)
    pieces = [(0, 0, 4 * P)]
    ctx.d2h_multi(host, param_buf.ptr, pieces)  # first touch of the pages outside the timing
    times = []
    for _ in range(reps):
        barrier_sync(world, ctx)
        t0 = time.perf_counter()
        ctx.d2h_multi(host, param_buf.ptr, pieces)
        times.append(time.perf_counter() - t0)
    dist_barrier(world)
    t = max_over_ranks(world, sorted(times)[len(times) // 2])
    del host
    return {"ms": round(t * 1e3, 3), "bytes_per_gpu_rank0": 4 * P, "GBps_per_gpu_rank0": round(4 * P / t / 1e9, 2),
            "reps": reps, "what": "new parameters D2H into one page-locked host array, every GPU its bucket at once "
                                  "(ShardedServerOptimizer._pull / to_host; fedavg_d2h_multi); max over ranks of the "
                                  "median of the reps"}


def wait_for_rank0(world, rank, key, timeout_s=1800.0):
    """Ranks != 0 block (sleeping on the rendezvous store's socket, not spinning on a GPU collective that would take
    host cores from rank 0's CPU baseline) until rank 0 has set ``key``."""
    if world == 1:
        return
    import datetime

    import torch.distributed as dist

    try:
        store = dist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001 -- no store API: a plain barrier
        dist.barrier()
        return
    if rank == 0:
        store.set(key, "1")
    else:
        store.wait([key], datetime.timedelta(seconds=timeout_s))


def kernel_name(K, epilogue, variant):
    # fewer client reads per launch than fedavg_capi.cpp's kBurstMinClients / kEpiBurstMinClients take the
    # per-tile-store kernels
    if epilogue != "none":
        if variant & 12 == 0 and K <= 3 and epilogue in ("adam", "sgd", "add_base"):
            return ("fedavg_tiles_epi_dma_f32x4 (1-3 client reads: inputs HBM -> LDS by LDS-DMA, results held on chip "
                    "and stored as chip-wide bursts)")
        if variant & 12 == 0 and K >= 64 and epilogue == "adam" and not variant & ((1 << 15) | 64):
            return ("fedavg_tiles_epi_split_f32x4 (the burst form's client phase on 4 waves, the epilogue on 8: "
                    "4 register- + 9 LDS-held tiles per block per launch)")
        return "fedavg_tiles_epi_burst_f32x4" if variant & 12 == 0 and K >= 4 else "fedavg_tiles_epi_f32x4"
    if K <= 3 and not variant & (11 | 256):
        return ("fedavg_tiles_few_f32x4 (1-3 client reads: every register-held tile's loads issued before any "
                "arithmetic, results stored as chip-wide bursts)")
    if (variant & 11 or K < 3) and not (K < 3 and variant & 256 and not variant & 11):
        return "fedavg_tiles_f32x4"
    return ("fedavg_tiles_burst_f32x4 (results staged on chip, stored as chip-wide bursts; "
            + ("8 register-held tiles per block per launch)" if variant & 32
               else "8 register- + 10 LDS-held tiles per block per launch, one block per CU)"
               if K >= 32 and not variant & 64 else "8 register- + 4 LDS-held tiles per block per launch)"))


def run_workload(args, ctx, world, rank, K, P_spec, scaling, epilogue, baseline, seed, min_warmup_s=0.0):
    """Stage one workload in HBM, time args.steps aggregations after args.warmup, spot-check, free it.

    Returns a dict (every rank) or, when the workload does not fit every rank's device, {"skipped": reason}."""
    from nvflare_amd import _native as N
    from nvflare_amd.device import TiledLayout

    col0, P = rank_span(scaling, rank, world, P_spec)
    op = N.FEDAVG_OP_TORCH if args.mode == "torch" else N.FEDAVG_OP_NUMPY
    fin = N.FEDAVG_FIN_DIV if args.mode == "torch" else N.FEDAVG_FIN_SCALE
    lay = TiledLayout(args.tile, K)  # the engine's slab layout: K client slots interleaved per tile
    end = (P + 3) // 4 * 4
    epi_bufs = {"none": 1, "add_base": 1, "sgd": 2}.get(epilogue, 3)  # out | p+buf | p+m+v
    need = lay.slab_elems(P) * 4 + epi_bufs * end * 4
    free, total = ctx.mem_info()
    if os.environ.get("NVFLARE_AMD_BENCH_SHARED_DEVICE") == "1":
        free //= world  # the one-GPU rehearsal: every rank on cuda:0
    fits = need + HEADROOM <= free
    if sum_over_ranks(world, [0 if fits else 1])[0]:
        return {"skipped": f"needs {need / 1e9:.1f} GB of HBM per GPU at {world} GPU(s) "
                           f"(this device: {free / 1e9:.1f} GB free of {total / 1e9:.1f})"}
    slab = ctx.alloc(lay.slab_elems(P) * 4)
    state = [ctx.alloc(end * 4) for _ in range(epi_bufs)]
    try:
        out = state[0]
        bases = [slab.ptr + lay.slot_offset_elems(k) * 4 for k in range(K)]
        for k, base in enumerate(bases):
            ctx.fill_synthetic_f32(base, P, seed, k, col0, lay.tile, lay.tile_stride)
        weights = synth_weights(K)
        count = arrival_count(weights)
        epi = None
        if epilogue != "none":
            for j, b in enumerate(state):  # initial params (or base weights), zero optimizer state
                if j == 0:
                    ctx.fill_synthetic_f32(b.ptr, end, seed + 7, 0, col0)
                else:
                    ctx.memset(b.ptr, 0, end * 4)
            epi = N.Epilogue()
            epi.kind = {"add_base": N.FEDAVG_EPI_ADD_BASE, "sgd": N.FEDAVG_EPI_SGD, "adam": N.FEDAVG_EPI_ADAM,
                        "adamax": N.FEDAVG_EPI_ADAMAX, "nadam": N.FEDAVG_EPI_NADAM,
                        "radam": N.FEDAVG_EPI_RADAM}[epilogue]
            if epilogue == "add_base":
                epi.base = out.ptr
            elif epilogue == "sgd":
                epi.param, epi.state1 = state[0].ptr, state[1].ptr
                epi.lr, epi.momentum = 1.0, 0.9
            else:
                from nvflare_amd import torch_sqrt

                epi.param, epi.state1, epi.state2 = state[0].ptr, state[1].ptr, state[2].ptr
                for k, v in ADAM_HP.items():
                    setattr(epi, k, v)
                epi.momentum_decay, epi.mu_product = 4e-3, 1.0  # NAdam (mu_product held at its first-step value)
                epi.torch_sqrt = torch_sqrt.epilogue_flag(sqrt_mode(args))
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
                                     out.ptr if epilogue == "add_base" else None, op, fin, count, epi)

        for _ in range(args.warmup):
            step()
        if min_warmup_s > 0:  # also entries: at least min_warmup_s of untimed steps (every rank decides the same)
            t_w = time.perf_counter()
            ctx.sync()
            go = 1
            while go:
                for _ in range(4):
                    step()
                ctx.sync()
                go = max_over_ranks(world, 1.0 if time.perf_counter() - t_w < min_warmup_s else 0.0) > 0
        barrier_sync(world, ctx)
        n_launch0 = ctx.launch_count()
        with gpu_sampler(args) as sampler:  # this rank's GPU clocks, power, temperatures over the timed steps
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
        sc = spot_check(args, ctx, K, P, col0, op, epilogue, state if epi is not None else [out], n_step[0], seed)
        if sc is not None and world > 1:  # every rank checks its own bucket; the counts are summed
            sampled, mism = sum_over_ranks(world, [sc["sampled"], sc["mismatches"]])
            sc.update(sampled=sampled, mismatches=mism, ranks=world)
        res = {"K": K, "P": P, "P_total": P_spec * world if scaling == "weak" else P_spec, "col0": col0,
               "wall": wall, "kernel_ms": kernel_ms, "kernel_ms_max": kernel_ms_max,
               "launches_per_step": launches_per_step, "spot_check": sc, "op": op,
               "gpu_state": sampler.summary() if sampler is not None else None}
        if epi is not None and epilogue != "add_base":
            res["handout_pull"] = handout_pull(args, ctx, world, state[0], P)
    finally:
        slab.close()
        for b in state:
            b.close()
    if baseline:
        res["cpu_baseline"] = cpu_baseline(args, K, P, op)
    return res


def fits_one_share(ctx, world, p):
    """Whether preset p under strong scaling fits every rank's device at this world size (agreed over ranks)."""
    from nvflare_amd.device import TiledLayout
    from nvflare_amd.sharding import bucket_ranges

    lay = TiledLayout(4096, p["clients"])
    lo, hi = bucket_ranges(p["params"], world)[0]
    need = lay.slab_elems(hi - lo) * 4 + (hi - lo + 3) // 4 * 16
    free, _ = ctx.mem_info()
    if os.environ.get("NVFLARE_AMD_BENCH_SHARED_DEVICE") == "1":
        free //= world
    return not sum_over_ranks(world, [0 if need + HEADROOM <= free else 1])[0]


def run_client_sharded(args, world, rank, local, K, P, seed):
    """BASELINE config 4 ingested as a multi-GPU server receives it: client g's WHOLE update (P params) lands on
    rank g mod N; RCCL all-to-alls move bucket b of every client to rank b, and each rank runs the arrival-ordered
    kernel over its bucket (nvflare_amd/client_shards.py, the bit-exact "exchange" strategy).  Timed twice over
    the same inputs: serial (all-to-all, then the kernels) and overlapped (the product path: chunked all-to-alls
    on one stream, the kernels over the tiles received so far on another).  Strong scaling: value counts the
    4*K*P client bytes once.  Returns {"skipped": ...} at N = 1 (nothing to exchange) or when it does not fit."""
    if world < 2:
        return {"skipped": "client-sharded ingest needs >= 2 GPUs (one rank has nothing to exchange)"}
    import torch

    from nvflare_amd.client_shards import ClientShardedFedAvg, ExchangePlan

    clients = [len(range(s, K, world)) for s in range(world)]
    plan = ExchangePlan(P, clients)
    need = 4 * (plan.slab_elems(rank) + plan.recv_elems(rank) + plan.bucket_pad())
    free, total = torch.cuda.mem_get_info(local)
    if os.environ.get("NVFLARE_AMD_BENCH_SHARED_DEVICE") == "1":
        free //= world  # the one-GPU rehearsal: every rank on cuda:0
    if sum_over_ranks(world, [0 if need + HEADROOM <= free else 1])[0]:
        return {"skipped": f"needs {need / 1e9:.1f} GB of HBM per GPU at {world} GPU(s) "
                           f"(this device: {free / 1e9:.1f} GB free of {total / 1e9:.1f})"}
    steps, warmup = max(1, min(args.steps, 5)), max(1, min(args.warmup, 1))
    agg = ClientShardedFedAvg(P, clients, device=local, mode=args.mode)
    try:
        agg.fill_synthetic(seed, [j * world + rank for j in range(clients[rank])])
        order = [(g % world, g // world) for g in range(K)]  # arrival order = global client id
        weights = synth_weights(K)
        nb = plan.bucket_len(rank)
        stream = torch.cuda.current_stream()

        def bracket(fn):
            torch.cuda.synchronize()
            dist_barrier(world)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            for _ in range(steps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            dist_barrier(world)
            return max_over_ranks(world, time.perf_counter() - t0), max_over_ranks(world, e0.elapsed_time(e1) / steps)

        for _ in range(warmup):
            agg.aggregate(order, weights, "exchange")
        # serial: the all-to-all alone, then the kernels alone (device times per phase)
        a2a_wall, a2a_ms = bracket(agg.exchange)
        kern_wall, kern_ms = bracket(lambda: agg.aggregate_exchanged(order, weights))
        serial = agg.out[:nb].clone()
        wall, ovl_ms = bracket(lambda: agg.aggregate(order, weights, "exchange"))
        differ = int(not torch.equal(agg.out[:nb].view(torch.int32), serial.view(torch.int32)))
        sc = None
        if args.spot_check > 0 and nb:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from oracle import fedavg_oracle as orc

            rng = np.random.default_rng(rank + 17)
            idx = np.unique(np.concatenate([rng.integers(0, nb, min(args.spot_check, nb)), [0, nb - 1]]))
            cols = (plan.buckets[rank][0] + idx).astype(np.uint64)
            want = orc.fedavg_c([orc.synth_values(seed, g, cols) for g in range(K)], weights,
                                orc.MODE_TORCH if args.mode == "torch" else orc.MODE_NUMPY)
            got = agg.out[torch.from_numpy(idx).to(agg.out.device)].cpu().numpy()
            sc = [int(idx.size), int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))]
        sampled, mism, differ = sum_over_ranks(world, (sc or [0, 0]) + [differ])
        a2a_out = 4.0 * (sum(plan.send_splits(rank)) - plan.send_splits(rank)[rank])
        return {"K": K, "P": nb, "P_total": P, "wall": wall * steps, "steps": steps, "warmup": warmup,
                "kernel_ms": kern_ms, "all_to_all_ms": a2a_ms, "overlapped_ms": ovl_ms,
                "all_to_all_bytes_out_rank0": a2a_out if rank == 0 else None,
                "bits_equal_serial": differ == 0,
                "spot_check": {"sampled": sampled, "mismatches": mism + differ, "ranks": world,
                               "oracle": "oracle/fedavg_oracle.c"} if sc is not None else None,
                "clients_per_rank": clients, "max_peer_bytes": agg.max_peer_bytes,
                "min_kernel_tiles": agg.min_kernel_tiles}
    finally:
        del agg
        torch.cuda.empty_cache()


def run_host_resident(args, world, rank, local, K, P, seed, sharded=False):
    """BASELINE config 2 as the server receives it (north_star's PCIe-inclusive rate): the K client updates are
    pageable numpy arrays in HOST memory (what the comm layer's decoder hands over), each goes through the drop-in
    WeightedAggregationHelper.add (weighted_aggregation_helper.py:153-224; the engine packs it through its pinned
    ring and H2D-copies it into the tiled slab) and get_result (:226-240; kernel + D2H into a new host array).
    One step = one round: K adds + get_result.  The whole result of the last step is compared with the oracle.

    2h (sharded=False), weak scaling: every rank runs its own config-2 round on its own GPU and PCIe link, so
    value = 4*K*P*N per step.  2s (sharded=True), strong scaling: rank 0 alone runs the round as ONE NVFlare server
    process would on an N-GPU node -- WeightedAggregationHelper(devices=[0..N-1]), every key split into N parameter
    buckets (sharding.ShardedFedAvg), bucket b of each client H2D-copied to GPU b over its own link by its own thread,
    the result buckets D2H-copied straight into one host array -- while the other ranks wait; value = 4*K*P per step."""
    import torch

    if sharded and world < 2:
        return {"skipped": "one process over N GPUs' buckets needs >= 2 GPUs (at N = 1 it is the 2h entry)"}
    active = rank == 0 or not sharded

    # three untimed rounds: the engine's page-locked result arrays are reused from round r - 2 on (the previous
    # round's result is still referenced by the caller, device.HostArenaPool), the steady state of a multi-round job
    steps, warmup = max(1, min(args.steps, 5)), 3
    weights = synth_weights(K)
    clients, helper = [], None
    if active:
        rng = np.random.default_rng(seed + 101 * rank)
        base = rng.standard_normal(P, dtype=np.float32)
        clients = [base * np.float32(1.0 + 0.01 * k) for k in range(K)]  # K distinct pageable host updates
        if sharded:
            shared = os.environ.get("NVFLARE_AMD_BENCH_SHARED_DEVICE") == "1"  # the one-GPU rehearsal
            helper = make_host_helper(local, devices=[0] * world if shared else list(range(world)))
        else:
            helper = make_host_helper(local)
    t_accept, t_drain, out, elapsed = 0.0, 0.0, None, 0.0
    try:
        def drain():
            """Wait until the staged client bytes are on the device(s): ``add`` returns once a client's bytes are in
            the pinned ring (the caller may reuse its array), with up to 4 x 64 MiB still crossing PCIe, and those
            DMAs would otherwise be counted in get_result."""
            eng = helper.engine
            for e in getattr(eng, "engines", [eng]):
                e.ctx.sync()

        def one_round(r):
            a0 = time.perf_counter()
            for k in range(K):
                helper.add({"w": clients[k]}, weights[k], f"site-{k}", r)
            a1 = time.perf_counter()
            drain()
            a2 = time.perf_counter()
            res = helper.get_result()["w"]
            return res, a1 - a0, a2 - a1

        # the warmup rounds hold the previous round's result, as the timed rounds do (a server keeps the last global
        # model): the result-array pool then alternates two page-locked arrays from the first timed round on.  Round
        # 3's warmup dropped its results, so the first timed round that held one paid the page-locking of a second
        # 500 MB array inside get_result (hipHostRegister, ~20 ms: profiles/r04/s3/trace2h_summary.json)
        for r in range(warmup if active else 0):
            out = one_round(r)[0]
        device_sync()
        dist_barrier(world)
        rounds_ms = []
        t0 = time.perf_counter()
        for r in range(steps if active else 0):
            r0 = time.perf_counter()
            out, dt, dd = one_round(warmup + r)
            rounds_ms.append(((time.perf_counter() - r0) - dt - dd) * 1e3)
            t_accept += dt
            t_drain += dd
        device_sync()
        elapsed = time.perf_counter() - t0
        dist_barrier(world)
        wall = max_over_ranks(world, elapsed)
        sc = None
        if args.spot_check > 0 and active:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from oracle import fedavg_oracle as orc

            threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1))
            want = orc.fedavg_c(clients, weights, orc.MODE_NUMPY, nthreads=threads)
            sc = [int(want.size), int(np.count_nonzero(np.asarray(out).view(np.uint32) != want.view(np.uint32)))]
        sampled, mism = sum_over_ranks(world, sc or [0, 0])
        return {"K": K, "P": P, "wall": wall, "steps": steps, "warmup": warmup, "sharded": sharded,
                "accept_s": max_over_ranks(world, t_accept / steps),
                "drain_s": max_over_ranks(world, t_drain / steps),
                "get_result_ms_rounds": [round(x, 2) for x in rounds_ms],
                "result_type": type(out).__name__ if active else None,
                "devices": len(helper.engine.engines) if sharded and active else 1,
                "spot_check": {"compared": sampled, "mismatches": mism, "ranks": 1 if sharded else world,
                               "oracle": "oracle/fedavg_oracle.c (every element of the last round's result)"}
                if args.spot_check > 0 else None}
    finally:
        if helper is not None:
            helper.reset_stats()
        del helper, clients
        if torch.cuda.is_available():
            torch.cuda.empty_cache()


def make_host_helper(local, devices=None):
    """The drop-in helper the 2h / 2s entries drive (a seam for the CPU tests' fake device)."""
    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    return WeightedAggregationHelper(devices=devices) if devices else WeightedAggregationHelper(device=local)


def device_sync():
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()


def summarize_host_resident(args, world, r):
    step_s = r["wall"] / r["steps"]
    exact = r["K"] == PRESETS[2]["clients"] and r["P"] == PRESETS[2]["params"]
    sharded = r["sharded"]
    per_step_bytes = 4.0 * r["K"] * r["P"] * (1 if sharded else world)
    return {
        "baseline_config": (PRESET_NAMES[2] if exact else f"custom (config 2 with {r['K']} x {r['P']})")
                           + (" -- host-resident, ONE server process over all GPUs' parameter buckets (PCIe-inclusive, "
                              "the drop-in helper with devices=[0..N-1])" if sharded else
                              " -- host-resident updates in, host result out (PCIe-inclusive, the drop-in helper)"),
        "value": round(per_step_bytes / step_s / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
        "scaling": "strong" if sharded else "weak", "steps": r["steps"], "warmup": r["warmup"],
        "ms_per_step": round(step_s * 1e3, 2),
        "accept_ms_per_step": round(r["accept_s"] * 1e3, 2),
        # the staging DMAs still in flight when the last add returned (the pinned ring's last slots)
        "staging_drain_ms": round(r["drain_s"] * 1e3, 2),
        ("h2d_GBps_all_gpus" if sharded else "h2d_GBps_per_gpu"):
            round(4.0 * r["K"] * r["P"] / (r["accept_s"] + r["drain_s"]) / 1e9, 2),
        "get_result_ms": round((step_s - r["accept_s"] - r["drain_s"]) * 1e3, 2),
        "get_result_ms_rounds": r.get("get_result_ms_rounds"),  # rank 0's rounds (kernel + D2H + host work)
        "spot_check": r["spot_check"],
        "config": {"clients": r["K"], ("params_total" if sharded else "params_per_gpu"): r["P"],
                   "container": "numpy (pageable)", "keys": 1, "mode": "numpy", "result": r["result_type"],
                   **({"devices": r["devices"], "process": "rank 0 alone; the other ranks wait"} if sharded else {})},
    }


def dist_barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def summarize_client_sharded(args, world, r):
    value = 4.0 * r["K"] * r["P_total"] * r["steps"] / r["wall"] / 2**30
    kern_bytes = 4.0 * r["K"] * r["P"] + 4.0 * r["P"]
    a2a_b = r["all_to_all_bytes_out_rank0"]
    return {
        "baseline_config": (PRESET_NAMES[4] if r["P_total"] == PRESETS[4]["params"]
                            else f"custom (config 4 with {r['P_total']} params)")
                           + " -- client-sharded ingest: client g's whole update on GPU g mod N, RCCL all-to-all of "
                             "buckets, overlapped with the kernels",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "scaling": "strong",
        "steps": r["steps"], "warmup": r["warmup"],
        "ms_per_step": round(r["wall"] / r["steps"] * 1e3, 3),
        "device_ms": {"overlapped": round(r["overlapped_ms"], 3), "serial_all_to_all": round(r["all_to_all_ms"], 3),
                      "serial_kernels": round(r["kernel_ms"], 3),
                      "hidden": round(r["all_to_all_ms"] + r["kernel_ms"] - r["overlapped_ms"], 3)},
        "all_to_all_GBps_out_rank0": round(a2a_b / (r["all_to_all_ms"] / 1e3) / 1e9, 1) if r["all_to_all_ms"] else None,
        "kernel_roofline_frac_rank0": round(kern_bytes / (r["kernel_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        "bits_equal_serial": r["bits_equal_serial"],
        "spot_check": r["spot_check"],
        "config": {"clients": r["K"], "params_total": r["P_total"], "params_bucket_rank0": r["P"],
                   "clients_per_rank": r["clients_per_rank"], "mode": args.mode,
                   "max_peer_bytes": r["max_peer_bytes"], "min_kernel_tiles": r["min_kernel_tiles"]},
    }


def summarize(args, world, res, K, scaling, epilogue, label):
    """The JSON fields of one measured workload (rank 0)."""
    P = res["P"]
    bytes_step = 4.0 * K * res["P_total"]  # aggregated client bytes per step, all ranks
    value = bytes_step * args.steps / res["wall"] / 2**30
    alg_bytes = 4.0 * K * P + EPI_STATE_BYTES.get(epilogue, 24.0) * P
    kernel_ms = res["kernel_ms"]
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
    traffic, traffic_src = pmc_traffic(args, K, P, epilogue)
    per_gpu = "per GPU" if scaling == "weak" else f"in all (model split over {world} GPU(s): {P} on GPU 0)"
    return {
        "value": round(value, 2),
        "ms_per_step": round(res["wall"] / args.steps * 1e3, 4),
        "scaling": scaling,
        "config": {
            "workload": f"{K} clients x {res['P_total'] if scaling == 'strong' else P} fp32 params {per_gpu}, weighted "
                        f"FedAvg, {args.mode}-mode arithmetic"
                        + ("" if epilogue == "none" else f", fused {epilogue} server update"),
            "baseline_config": label,
            "epilogue": epilogue,
            "clients": K,
            "params_per_gpu": P,
            "params_total": res["P_total"],
            "mode": args.mode,
            "parallelism": (f"param-bucket shards x{world}, no data-path collective"
                            + (" (each GPU its own bucket)" if scaling == "weak" else " (one model split in buckets)")),
            "layout": f"tiled slab, {args.tile}-element tiles x {K} slots",
            "kernel": kernel_name(K, epilogue, args.variant),
            **({"sqrt": sqrt_mode(args)} if epilogue in ("adam", "nadam", "radam") else {}),
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
            "kernel_ms_avg_max_rank": round(res["kernel_ms_max"], 4),
            "alg_bytes_per_launch": alg_bytes,
            # one aggregation = launches_per_step kernel launches (the burst kernel: one per grid x tiles-per-block);
            # kernel_ms_avg, alg_bytes_per_launch and traffic are per aggregation (rank 0's GPU), launch_us_avg is the
            # per-launch figure a rocprofv3 --stats average compares with
            "launches_per_step": res["launches_per_step"],
            "launch_us_avg": round(kernel_ms * 1e3 / max(res["launches_per_step"], 1), 2),
        },
    }


def entry_name(token) -> str:
    return {CLIENT_SHARDED: PRESET_NAMES[4] + " -- client-sharded ingest",
            HOST_RESIDENT: PRESET_NAMES[2] + " -- host-resident",
            HOST_SHARDED: PRESET_NAMES[2] + " -- host-resident, one process over all GPUs"}[token]


def guarded_entry(args, world, rank, local, line, also, state, token):
    """Run one collective-bearing ``also`` entry (4x: client-sharded config 4; 2h: host-resident config 2) and
    append it (rank 0).  A watchdog bounds it and whatever follows until the caller cancels it (the next entry, the
    process-group teardown): if that has not finished after --watchdog-s, rank 0 prints the line measured so far
    (the entry marked timed out) unless it already has, and every rank exits -- the main measurement is never lost
    to a stuck collective or a rank that failed alone.  Returns (spot check failed, the watchdog)."""
    import threading

    def on_timeout():
        if rank == 0 and not state.get("printed"):
            also.append({"baseline_config": entry_name(token), "n_gpus": world,
                         "error": f"did not finish within {args.watchdog_s:g} s (watchdog); measurement abandoned"})
            line["also"] = also
            print(json.dumps(line), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)

    dog = threading.Timer(args.watchdog_s, on_timeout)
    dog.daemon = True
    dog.start()
    t_entry = time.perf_counter()
    try:
        if token in (HOST_RESIDENT, HOST_SHARDED):
            p = PRESETS[2]
            P = int(args.host_resident_params) if args.host_resident_params else p["params"]
            r = run_host_resident(args, world, rank, local, p["clients"], P, args.seed, sharded=token == HOST_SHARDED)
        else:
            p = PRESETS[4]
            P = int(args.client_sharded_params) if args.client_sharded_params else p["params"]
            r = run_client_sharded(args, world, rank, local, p["clients"], P, args.seed)
    except Exception as e:  # noqa: BLE001 -- recorded in the line, the main measurement stands
        if rank == 0:
            also.append({"baseline_config": entry_name(token), "n_gpus": world, "error": f"{type(e).__name__}: {e}"})
        return False, dog
    if rank == 0:
        if "skipped" in r:
            also.append({"baseline_config": entry_name(token), "n_gpus": world, "skipped": r["skipped"]})
        elif token in (HOST_RESIDENT, HOST_SHARDED):
            also.append(summarize_host_resident(args, world, r))
        else:
            also.append(summarize_client_sharded(args, world, r))
        also[-1]["elapsed_s"] = round(time.perf_counter() - t_entry, 2)  # the entry's whole wall time
    return bool("skipped" not in r and (r.get("spot_check") or {}).get("mismatches")), dog


def client_sharded_entry(args, world, rank, local, line, also, state):
    return guarded_entry(args, world, rank, local, line, also, state, CLIENT_SHARDED)


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started here (no torchrun around us); nothing in this process touches the GPU
        code = launch_ranks(args, argv)
        if code:
            sys.exit(code)
        return
    world, rank, local = dist_setup(args)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from nvflare_amd.device import DeviceContext

    ctx = DeviceContext.get(local)
    ctx.set_launch(args.blocks_per_cu, args.unroll)
    ctx.set_variant(args.variant)
    args.gpu_monitor = gpu_monitor(local)
    state_before = gpu_snapshot(args) if rank == 0 else None
    K = args.clients
    label = (PRESET_NAMES[args.config] if args.preset_exact
             else f"custom (preset {args.config} overridden: {K} clients x {args.params} params, {args.epilogue})")
    t_main = time.perf_counter()
    main_res = run_workload(args, ctx, world, rank, K, args.params, args.scaling, args.epilogue, baseline=False,
                            seed=args.seed)
    main_s = time.perf_counter() - t_main
    if "skipped" in main_res:
        raise SystemExit(f"rank {rank}: workload {main_res['skipped']}")
    also = []
    failed = bool((main_res.get("spot_check") or {}).get("mismatches"))  # counts summed over ranks: all agree
    for cfg in args.also:
        if cfg in (CLIENT_SHARDED, HOST_RESIDENT, HOST_SHARDED):
            continue  # last, each under a watchdog (below)
        p = PRESETS[cfg]
        P_run, name, share = p["params"], PRESET_NAMES[cfg], None
        if cfg == 4 and world < SHARE_GPUS and not fits_one_share(ctx, world, p):
            # config 4 does not fit this many GPUs (one GPU: 359.8 GB of slab): run ONE GPU's share of the 8-GPU split
            # instead -- the largest bucket of sharding.bucket_ranges(350M, 8), all 256 clients -- labelled as the share
            from nvflare_amd.sharding import bucket_ranges

            lo, hi = max(bucket_ranges(p["params"], SHARE_GPUS), key=lambda b: b[1] - b[0])  # the slowest GPU's
            P_run, share = hi - lo, {"of_params_total": p["params"], "gpus": SHARE_GPUS, "bucket": [lo, hi]}
            name = (f"{PRESET_NAMES[cfg]} -- ONE GPU's share of the {SHARE_GPUS}-GPU split (the largest bucket of "
                    f"sharding.bucket_ranges({p['params']}, {SHARE_GPUS}): {p['clients']} clients x {P_run} params)")
        t_entry = time.perf_counter()
        r = run_workload(args, ctx, world, rank, p["clients"], P_run, "weak" if share else p["scaling"], p["epilogue"],
                         baseline=False, seed=args.seed, min_warmup_s=args.entry_warmup_s)
        failed = failed or bool((r.get("spot_check") or {}).get("mismatches"))
        if rank == 0:
            if "skipped" in r:
                also.append({"baseline_config": name, "n_gpus": world, "skipped": r["skipped"]})
            else:
                entry = summarize(args, world, r, p["clients"], "weak" if share else p["scaling"], p["epilogue"], name)
                entry["n_gpus"] = world
                entry["spot_check"] = r["spot_check"]
                if share:
                    entry["config"]["share"] = share
                if r.get("handout_pull"):
                    entry["handout_pull"] = r["handout_pull"]
                entry["gpu_state"] = r.get("gpu_state")
                entry["elapsed_s"] = round(time.perf_counter() - t_entry, 2)  # fill, warmup, steps, spot check
                also.append(entry)
    line = None
    if rank == 0:
        s = summarize(args, world, main_res, K, args.scaling, args.epilogue, label)
        line = {
            "metric": METRIC,
            "value": s["value"],
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": s["ms_per_step"],
            "higher_is_better": True,
            "scaling": s["scaling"],
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: device counter-hash generator (Irwin-Hall(4) ~N(0,1)), host twin in oracle/",
            "config": s["config"],
            "pct_hbm_peak": s["pct_hbm_peak"],
            "roofline": s["roofline"],
            "cpu_baseline": None,  # rank 0, after every GPU entry (below)
            "elapsed_s": round(main_s, 2),  # the main entry's wall time: fill, warmup, steps, spot check
            "gpu_state": {"before": state_before, "main_timed": main_res.get("gpu_state")},
        }
        if main_res.get("handout_pull"):
            line["handout_pull"] = main_res["handout_pull"]
        if main_res.get("spot_check") is not None:
            line["spot_check"] = main_res["spot_check"]
    state, dog = {}, None
    for token in (HOST_RESIDENT, HOST_SHARDED, CLIENT_SHARDED):
        if token in args.also:
            if dog is not None:
                dog.cancel()
            e_failed, dog = guarded_entry(args, world, rank, local, line, also, state, token)
            failed = e_failed or failed
    if dog is not None:
        dog.cancel()
        dog = None
    # the CPU baseline on rank 0 at EVERY N, after all GPU entries so it perturbs none of them;
    # the other ranks sleep on the rendezvous store meanwhile (wait_for_rank0), not in a spinning collective
    if rank == 0 and not args.no_cpu_baseline:
        t_cpu = time.perf_counter()
        try:
            line["cpu_baseline"] = cpu_baseline(args, K, min(args.params, main_res["P"]), main_res["op"])
            line["cpu_baseline"]["elapsed_s"] = round(time.perf_counter() - t_cpu, 2)
            line["cpu_baseline"]["n_gpus_in_run"] = world
        except Exception as e:  # noqa: BLE001 -- recorded; the GPU measurements stand
            line["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
    wait_for_rank0(world, rank, "nvflare_amd_bench_cpu_baseline_done")
    if rank == 0:
        line["gpu_state"]["after"] = gpu_snapshot(args)
        if also:
            line["also"] = also
        state["printed"] = True
        print(json.dumps(line), flush=True)
        if failed:
            print("SPOT CHECK FAILED", file=sys.stderr)
    if world > 1:
        import threading

        import torch.distributed as dist

        # the teardown under a watchdog as well: the line is out; a stuck barrier must not hold the run
        dog = threading.Timer(args.watchdog_s, lambda: (sys.stdout.flush(), sys.stderr.flush(), os._exit(3 if failed else 0)))
        dog.daemon = True
        dog.start()
        dist.barrier()
        dist.destroy_process_group()
    if dog is not None:
        dog.cancel()
    if failed:
        sys.exit(3)


if __name__ == "__main__":
    main()
