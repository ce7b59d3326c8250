"""Client-sharded ingest benchmark (nvflare_amd/client_shards.py): K clients dealt
round-robin to the ranks (client g on rank g mod N, as a server's ranks would split the connections), each
rank holding its clients' WHOLE updates of P = N x params_per_gpu fp32 values; per-GPU memory and bucket size
stay fixed as N grows (at N = 8 the defaults are config 4: 256 clients x 350 M).

Two strategies, each timed with barrier + synchronize brackets (max over ranks) and torch events on the stream
both the collectives and the kernels run on:
  exchange -- all-to-all (bucket b of every client to rank b), then the arrival-ordered kernel over all K
              clients on the bucket: bit-exact (sampled outputs checked against the oracle);
  reduce   -- per-rank partial over the local clients, reduce-scatter of the partials, finalise: NOT
              bit-exact (sampled outputs checked against the fp64 summation bound, differing bits counted).

  python tools/bench_client_shards.py                               # N = 1 (the exchange is a self copy)
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_client_shards.py
Prints one JSON line (rank 0).  Oracle use is the spot check only (test infrastructure).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_PEAK_GBS = 8000.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=256)
    ap.add_argument("--params-per-gpu", type=float, default=43.75e6)
    ap.add_argument("--mode", choices=["torch", "numpy"], default="torch")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--spot-check", type=int, default=2048)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--max-peer-mib", type=int, default=0, help="all-to-all chunk per peer (0 = library default)")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    shared = os.environ.get("NVFLARE_AMD_BENCH_SHARED_DEVICE") == "1"
    if "WORLD_SIZE" not in os.environ:
        os.environ.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(_free_port()))
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    local = 0 if shared else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if shared:  # one-GPU rehearsal of the multi-rank flow (gloo, host-copied collectives): never a measurement
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from nvflare_amd.client_shards import ClientShardedFedAvg

    K = a.clients
    P = int(a.params_per_gpu) * world
    clients = [len(range(s, K, world)) for s in range(world)]
    order = [(g % world, g // world) for g in range(K)]  # arrival order = global client id
    weights = [1.0 * float(1 + (37 * g) % 100) for g in range(K)]
    agg = ClientShardedFedAvg(P, clients, device=local, mode=a.mode)
    agg.fill_synthetic(a.seed, [j * world + rank for j in range(clients[rank])])
    if a.max_peer_mib:
        agg.max_peer_bytes = a.max_peer_mib << 20
    b0, b1 = agg.plan.buckets[rank]
    nb = b1 - b0
    stream = torch.cuda.current_stream()

    def sync():
        torch.cuda.synchronize()
        dist.barrier()

    def tmax(x):
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if shared else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for _ in range(a.warmup):
        agg.aggregate(order, weights, "exchange")
        agg.aggregate(order, weights, "reduce")
    sync()

    # exchange strategy: all-to-all, then the kernel
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e in ev:
        e[0].record(stream)
        agg.exchange()
        e[1].record(stream)
        agg.aggregate_exchanged(order, weights)
        e[2].record(stream)
    sync()
    wall_x = tmax(time.perf_counter() - t0) / a.steps
    a2a_ms = tmax(sum(e[0].elapsed_time(e[1]) for e in ev) / a.steps)
    agg_ms = tmax(sum(e[1].elapsed_time(e[2]) for e in ev) / a.steps)
    exact = agg.out[:nb].clone()

    # exchange strategy, overlapped: the chunked all-to-all on one stream, the kernels over the tiles received so
    # far on another (ClientShardedFedAvg.aggregate -> _exchange_overlapped)
    evo = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e in evo:
        e[0].record(stream)
        agg.aggregate(order, weights, "exchange")
        e[1].record(stream)
    sync()
    wall_o = tmax(time.perf_counter() - t0) / a.steps
    ovl_ms = tmax(sum(e[0].elapsed_time(e[1]) for e in evo) / a.steps)
    same_o = int(not torch.equal(agg.out[:nb].view(torch.int32), exact.view(torch.int32)))
    same_o = int(tmax(float(same_o)))

    # reduce strategy
    evr = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e in evr:
        e[0].record(stream)
        agg.aggregate(order, weights, "reduce")
        e[1].record(stream)
    sync()
    wall_r = tmax(time.perf_counter() - t0) / a.steps
    red_ms = tmax(sum(e[0].elapsed_time(e[1]) for e in evr) / a.steps)
    reduced = agg.out[:nb].clone()

    # spot check (oracle = test infrastructure): sampled bucket columns of this rank
    from oracle import fedavg_oracle as orc

    rng = np.random.default_rng(rank + 17)
    m = min(a.spot_check, nb)
    idx = np.unique(np.concatenate([rng.integers(0, nb, m), [0, nb - 1]])) if nb else np.zeros(0, np.int64)
    cols = (b0 + idx).astype(np.uint64)
    rows = [orc.synth_values(a.seed, g, cols) for g in range(K)]
    want = orc.fedavg_c(rows, weights, orc.MODE_TORCH if a.mode == "torch" else orc.MODE_NUMPY)
    sel = torch.from_numpy(idx).to(exact.device)
    got_x = exact[sel].cpu().numpy()
    got_r = reduced[sel].cpu().numpy()
    mism = int(np.count_nonzero(got_x.view(np.uint32) != want.view(np.uint32)))
    w64 = np.asarray(weights)[:, None]
    v64 = np.stack(rows).astype(np.float64)
    cnt = 0.0
    for i, w in enumerate(weights):
        cnt = w if i == 0 else cnt + w
    ref = (w64 * v64).sum(axis=0) / cnt
    bound = (K + 2) * 2.0 ** -24 * np.abs(w64 * v64).sum(axis=0) / cnt + np.spacing(np.abs(ref).astype(np.float32))
    ratio = float(np.max(np.abs(got_r - ref) / bound)) if idx.size else 0.0
    differ = int(np.count_nonzero(got_r.view(np.uint32) != want.view(np.uint32)))
    t = torch.tensor([idx.size, mism, differ], dtype=torch.int64, device="cpu" if shared else "cuda")
    dist.all_reduce(t)
    ratio = tmax(ratio)

    if rank == 0:
        elems = 4.0 * K * P
        kern_bytes = 4.0 * K * nb + 4.0 * nb
        a2a_bytes = 4.0 * (sum(agg.plan.send_splits(rank)) - agg.plan.send_splits(rank)[rank])
        line = {
            "metric": "GiB/s aggregated, client-sharded ingest (K clients x P fp32 params over N ranks)",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "unit": "GiB/s", "higher_is_better": True,
            "scaling": "weak", "dtype": "f32", "shared_device_rehearsal": shared,
            "config": {"clients": K, "params_total": P, "params_per_gpu": int(a.params_per_gpu), "mode": a.mode,
                       "placement": "client g on rank g mod N", "clients_per_rank": clients},
            "exchange": {
                "value": round(elems / wall_x / 2**30, 2), "ms_per_step": round(wall_x * 1e3, 3),
                "all_to_all_ms": round(a2a_ms, 3), "kernel_ms": round(agg_ms, 3),
                "all_to_all_bytes_out_per_rank": a2a_bytes,
                "all_to_all_GBps_per_rank": round(a2a_bytes / (a2a_ms / 1e3) / 1e9, 1) if world > 1 else None,
                "kernel_roofline_frac": round(kern_bytes / (agg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "spot_check": {"sampled": int(t[0]), "mismatches": int(t[1]), "oracle": "oracle/fedavg_oracle.c"},
            },
            "exchange_overlapped": {
                "value": round(elems / wall_o / 2**30, 2), "ms_per_step": round(wall_o * 1e3, 3),
                "device_ms": round(ovl_ms, 3),
                "serial_device_ms": round(a2a_ms + agg_ms, 3),
                "hidden_kernel_ms": round(a2a_ms + agg_ms - ovl_ms, 3),
                "bits_equal_serial": same_o == 0,
                "min_kernel_tiles": agg.min_kernel_tiles, "max_peer_bytes": agg.max_peer_bytes,
            },
            "reduce": {
                "value": round(elems / wall_r / 2**30, 2), "ms_per_step": round(wall_r * 1e3, 3),
                "device_ms": round(red_ms, 3),
                "bit_exact": False,
                "differing_from_exact_sampled": int(t[2]),
                "max_err_over_fp64_bound": round(ratio, 4),
            },
        }
        print(json.dumps(line), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if int(t[1]) or same_o:
        sys.exit(3)


if __name__ == "__main__":
    main()
