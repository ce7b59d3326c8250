#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the drop-in: client updates arrive in HOST memory, go through
InTimeAccumulateWeightedAggregator.accept (H2D staging into the tiled slab) and aggregate() (kernel +
D2H of the global model) -- DESIGN.md section 4, "PCIe-inclusive rate".  Not the bench's `value`.

  python tools/e2e_bench.py [--clients 8 --params 125e6 --container numpy|torch|pinned --keys 1|437]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=float, default=125e6)
    ap.add_argument("--container", choices=["numpy", "torch", "pinned"], default="numpy")
    ap.add_argument("--keys", type=int, default=1, help="split the model into this many tensors (437 ~ GPT-2 large)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--devices", default="0")
    args = ap.parse_args()
    import torch

    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    K, P = args.clients, int(args.params)
    rng = np.random.default_rng(0)
    sizes = np.full(args.keys, P // args.keys)
    sizes[-1] += P - sizes.sum()
    base = rng.standard_normal(P, dtype=np.float32)
    clients = []
    for k in range(K):
        flat = base * np.float32(1.0 + 0.01 * k)
        parts, off = {}, 0
        for j, n in enumerate(sizes):
            a = flat[off: off + n]
            if args.container == "torch":
                a = torch.from_numpy(a)
            elif args.container == "pinned":
                a = torch.from_numpy(a).pin_memory()
            parts[f"layer{j}.weight"] = a
            off += n
        clients.append(parts)
    devices = [int(d) for d in args.devices.split(",")]
    h = WeightedAggregationHelper(devices=devices)
    ws = [float(1 + (37 * k) % 100) for k in range(K)]
    res = []
    for r in range(args.rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t_acc = []
        for k in range(K):
            a0 = time.perf_counter()
            h.add(clients[k], ws[k], f"site-{k}", r)
            t_acc.append(time.perf_counter() - a0)
        t1 = time.perf_counter()
        out = h.get_result()
        t2 = time.perf_counter()
        nbytes = 4.0 * K * P
        res.append({"round": r, "accept_s": round(t1 - t0, 4), "aggregate_s": round(t2 - t1, 4),
                    "h2d_GBps": round(nbytes / (t1 - t0) / 1e9, 2),
                    "e2e_GiBps_aggregated": round(nbytes / (t2 - t0) / 2**30, 2),
                    "accept_first_s": round(t_acc[0], 4), "accept_last_s": round(t_acc[-1], 4)})
        print(json.dumps(res[-1]), flush=True)
        del out
    best = max(res[1:] or res, key=lambda x: x["e2e_GiBps_aggregated"])
    print(json.dumps({"summary": "e2e (host arrays in, host result out)", "clients": K, "params": P,
                      "keys": args.keys, "container": args.container, "devices": devices, **best}))


if __name__ == "__main__":
    main()
