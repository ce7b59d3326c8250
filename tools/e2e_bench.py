#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the drop-in: client updates arrive in HOST memory, go through
InTimeAccumulateWeightedAggregator.accept (H2D staging into the tiled slab) and aggregate() (kernel +
D2H of the global model) -- DESIGN.md section 4, "PCIe-inclusive rate".  Not the bench's `value`.

  python tools/e2e_bench.py [--clients 8 --params 125e6 --container numpy|torch|pinned --keys 1|437]
                            [--quant none|float16|blockwise8|normfloat4 [--eager]]

--quant: clients send quantized payloads (row f4) -- ModelDequantizer(lazy=True) values that the engine
dequantizes into the slab slot after moving only the compressed bytes; --eager dequantizes on the device
and returns them to the host first (the reference filter's behaviour), then stages fp32.
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
    ap.add_argument("--quant", choices=["none", "float16", "blockwise8", "normfloat4"], default="none")
    ap.add_argument("--eager", action="store_true")
    args = ap.parse_args()
    import torch

    from nvflare_amd.app_common.aggregators.weighted_aggregation_helper import WeightedAggregationHelper

    K, P = args.clients, int(args.params)
    rng = np.random.default_rng(0)
    sizes = np.full(args.keys, P // args.keys)
    sizes[-1] += P - sizes.sum()
    base = rng.standard_normal(P, dtype=np.float32)
    clients = []
    if args.quant != "none":
        from nvflare_amd import _native as N
        from nvflare_amd.quantized import QuantizedPayload

        def quantized(n, seed):
            g = np.random.default_rng(seed)
            if args.quant == "float16":
                return QuantizedPayload(N.FEDAVG_Q_F16, g.standard_normal(n).astype(np.float16).view(np.uint16),
                                        (n,), "numpy")
            if args.quant == "blockwise8":
                return QuantizedPayload(N.FEDAVG_Q_BLOCKWISE8, g.integers(0, 256, n, dtype=np.uint8), (n,), "numpy",
                                        absmax=g.random((n + 4095) // 4096, dtype=np.float32),
                                        code=np.linspace(-1, 1, 256, dtype=np.float32), blocksize=4096)
            return QuantizedPayload(N.FEDAVG_Q_NF4, g.integers(0, 256, (n + 1) // 2, dtype=np.uint8), (n,), "numpy",
                                    absmax=g.random((n + 63) // 64, dtype=np.float32), blocksize=64)

        for k in range(K):
            clients.append({f"layer{j}.weight": quantized(int(n), 1000 * k + j) for j, n in enumerate(sizes)})
    for k in range(K if args.quant == "none" else 0):
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
            c = clients[k]
            if args.quant != "none" and args.eager:
                c = {key: v.materialize() for key, v in c.items()}
            h.add(c, ws[k], f"site-{k}", r)
            t_acc.append(time.perf_counter() - a0)
        t1 = time.perf_counter()
        out = h.get_result()
        t2 = time.perf_counter()
        nbytes = 4.0 * K * P
        wire = sum(v.nbytes for c in clients for v in c.values())
        res.append({"round": r, "accept_s": round(t1 - t0, 4), "aggregate_s": round(t2 - t1, 4),
                    "h2d_GBps": round(wire / (t1 - t0) / 1e9, 2), "host_bytes_per_client": wire // K,
                    "e2e_GiBps_aggregated": round(nbytes / (t2 - t0) / 2**30, 2),
                    "accept_first_s": round(t_acc[0], 4), "accept_last_s": round(t_acc[-1], 4)})
        print(json.dumps(res[-1]), flush=True)
        del out
    best = max(res[1:] or res, key=lambda x: x["e2e_GiBps_aggregated"])
    print(json.dumps({"summary": "e2e (host arrays in, host result out)", "clients": K, "params": P,
                      "keys": args.keys, "container": args.container, "devices": devices, "quant": args.quant,
                      "eager": args.eager, **best}))


if __name__ == "__main__":
    main()
